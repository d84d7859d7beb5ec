// controller_gpu_hook.go - the seam between the reference's NewController
// (controller.go:80-152) and the MI355X engine: nil in a default build, set by
// controller_mi355x.go in a `-tags kwok_mi355x` build.

package controllers

import "context"

type starter interface {
	Start(ctx context.Context) error
}

var gpuController func(conf Config) (starter, error)
