//go:build kwok_mi355x

// controller_mi355x.go - with -tags kwok_mi355x, NewController (controller.go,
// patched as in ../../../../README.md) builds the engine-backed controller: the
// same Config, the same Start, the reference's 30 s heartbeat interval.

package controllers

import "time"

func init() {
	gpuController = func(conf Config) (starter, error) {
		return newGPUController(conf, 30*time.Second)
	}
}
