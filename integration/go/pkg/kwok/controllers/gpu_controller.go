//go:build kwok_mi355x

// gpu_controller.go - the client-go side of the drop-in: watch events are
// batched, encoded as object JSON, decoded by the engine's host codec and
// ingested before each tick; every body the tick returns is applied through the
// clientset with the reference's 16-wide task pools (utils.go:119-161).  The
// watch echoes of the engine's own patches are dropped by resourceVersion
// (echoes).  kwok_amd/controller.py is the same controller in Python, which
// the tests run against a fake clientset (tests/test_controller*.py).
// NewController builds this in place of NodeController + PodController when
// the package is built with -tags kwok_mi355x (controller_mi355x.go).
//
// Not compiled in this repository (no Go toolchain in the image).

package controllers

/*
#include "kwok_engine.h"
*/
import "C"

import (
	"bytes"
	"context"
	"encoding/binary"
	"encoding/json"
	"fmt"
	"net"
	"os"
	"runtime"
	"sync"
	"time"

	corev1 "k8s.io/api/core/v1"
	apierrors "k8s.io/apimachinery/pkg/api/errors"
	metav1 "k8s.io/apimachinery/pkg/apis/meta/v1"
	"k8s.io/apimachinery/pkg/types"
	"k8s.io/apimachinery/pkg/watch"

	"sigs.k8s.io/kwok/pkg/cni"
	"sigs.k8s.io/kwok/pkg/log"
)

// watchObj: one watch event since the last tick.  The object is encoded to
// JSON only at the next tick, after the echoes of the engine's own patches are
// dropped (echoes).
type watchObj struct {
	obj     interface{}
	uid     types.UID
	rv      string // metadata.resourceVersion
	deleted bool
}

// objBatch: the watch objects of one tick as concatenated JSON (the codec's input)
type objBatch struct {
	arena []byte
	offs  []uint64
	lens  []uint32
	del   []bool
	uids  []types.UID
	refs  []types.NamespacedName // namespace / name (a pod's: the apply's target; a node's name)
	nodes []string               // pods: spec.nodeName (EnableCNI's cni.Remove check)
}

func (b *objBatch) add(w watchObj) error {
	raw, err := json.Marshal(w.obj)
	if err != nil {
		return err
	}
	b.offs = append(b.offs, uint64(len(b.arena)))
	b.lens = append(b.lens, uint32(len(raw)))
	b.arena = append(b.arena, raw...)
	b.del = append(b.del, w.deleted)
	b.uids = append(b.uids, w.uid)
	var ref types.NamespacedName // (one entry per object, so the indices stay aligned)
	var node string
	switch o := w.obj.(type) {
	case *corev1.Pod:
		ref, node = types.NamespacedName{Namespace: o.Namespace, Name: o.Name}, o.Spec.NodeName
	case *corev1.Node:
		ref = types.NamespacedName{Name: o.Name}
	}
	b.refs = append(b.refs, ref)
	b.nodes = append(b.nodes, node)
	return nil
}

// echoes: the resourceVersions the engine's own patches returned, per object.
// Their Modified watch events (the echoes) are states the engine already
// assumed when it emitted the patches (DESIGN.md §1: patches are assumed
// applied; a heartbeat's echo re-lock, node_controller.go:152 -> :256-263, is
// part of every tick), so echoes are dropped instead of re-ingested.  An object
// can take several patches in one tick (a node's heartbeat and its init patch,
// a pod's finalizer patch), each with its own echo: every returned version is
// kept until its echo is seen (the last echoKeep per object, so echoes lost to a
// watch restart do not pile up).  Any other event of the object is ingested.
type echoes struct {
	mu sync.Mutex
	rv map[types.UID][]string
}

const echoKeep = 8

func (x *echoes) note(uid types.UID, rv string) {
	if uid == "" || rv == "" {
		return
	}
	x.mu.Lock()
	v := append(x.rv[uid], rv)
	if len(v) > echoKeep {
		v = v[1:]
	}
	x.rv[uid] = v
	x.mu.Unlock()
}

// is: the event is the echo of one of the engine's patches of the object (each
// echo is consumed: a second event with that resourceVersion is not expected)
func (x *echoes) is(uid types.UID, rv string) bool {
	x.mu.Lock()
	defer x.mu.Unlock()
	v := x.rv[uid]
	for i, r := range v {
		if r == rv {
			v = append(v[:i], v[i+1:]...)
			if len(v) == 0 {
				delete(x.rv, uid)
			} else {
				x.rv[uid] = v
			}
			return true
		}
	}
	return false
}

func (x *echoes) forget(uid types.UID) {
	x.mu.Lock()
	delete(x.rv, uid)
	x.mu.Unlock()
}

// encode drops the echoes among ws (those whose patch returned after the watch
// event arrived: onEvent could not match them yet) and encodes the rest
func (x *echoes) encode(ws []watchObj) (objBatch, int, error) {
	var b objBatch
	dropped := 0
	seen := map[types.UID]struct{}{} // (the rule of onEvent: only before any kept event of the object)
	for _, w := range ws {
		_, after := seen[w.uid]
		if !w.deleted && x.is(w.uid, w.rv) && !after {
			dropped++
			continue
		}
		seen[w.uid] = struct{}{}
		if err := b.add(w); err != nil {
			return b, dropped, err
		}
		if w.deleted { // the object's last event: echoes still noted for it will not come
			x.forget(w.uid)
		}
	}
	return b, dropped, nil
}

// GPUController: one engine (one GPU) behind the reference's Controller API.
type GPUController struct {
	conf      Config
	eng       *gpuEngine
	codec     *gpuCodec
	interval  time.Duration
	finalizer []byte

	mu    sync.Mutex // guards the batches (watch goroutines append, the tick loop swaps)
	nodes  []watchObj
	pods   []watchObj
	queued map[types.UID]struct{} // objects with an event in the batches
	echo   echoes

	// tick loop only
	nodeName   map[int32]string // node handle -> name
	nodeHandle map[string]int32 // name -> node handle (nodes the engine holds; pods name them by handle)
	podByUID   map[types.UID]int32
	podUID   map[int32]types.UID // pod handle -> UID (the reverse of podByUID)
	podRef   map[int32]types.NamespacedName

	gpuCodec    bool // pod documents decoded on the GPU (kwok_ingest_pods_json); KWOK_GPU_CODEC=0: the host codec
	podDocsHost int  // pod documents the GPU codec left to the host codec (logged)
	nodeDocsHost int // node documents the GPU codec left to the host codec (logged)
}

func newGPUController(conf Config, interval time.Duration) (*GPUController, error) {
	st, err := time.Parse(time.RFC3339, startTime) // the StartTime() value (controller.go:33)
	if err != nil {
		return nil, err
	}
	eng, err := newGPUEngine(conf, st.Unix(), 0, 1, nil)
	if err != nil {
		return nil, err
	}
	codec, err := newGPUCodec(conf)
	if err != nil {
		eng.close()
		return nil, err
	}
	return &GPUController{
		conf: conf, eng: eng, codec: codec, interval: interval, finalizer: finalizerPatch(),
		nodeName: map[int32]string{}, nodeHandle: map[string]int32{}, podByUID: map[types.UID]int32{},
		podUID: map[int32]types.UID{},
		podRef: map[int32]types.NamespacedName{},
		echo:     echoes{rv: map[types.UID][]string{}},
		queued:   map[types.UID]struct{}{},
		gpuCodec: os.Getenv("KWOK_GPU_CODEC") != "0",
	}, nil
}

// Start: the node and pod watches of NodeController.Start / PodController.Start
// (node_controller.go:119-143, pod_controller.go:130-153) feed the batches; the
// tick loop replaces KeepNodeHeartbeat, LockNodes, LockPods and DeletePods.
func (c *GPUController) Start(ctx context.Context) error {
	nodeOpt := metav1.ListOptions{LabelSelector: c.conf.ManageNodesWithLabelSelector}
	podOpt := metav1.ListOptions{FieldSelector: podFieldSelector}
	if err := c.watch(ctx, true, nodeOpt); err != nil {
		return fmt.Errorf("failed to watch nodes: %w", err)
	}
	if err := c.watch(ctx, false, podOpt); err != nil {
		return fmt.Errorf("failed to watch pods: %w", err)
	}
	go c.loop(ctx)
	return nil
}

// watch from the current state (a watch without resourceVersion first sends an
// Added event per existing object, as ListNodes / ListPods would), re-opened
// when the server closes it, like WatchNodes / WatchPods
func (c *GPUController) watch(ctx context.Context, nodes bool, opt metav1.ListOptions) error {
	open := func() (watch.Interface, error) {
		if nodes {
			return c.conf.ClientSet.CoreV1().Nodes().Watch(ctx, opt)
		}
		return c.conf.ClientSet.CoreV1().Pods(corev1.NamespaceAll).Watch(ctx, opt)
	}
	w, err := open()
	if err != nil {
		return err
	}
	logger := log.FromContext(ctx)
	go func() {
		rc := w.ResultChan()
		for {
			select {
			case <-ctx.Done():
				w.Stop()
				return
			case ev, ok := <-rc:
				if !ok {
					for {
						if w, err = open(); err == nil {
							rc = w.ResultChan()
							break
						}
						logger.Error("Failed to re-watch", err)
						select {
						case <-ctx.Done():
							return
						case <-time.After(time.Second * 5):
						}
					}
					continue
				}
				c.onEvent(ctx, nodes, ev)
			}
		}
	}()
	return nil
}

func (c *GPUController) onEvent(ctx context.Context, nodes bool, ev watch.Event) {
	if ev.Type != watch.Added && ev.Type != watch.Modified && ev.Type != watch.Deleted {
		return
	}
	var w watchObj
	switch obj := ev.Object.(type) {
	case *corev1.Node:
		if !nodes {
			return
		}
		w = watchObj{obj, obj.UID, obj.ResourceVersion, ev.Type == watch.Deleted}
	case *corev1.Pod:
		if nodes {
			return
		}
		w = watchObj{obj, obj.UID, obj.ResourceVersion, ev.Type == watch.Deleted}
	default:
		return
	}
	c.mu.Lock()
	defer c.mu.Unlock()
	// the echo of one of the engine's own patches (its apply already returned):
	// not queued, not encoded - unless another event of the object waits in this
	// tick's batch: that one is a change the engine has not seen, older than the
	// patch, and the echo is the object's newest state, carrying both
	_, waiting := c.queued[w.uid]
	if ev.Type == watch.Modified && c.echo.is(w.uid, w.rv) && !waiting {
		return
	}
	c.queued[w.uid] = struct{}{}
	if nodes {
		c.nodes = append(c.nodes, w)
	} else {
		c.pods = append(c.pods, w)
	}
}

func (c *GPUController) loop(ctx context.Context) {
	logger := log.FromContext(ctx)
	tasks := newParallelTasks(16) // the reference's heartbeat / lock / delete parallelism
	t := time.NewTimer(c.interval)
	defer func() {
		t.Stop()
		tasks.Wait()
		c.codec.close()
		c.eng.close()
	}()
	for {
		select {
		case <-ctx.Done():
			return
		case <-t.C:
			start := time.Now()
			n, err := c.step(ctx, tasks, start.Unix())
			tasks.Wait()
			if err != nil {
				logger.Error("Failed to tick", err)
			}
			logger.Info("Tick", "bodies", n, "elapsed", time.Since(start))
			t.Reset(c.interval)
		}
	}
}

// Has / Size: NodeController.Has / Size (node_controller.go:403-409) of the
// engine's managed-node set
func (c *GPUController) Has(nodeName string) bool { return c.eng.nodeHas(nodeName) }
func (c *GPUController) Size() int               { return c.eng.nodeSize() }

// step: ingest the batches (nodes first, so new pods find their node), give
// the tick's pending pods their CNI IPs (EnableCNI), run the tick, hand every
// body to the task pool; then the same interval again for the pods patched
// without a podIP (created with an empty status: pod.status.tpl renders no IPs
// then, `{{ with .status }}`).  In the reference that patch's own Modified event
// re-enters lockPodChan (pod_controller.go:279-319) and the pod gets hostIP /
// podIP at once; here the object the patch returned is ingested as that event
// (its watch echo is dropped like every echo) and the engine ticks again at the
// same clock, applying that tick's pod patches, node inits and deletes but not
// its heartbeats (the interval's heartbeats were sent).
func (c *GPUController) step(ctx context.Context, tasks *parallelTasks, now int64) (int, error) {
	c.mu.Lock()
	nw, pw := c.nodes, c.pods
	c.nodes, c.pods, c.queued = nil, nil, map[types.UID]struct{}{}
	c.mu.Unlock()
	// every apply of the previous tick has returned (loop waits for the task pool):
	// the echoes that overtook their patch's response are dropped here
	nb, _, err := c.echo.encode(nw)
	if err != nil {
		return 0, err
	}
	pb, _, err := c.echo.encode(pw)
	if err != nil {
		return 0, err
	}
	if err := c.flushNodes(ctx, nb); err != nil {
		return 0, err
	}
	if err := c.flushPods(ctx, tasks, pb); err != nil {
		return 0, err
	}
	if c.conf.EnableCNI {
		if err := c.setupCNI(ctx, tasks); err != nil {
			return 0, err
		}
	}
	var re reentry
	n, err := c.tickApply(ctx, tasks, now, true, &re)
	for round := 0; round < 4 && err == nil; round++ { // (a re-entered pod's second patch carries its IPs)
		tasks.Wait()
		if len(re.objs) == 0 {
			break
		}
		var b objBatch
		for _, p := range re.objs {
			if err = b.add(watchObj{p, p.UID, p.ResourceVersion, false}); err != nil {
				return n, err
			}
		}
		re.objs = nil
		if err = c.flushPods(ctx, tasks, b); err != nil {
			return n, err
		}
		if c.conf.EnableCNI {
			if err = c.setupCNI(ctx, tasks); err != nil {
				return n, err
			}
		}
		var m int
		m, err = c.tickApply(ctx, tasks, now, false, &re)
		n += m
	}
	return n, err
}

// reentry: the objects returned by pod patches that carried no podIP
type reentry struct {
	mu   sync.Mutex
	objs []*corev1.Pod
}

var podIPKey = []byte(`"podIP"`)

// tickApply: one tick at now, every body handed to the task pool (heartbeats
// only when asked); pod patches without a podIP leave their returned object in re
func (c *GPUController) tickApply(ctx context.Context, tasks *parallelTasks, now int64, heartbeats bool,
	re *reentry) (int, error) {
	logger := log.FromContext(ctx)
	nodesAPI := c.conf.ClientSet.CoreV1().Nodes()
	var gone []int32
	n := 0
	err := c.eng.tick(now, func(kind int, h int32, body []byte) {
		if kind == kindHeartbeat && !heartbeats {
			return
		}
		n++
		switch kind {
		case kindHeartbeat, kindNodeInit: // configureHeartbeatNode / configureNode bodies
			name := c.nodeName[h]
			tasks.Add(func() {
				n, err := nodesAPI.PatchStatus(ctx, name, body)
				if err != nil {
					logger.Error("Failed to patch node status", err, "node", name)
					return
				}
				c.echo.note(n.UID, n.ResourceVersion)
			})
		case kindPodPatch: // LockPod (pod_controller.go:205-231)
			ref := c.podRef[h]
			tasks.Add(func() {
				p, err := c.conf.ClientSet.CoreV1().Pods(ref.Namespace).Patch(ctx, ref.Name,
					types.StrategicMergePatchType, body, metav1.PatchOptions{}, "status")
				if err != nil {
					if !apierrors.IsNotFound(err) {
						logger.Error("Failed to lock pod", err, "pod", ref.String())
					}
					return
				}
				c.echo.note(p.UID, p.ResourceVersion)
				if !bytes.Contains(body, podIPKey) { // an empty status: its echo re-enters
					re.mu.Lock()
					re.objs = append(re.objs, p)
					re.mu.Unlock()
				}
			})
		case kindDelete, kindDeleteFin: // DeletePod (pod_controller.go:155-183); the engine freed the handle
			ref, fin := c.podRef[h], kind == kindDeleteFin
			gone = append(gone, h)
			// the pod's noted echoes go here, before the task: the echo its finalizer
			// patch notes (whenever the task runs) is then dropped, not re-ingested
			c.echo.forget(c.podUID[h])
			tasks.Add(func() {
				pods := c.conf.ClientSet.CoreV1().Pods(ref.Namespace)
				if fin { // only pods with finalizers (len(pod.Finalizers) != 0, :161)
					p, err := pods.Patch(ctx, ref.Name, types.MergePatchType, c.finalizer, metav1.PatchOptions{})
					if err != nil {
						if !apierrors.IsNotFound(err) {
							logger.Error("Failed to patch pod finalizers", err, "pod", ref.String())
						}
						return
					}
					// its echo (deletionTimestamp, no finalizers) would re-enter DeletePod
					// for a pod the engine already deleted
					c.echo.note(p.UID, p.ResourceVersion)
				}
				if err := pods.Delete(ctx, ref.Name, deleteOpt); err != nil && !apierrors.IsNotFound(err) {
					logger.Error("Failed to delete pod", err, "pod", ref.String())
				}
			})
		}
	})
	for _, h := range gone { // the later Deleted watch event finds no handle (CNI: it still runs cni.Remove)
		delete(c.podByUID, c.podUID[h])
		delete(c.podUID, h)
		delete(c.podRef, h)
	}
	return n, err
}

// setupCNI: configurePod's cni.Setup for the pods the next tick evaluates that
// hold no podIP (pod_controller.go:383-389), 16 at a time; the engine patches
// them with the first returned IP.  A failed Setup leaves the pod unpatched
// this tick, as configurePod's error does.
func (c *GPUController) setupCNI(ctx context.Context, tasks *parallelTasks) error {
	hs, err := c.eng.cniPending()
	if err != nil || len(hs) == 0 {
		return err
	}
	logger := log.FromContext(ctx)
	ips := make([]uint32, len(hs))
	for i, h := range hs {
		i, uid, ref := i, c.podUID[h], c.podRef[h]
		tasks.Add(func() {
			got, err := cni.Setup(ctx, string(uid), ref.Name, ref.Namespace)
			if err != nil {
				logger.Error("cni setup", err, "pod", ref.String())
				return
			}
			if ip := net.ParseIP(got[0]).To4(); ip != nil {
				ips[i] = binary.BigEndian.Uint32(ip)
			}
		})
	}
	tasks.Wait()
	keep, kept := hs[:0], ips[:0]
	for i := range hs {
		if ips[i] != 0 {
			keep, kept = append(keep, hs[i]), append(kept, ips[i])
		}
	}
	return c.eng.cniAssign(keep, kept)
}

// flushNodes: the batch's node documents decoded on the GPU (kwok_ingest_nodes_json:
// a Deleted event's status is not read; a non-empty addresses / allocatable /
// capacity blob goes to the host codec inside the call) and routed by the GPU
// event switch; flushNodesHost decodes on the host (KWOK_GPU_CODEC=0).
// kwok_amd/controller.py _flush_nodes_gpu is this function in Python.
func (c *GPUController) flushNodes(ctx context.Context, b objBatch) error {
	if len(b.offs) == 0 {
		return nil
	}
	if !c.gpuCodec {
		return c.flushNodesHost(ctx, b)
	}
	logger := log.FromContext(ctx)
	ops := make([]uint8, len(b.offs))
	for i := range ops {
		ops[i] = C.KWOK_OP_UPSERT
		if b.del[i] {
			ops[i] = C.KWOK_OP_DELETE
		}
	}
	hs, ss, nHost, err := c.eng.ingestNodesJSON(c.codec, b.arena, b.offs, b.lens, ops)
	if err != nil {
		return err
	}
	c.nodeDocsHost += nHost
	for i := range ops {
		if ss[i] != C.KWOK_OK {
			if ss[i] == C.KWOK_EDOMAIN || ss[i] == C.KWOK_EINVAL { // outside the engine's domain (DESIGN.md §2)
				logger.Warn("Node outside the supported domain", fmt.Errorf("kwok status %d", ss[i]))
			}
			continue
		}
		name := b.refs[i].Name
		if b.del[i] {
			delete(c.nodeName, hs[i])
			delete(c.nodeHandle, name)
		} else {
			c.nodeName[hs[i]] = name
			c.nodeHandle[name] = hs[i]
		}
	}
	return nil
}

// flushNodesHost: flushNodes with the host codec (kwok_decode_nodes)
func (c *GPUController) flushNodesHost(ctx context.Context, b objBatch) error {
	logger := log.FromContext(ctx)
	ev, st := c.codec.decodeNodes(b.arena, b.offs, b.lens, runtime.NumCPU())
	keep := make([]C.kwok_node_event, 0, len(ev))
	names := make([]string, 0, len(ev))
	for i := range ev {
		if st[i] != C.KWOK_OK { // outside the engine's domain: not simulated (DESIGN.md §2)
			logger.Warn("Node outside the supported domain", fmt.Errorf("kwok status %d", st[i]))
			continue
		}
		ev[i].op = C.KWOK_OP_UPSERT
		if b.del[i] {
			ev[i].op = C.KWOK_OP_DELETE
		}
		keep = append(keep, ev[i])
		names = append(names, str(b.arena, ev[i].name))
	}
	hs, ss, err := c.eng.ingestNodes(keep, b.arena)
	if err != nil {
		return err
	}
	for i := range keep {
		if ss[i] != C.KWOK_OK {
			continue
		}
		if keep[i].op == C.KWOK_OP_DELETE {
			delete(c.nodeName, hs[i])
			delete(c.nodeHandle, names[i])
		} else {
			c.nodeName[hs[i]] = names[i]
			c.nodeHandle[names[i]] = hs[i]
		}
	}
	return nil
}

// flushPods ingests the batch in event order.  A pod's first event in the
// batch may create it (handle -1); its later events need that handle, so the
// batch is cut into runs in which no new pod appears twice: run k+1 is
// ingested after run k, once run k's handles are known.  (Added then Modified,
// or Added then Deleted, within one interval: one slot, then its update or its
// Deleted event with the pod's podIP release, pod_controller.go:329-336.)
// flushPods: the batch's pod documents decoded on the GPU (kwok_ingest_pods_json)
// in runs in which no new pod appears twice - a pod's first event may create it
// and its later events need that handle (Added + Modified, Added + Deleted in one
// interval) - the same runs as flushPodsHost, which decodes on the host
// (kwok_decode_pods) and is kept for engines built without the device codec
// (kwok_amd/controller.py ingest_doc_runs is this function in Python)
func (c *GPUController) flushPods(ctx context.Context, tasks *parallelTasks, b objBatch) error {
	if len(b.offs) == 0 {
		return nil
	}
	if !c.gpuCodec {
		return c.flushPodsHost(ctx, tasks, b)
	}
	logger := log.FromContext(ctx)
	var run []int
	created := map[types.UID]bool{} // new pods of the current run
	flush := func() error {
		offs, lens := make([]uint64, 0, len(run)), make([]uint32, 0, len(run))
		ops, hs := make([]uint8, 0, len(run)), make([]int32, 0, len(run))
		keep := run[:0]
		for _, i := range run {
			h, known := c.podByUID[b.uids[i]]
			if b.del[i] {
				// EnableCNI: cni.Remove for a pod on a managed node (pod_controller.go:337-342),
				// also when the engine deleted it already (its handle is gone)
				if c.conf.EnableCNI && c.eng.nodeHas(b.nodes[i]) {
					uid, ref := b.uids[i], b.refs[i]
					tasks.Add(func() {
						if err := cni.Remove(context.Background(), string(uid), ref.Name, ref.Namespace); err != nil {
							logger.Error("cni remove", err)
						}
					})
				}
				if !known { // never ingested, or already deleted by the engine
					continue
				}
				ops = append(ops, C.KWOK_OP_DELETE) // releases status.podIP (pod_controller.go:329-336)
				hs = append(hs, h)
			} else {
				ops = append(ops, C.KWOK_OP_UPSERT)
				if !known {
					h = -1
				}
				hs = append(hs, h)
			}
			offs, lens = append(offs, b.offs[i]), append(lens, b.lens[i])
			keep = append(keep, i)
		}
		run = run[:0]
		for k := range created {
			delete(created, k)
		}
		out, ss, nHost, err := c.eng.ingestPodsJSON(c.codec, b.arena, offs, lens, ops, hs)
		if err != nil {
			return err
		}
		c.podDocsHost += nHost
		for k, i := range keep {
			if ss[k] != C.KWOK_OK {
				logger.Warn("Pod outside the supported domain", fmt.Errorf("kwok status %d", ss[k]))
				continue
			}
			uid := b.uids[i]
			if ops[k] == C.KWOK_OP_DELETE {
				delete(c.podByUID, uid)
				delete(c.podUID, out[k])
				delete(c.podRef, out[k])
			} else {
				c.podByUID[uid] = out[k]
				c.podUID[out[k]] = uid
				c.podRef[out[k]] = b.refs[i]
			}
		}
		return nil
	}
	for i := range b.offs {
		uid := b.uids[i]
		if created[uid] { // its handle comes from the run before
			if err := flush(); err != nil {
				return err
			}
		}
		if _, known := c.podByUID[uid]; !known && !b.del[i] {
			created[uid] = true
		}
		run = append(run, i)
	}
	return flush()
}

// flushPodsHost: flushPods with the host codec (kwok_decode_pods) and the packed
// wire forms (ingestPods)
func (c *GPUController) flushPodsHost(ctx context.Context, tasks *parallelTasks, b objBatch) error {
	logger := log.FromContext(ctx)
	docs, st := c.codec.decodePods(b.arena, b.offs, b.lens, runtime.NumCPU())
	type rec struct {
		i   int // index in the batch
		ref types.NamespacedName
	}
	var run []rec
	created := map[types.UID]bool{} // new pods of the current run
	flush := func() error {
		evs := make([]C.kwok_pod_event, 0, len(run))
		keep := run[:0]
		for _, r := range run {
			d := &docs[r.i]
			h, known := c.podByUID[b.uids[r.i]]
			if b.del[r.i] {
				// EnableCNI: cni.Remove for a pod on a managed node (pod_controller.go:337-342),
				// also when the engine deleted it already (its handle is gone)
				if c.conf.EnableCNI && c.eng.nodeHas(str(b.arena, d.ev.node_name)) {
					uid, ref := b.uids[r.i], r.ref
					tasks.Add(func() {
						if err := cni.Remove(context.Background(), string(uid), ref.Name, ref.Namespace); err != nil {
							logger.Error("cni remove", err)
						}
					})
				}
				if !known { // never ingested, or already deleted by the engine
					continue
				}
				d.ev.op = C.KWOK_OP_DELETE // releases status.podIP (pod_controller.go:329-336)
				d.ev.handle = C.int32_t(h)
			} else {
				id, err := c.eng.registerPodSpec(d, b.arena)
				if err != nil {
					logger.Warn("Pod spec outside the supported domain", err)
					continue
				}
				d.ev.op = C.KWOK_OP_UPSERT
				d.ev.handle = -1
				if known {
					d.ev.handle = C.int32_t(h)
				}
				d.ev.spec_id = C.int32_t(id)
				// the node by handle when the engine holds it (no name lookup on the host);
				// otherwise by spec.nodeName (a deleted node pods still reference, or none yet)
				d.ev.node_handle = -1
				if nh, ok := c.nodeHandle[str(b.arena, d.ev.node_name)]; ok {
					d.ev.node_handle = C.int32_t(nh)
				}
			}
			evs = append(evs, d.ev)
			keep = append(keep, r)
		}
		run = run[:0]
		for k := range created {
			delete(created, k)
		}
		hs, ss, _, err := c.eng.ingestPods(evs, b.arena)
		if err != nil {
			return err
		}
		for k, r := range keep {
			if ss[k] != C.KWOK_OK {
				continue
			}
			uid := b.uids[r.i]
			if evs[k].op == C.KWOK_OP_DELETE {
				delete(c.podByUID, uid)
				delete(c.podUID, hs[k])
				delete(c.podRef, hs[k])
			} else {
				c.podByUID[uid] = hs[k]
				c.podUID[hs[k]] = uid
				c.podRef[hs[k]] = r.ref
			}
		}
		return nil
	}
	for i := range docs {
		if st[i] != C.KWOK_OK {
			logger.Warn("Pod outside the supported domain", fmt.Errorf("kwok status %d", st[i]))
			continue
		}
		uid := b.uids[i]
		if created[uid] { // its handle comes from the run before
			if err := flush(); err != nil {
				return err
			}
		}
		if _, known := c.podByUID[uid]; !known && !b.del[i] {
			created[uid] = true
		}
		d := &docs[i]
		run = append(run, rec{i, types.NamespacedName{Namespace: str(b.arena, d.namespace_), Name: str(b.arena, d.name)}})
	}
	return flush()
}
