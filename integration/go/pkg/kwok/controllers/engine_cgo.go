//go:build kwok_mi355x

// engine_cgo.go - the cgo binding of the MI355X engine (include/kwok_engine.h)
// for pkg/kwok/controllers.  Copy this directory's files into the reference's
// pkg/kwok/controllers and build with `-tags kwok_mi355x`; libkwok_engine.so
// and kwok_engine.h are expected under third_party/kwok_amd (INTEGRATION.md).
//
// Not compiled in this repository: the image has no Go toolchain.  Every C
// entry point called here is exercised through the same ABI by the ctypes
// tests (tests/test_abi.py and the GPU parity tests).

package controllers

/*
#cgo CFLAGS: -I${SRCDIR}/../../../third_party/kwok_amd/include
#cgo LDFLAGS: -L${SRCDIR}/../../../third_party/kwok_amd/lib -lkwok_engine -Wl,-rpath,${SRCDIR}/../../../third_party/kwok_amd/lib
#include <stdlib.h>
#include "kwok_engine.h"
*/
import "C"

import (
	"encoding/binary"
	"fmt"
	"net"
	"unsafe"

	"sigs.k8s.io/kwok/pkg/kwok/controllers/templates"
)

// output kinds handed to the apply callback of tick
const (
	kindHeartbeat = iota // configureHeartbeatNode body (node_controller.go:393-401)
	kindNodeInit         // configureNode body (node_controller.go:356-391)
	kindPodPatch         // configurePod body (pod_controller.go:377-402)
	kindDelete           // DeletePod of a pod without finalizers: Delete(grace 0) (pod_controller.go:155-183)
	kindDeleteFin        // DeletePod of a pod with finalizers: kwok_finalizer_patch, then Delete
)

// readChunk bounds one kwok_read_arena copy: the initial tick of a 1M-node /
// 10M-pod fleet is ~7 GB of patches, read and handed out piece by piece
const readChunk = 64 << 20

func boolToC(b bool) C.int32_t {
	if b {
		return 1
	}
	return 0
}

type gpuEngine struct {
	h       *C.kwok_engine
	hb      []int32 // heartbeat handle list of heartbeat epoch hbEpoch
	hbEpoch uint32
	// page-locked batch buffers (kwok_host_alloc), reused: kwok_ingest_pods reads
	// the records and strings in place from these (batches over KWOK_INGEST_CHUNK
	// records: copied by DMA, chunk by chunk), and writes the per-record results to
	// resBuf (a copy into pageable Go memory would stall the engine's next
	// transfers, DESIGN.md §11)
	evBuf, arBuf, resBuf, recBuf, rec12Buf hostBuf
	nodeIP                               uint32 // Config.NodeIP (kwok_pod_rec12's KWOK_REC_HOST_NODE_IP)
}

type hostBuf struct {
	p unsafe.Pointer
	n int
}

func (b *hostBuf) get(n int) (unsafe.Pointer, error) {
	if n > b.n || b.p == nil {
		if b.p != nil {
			C.kwok_host_free(b.p)
			b.p, b.n = nil, 0
		}
		want := n + n/4 + 64
		p := C.kwok_host_alloc(C.size_t(want))
		if p == nil {
			return nil, fmt.Errorf("kwok_host_alloc(%d): out of page-locked memory", want)
		}
		b.p, b.n = p, want
	}
	return b.p, nil
}

func (b *hostBuf) free() {
	if b.p != nil {
		C.kwok_host_free(b.p)
		b.p, b.n = nil, 0
	}
}

func (g *gpuEngine) lastError() string { return C.GoString(C.kwok_last_error(g.h)) }

// newGPUEngine replaces the per-object work of NewNodeController /
// NewPodController (node_controller.go:79-117, pod_controller.go:84-128) for
// one GPU.  startUnix is the StartTime() template value (controller.go:33).
func newGPUEngine(conf Config, startUnix int64, rank, world int, commID []byte) (*gpuEngine, error) {
	cidr, nodeIP := C.CString(conf.CIDR), C.CString(conf.NodeIP)
	defer C.free(unsafe.Pointer(cidr))
	defer C.free(unsafe.Pointer(nodeIP))
	// custom pod status / node initialization / heartbeat templates are compiled by
	// the engine (KWOK_EDOMAIN with the reason when one does not fit the kernels' programs)
	var custom C.int32_t
	podTpl, nodeTpl := C.CString(conf.PodStatusTemplate), C.CString(conf.NodeInitializationTemplate)
	hbTpl := C.CString(conf.NodeHeartbeatTemplate)
	defer C.free(unsafe.Pointer(podTpl))
	defer C.free(unsafe.Pointer(nodeTpl))
	defer C.free(unsafe.Pointer(hbTpl))
	if conf.PodStatusTemplate != templates.DefaultPodStatusTemplate {
		custom |= C.KWOK_TPL_POD
	}
	if conf.NodeInitializationTemplate != templates.DefaultNodeStatusTemplate {
		custom |= C.KWOK_TPL_NODE_INIT
	}
	if conf.NodeHeartbeatTemplate != templates.DefaultNodeHeartbeatTemplate {
		custom |= C.KWOK_TPL_HEARTBEAT
	}
	cfg := C.kwok_config{
		abi_version:             C.KWOK_ABI_VERSION,
		cidr:                    cidr,
		node_ip:                 nodeIP,
		start_time_unix:         C.int64_t(startUnix),
		enable_cni:              boolToC(conf.EnableCNI), // IPs from cni.Setup: INTEGRATION.md "EnableCNI"
		custom_templates:        custom,
		pod_status_template:     podTpl,
		node_init_template:      nodeTpl,
		node_heartbeat_template: hbTpl,
		// every heartbeat patch of a tick is the same body (node_controller.go:393-401): the
		// tick materialises ONE, tick() reads it once and sends it to every managed node
		flags:                   C.KWOK_CFG_HEARTBEAT_ONCE,
		buckets:                 4096,
		node_slots_per_bucket:   64,
		pod_slots_per_bucket:    640,   // initial capacity; a bucket grows when a batch would fill it ...
		pod_handle_stride:       65528, // ... up to this many pods (e.g. 1000+ pods on one node)
		max_pod_specs:           4096,
		rank:                    C.int32_t(rank),
		world_size:              C.int32_t(world),
		device:                  C.int32_t(rank),
	}
	if world > 1 {
		if len(commID) != C.KWOK_COMM_ID_BYTES {
			return nil, fmt.Errorf("kwok: %d ranks need a %d-byte communicator id (kwokCommID on rank 0)", world, C.KWOK_COMM_ID_BYTES)
		}
		id := C.CBytes(commID)
		defer C.free(id)
		cfg.comm_id = (*C.uint8_t)(id)
	}
	var h *C.kwok_engine
	if rc := C.kwok_engine_create(&cfg, &h); rc != C.KWOK_OK {
		return nil, fmt.Errorf("kwok_engine_create: %d: %s", int(rc), C.GoString(C.kwok_last_error(nil)))
	}
	g := &gpuEngine{h: h}
	if ip := net.ParseIP(conf.NodeIP).To4(); ip != nil {
		g.nodeIP = binary.BigEndian.Uint32(ip)
	}
	return g, nil
}

// kwokCommID: the RCCL communicator id rank 0 creates and sends to the other ranks.
func kwokCommID() ([]byte, error) {
	buf := make([]byte, C.KWOK_COMM_ID_BYTES)
	if rc := C.kwok_comm_id((*C.uint8_t)(unsafe.Pointer(&buf[0]))); rc != C.KWOK_OK {
		return nil, fmt.Errorf("kwok_comm_id: %d", int(rc))
	}
	return buf, nil
}

func (g *gpuEngine) close() {
	if g.h != nil {
		C.kwok_engine_destroy(g.h)
		g.h = nil
	}
	g.evBuf.free()
	g.arBuf.free()
	g.resBuf.free()
	g.recBuf.free()
	g.rec12Buf.free()
}

func arenaPtr(arena []byte) *C.char {
	if len(arena) == 0 {
		return nil
	}
	return (*C.char)(unsafe.Pointer(&arena[0]))
}

// registerPodSpec: the spec id of a decoded pod's containers / init containers /
// readiness gates (their strings are kwok_str refs into arena).
func (g *gpuEngine) registerPodSpec(doc *C.kwok_pod_doc, arena []byte) (int32, error) {
	spec := C.kwok_pod_spec{
		containers:        &doc.containers[0],
		n_containers:      doc.n_containers,
		init_containers:   &doc.init_containers[0],
		n_init_containers: doc.n_init_containers,
		readiness_gates:   &doc.readiness_gates[0],
		n_readiness_gates: doc.n_readiness_gates,
	}
	var id C.int32_t
	if rc := C.kwok_register_pod_spec(g.h, &spec, arenaPtr(arena), C.size_t(len(arena)), &id); rc != C.KWOK_OK {
		return -1, fmt.Errorf("kwok_register_pod_spec: %d: %s", int(rc), g.lastError())
	}
	return int32(id), nil
}

// ingestNodes: one batch of node watch records in event order; per record the
// handle and status (KWOK_OK, KWOK_EDOMAIN, ...).  The records go into the
// page-locked record buffer and the strings they reference (the name, the status
// JSON and nodeInfo fields) into the page-locked arena, which kwok_ingest_nodes'
// prep kernel reads in place: the batch's object JSON stays on the host.
func (g *gpuEngine) ingestNodes(evs []C.kwok_node_event, arena []byte) (handles, status []int32, err error) {
	n := len(evs)
	handles, status = make([]int32, n), make([]int32, n)
	if n == 0 {
		return
	}
	evp, err := g.evBuf.get(n * int(unsafe.Sizeof(evs[0])))
	if err != nil {
		return
	}
	ev := unsafe.Slice((*C.kwok_node_event)(evp), n)
	strs := func(x *C.kwok_node_event) []*C.kwok_str {
		out := []*C.kwok_str{&x.name, &x.addresses, &x.allocatable, &x.capacity}
		for k := range x.node_info {
			out = append(out, &x.node_info[k])
		}
		return out
	}
	need := 0
	for i := range evs {
		for _, s := range strs(&evs[i]) {
			need += int(s.len)
		}
	}
	arp, err := g.arBuf.get(need + 1)
	if err != nil {
		return
	}
	ar := unsafe.Slice((*byte)(arp), need+1)
	off := 0
	for i := range evs {
		ev[i] = evs[i]
		for _, s := range strs(&ev[i]) {
			k := copy(ar[off:], arena[s.off:s.off+s.len])
			s.off, s.len = C.uint32_t(off), C.uint32_t(k)
			off += k
		}
	}
	resp, err := g.resBuf.get(2 * 4 * n)
	if err != nil {
		return
	}
	res := unsafe.Slice((*int32)(resp), 2*n)
	rc := C.kwok_ingest_nodes(g.h, &ev[0], C.size_t(n), (*C.char)(unsafe.Pointer(&ar[0])), C.size_t(off),
		(*C.int32_t)(&res[0]), (*C.int32_t)(&res[n]))
	if rc < 0 {
		err = fmt.Errorf("kwok_ingest_nodes: %d: %s", int(rc), g.lastError())
		return
	}
	copy(handles, res[:n])
	copy(status, res[n:])
	return
}

// ingestPods: one batch of pod records in event order.  Every record the
// compact wire forms can carry (kwok_pack_pod_events: IPs as integers, a new
// pod's node by handle) goes as a 12-byte kwok_pod_rec12 through
// kwok_ingest_pods_packed12 when its hostIP is empty or NodeIP (every pod kwok
// runs: pod.status.tpl renders NodeIP) and it is no create holding a podIP, else
// as a 20-byte kwok_pod_rec through kwok_ingest_pods_packed; the rest (a pod naming a node the engine holds no
// handle for) as kwok_pod_event with its strings through kwok_ingest_pods.
// Consecutive records of one form are one call: applying the calls in order is
// applying the batch.  All read page-locked buffers (kwok_host_alloc).
func (g *gpuEngine) ingestPods(evs []C.kwok_pod_event, arena []byte) (handles, status []int32, released []uint32, err error) {
	n := len(evs)
	handles, status, released = make([]int32, n), make([]int32, n), make([]uint32, n)
	if n == 0 {
		return
	}
	recp, err := g.recBuf.get(n * int(unsafe.Sizeof(C.kwok_pod_rec{})))
	if err != nil {
		return
	}
	recs := unsafe.Slice((*C.kwok_pod_rec)(recp), n)
	pst := make([]int32, n)
	C.kwok_pack_pod_events(&evs[0], C.size_t(n), arenaPtr(arena), C.size_t(len(arena)), &recs[0], (*C.int32_t)(&pst[0]))
	form := func(k int) int {
		if pst[k] != C.KWOK_OK {
			return 0
		}
		newWithIP := recs[k].op&C.KWOK_REC_NEW != 0 && recs[k].pod_ip != 0
		if h := uint32(recs[k].host_ip); (h == 0 || h == g.nodeIP) && !newWithIP {
			return 12
		}
		return 20
	}
	for i := 0; i < n; {
		f := form(i)
		j := i + 1
		for j < n && form(j) == f {
			j++
		}
		if f == 12 {
			err = g.ingestPacked12(recs[i:j], handles[i:j], status[i:j], released[i:j])
		} else if f == 20 {
			err = g.ingestPacked(recs[i:j], handles[i:j], status[i:j], released[i:j])
		} else {
			err = g.ingestFull(evs[i:j], arena, handles[i:j], status[i:j], released[i:j])
		}
		if err != nil {
			return
		}
		i = j
	}
	return
}

// ingestPacked: kwok_ingest_pods_packed of records in page-locked memory
// (statuses come back as bytes)
func (g *gpuEngine) ingestPacked(recs []C.kwok_pod_rec, handles, status []int32, released []uint32) error {
	n := len(recs)
	resp, err := g.resBuf.get(9 * n)
	if err != nil {
		return err
	}
	h := unsafe.Slice((*int32)(resp), n)
	rel := unsafe.Slice((*uint32)(unsafe.Add(resp, 4*n)), n)
	st := unsafe.Slice((*int8)(unsafe.Add(resp, 8*n)), n)
	rc := C.kwok_ingest_pods_packed(g.h, &recs[0], C.size_t(n), (*C.int32_t)(&h[0]), (*C.int8_t)(&st[0]),
		(*C.uint32_t)(&rel[0]))
	if rc < 0 {
		return fmt.Errorf("kwok_ingest_pods_packed: %d: %s", int(rc), g.lastError())
	}
	copy(handles, h)
	copy(released, rel)
	for i := range st {
		status[i] = int32(st[i])
	}
	return nil
}

// ingestPacked12: kwok_ingest_pods_packed12 of the records as kwok_pod_rec12 in
// page-locked memory (value: a create's creationTimestamp, any other record's
// podIP); the creates' handles come back in create order, every other record's
// handle is its target
func (g *gpuEngine) ingestPacked12(recs []C.kwok_pod_rec, handles, status []int32, released []uint32) error {
	n := len(recs)
	rp, err := g.rec12Buf.get(n * int(unsafe.Sizeof(C.kwok_pod_rec12{})))
	if err != nil {
		return err
	}
	r12 := unsafe.Slice((*C.kwok_pod_rec12)(rp), n)
	nNew := 0
	for i := range recs {
		op := recs[i].op
		if recs[i].host_ip != 0 {
			op |= C.KWOK_REC_HOST_NODE_IP
		}
		value := recs[i].pod_ip
		if recs[i].op&C.KWOK_REC_NEW != 0 {
			nNew++
			value = recs[i].creation
		}
		r12[i] = C.kwok_pod_rec12{op: op, flags: recs[i].flags, spec_id: recs[i].spec_id, target: recs[i].target,
			value: value}
	}
	resp, err := g.resBuf.get(9 * n)
	if err != nil {
		return err
	}
	h := unsafe.Slice((*int32)(resp), n) // (the first nNew entries: the creates' handles)
	rel := unsafe.Slice((*uint32)(unsafe.Add(resp, 4*n)), n)
	st := unsafe.Slice((*int8)(unsafe.Add(resp, 8*n)), n)
	rc := C.kwok_ingest_pods_packed12(g.h, &r12[0], C.size_t(n), (*C.int32_t)(&h[0]), C.size_t(nNew),
		(*C.int8_t)(&st[0]), (*C.uint32_t)(&rel[0]))
	if rc < 0 {
		return fmt.Errorf("kwok_ingest_pods_packed12: %d: %s", int(rc), g.lastError())
	}
	k := 0
	for i := range recs {
		if recs[i].op&C.KWOK_REC_NEW != 0 {
			handles[i] = h[k]
			k++
		} else {
			handles[i] = int32(recs[i].target)
		}
		status[i] = int32(st[i])
	}
	copy(released, rel)
	return nil
}

// ingestFull copies the records into the page-locked record buffer and packs
// the strings they reference (spec.nodeName, status.hostIP / podIP) into the
// page-locked arena: the batch's object JSON stays on the host.
func (g *gpuEngine) ingestFull(evs []C.kwok_pod_event, arena []byte, handles, status []int32, released []uint32) error {
	evp, err := g.evBuf.get(len(evs) * int(unsafe.Sizeof(evs[0])))
	if err != nil {
		return err
	}
	ev := unsafe.Slice((*C.kwok_pod_event)(evp), len(evs))
	need := 0
	for i := range evs {
		need += int(evs[i].node_name.len + evs[i].host_ip.len + evs[i].pod_ip.len)
	}
	arp, err := g.arBuf.get(need + 1)
	if err != nil {
		return err
	}
	ar := unsafe.Slice((*byte)(arp), need+1)
	off := 0
	pack := func(s C.kwok_str) C.kwok_str {
		n := copy(ar[off:], arena[s.off:s.off+s.len])
		r := C.kwok_str{off: C.uint32_t(off), len: C.uint32_t(n)}
		off += n
		return r
	}
	for i := range evs {
		ev[i] = evs[i]
		ev[i].node_name, ev[i].host_ip, ev[i].pod_ip = pack(evs[i].node_name), pack(evs[i].host_ip), pack(evs[i].pod_ip)
	}
	n := len(ev)
	resp, err := g.resBuf.get(3 * 4 * n)
	if err != nil {
		return err
	}
	res := unsafe.Slice((*int32)(resp), 3*n)
	rc := C.kwok_ingest_pods(g.h, &ev[0], C.size_t(n), (*C.char)(unsafe.Pointer(&ar[0])), C.size_t(off),
		(*C.int32_t)(&res[0]), (*C.int32_t)(&res[n]), (*C.uint32_t)(unsafe.Pointer(&res[2*n])))
	if rc < 0 {
		return fmt.Errorf("kwok_ingest_pods: %d: %s", int(rc), g.lastError())
	}
	copy(handles, res[:n])
	copy(status, res[n:2*n])
	for i := range released {
		released[i] = uint32(res[2*n+i])
	}
	return nil
}

// ingestPodsJSON: kwok_ingest_pods_json - the pod documents themselves (one run of
// a batch, see flushPods) decoded on the GPU (the host codec only for the
// documents the device scanner leaves undecided, specs registered as they
// first appear) and routed by the GPU event switch, the records never leaving
// HBM.  The documents are staged in page-locked memory (the engine copies them
// in pieces, each decoded as it lands).  ops[i] / handles[i]: Deleted ->
// KWOK_OP_DELETE with the pod's handle; else KWOK_OP_UPSERT with its handle, -1
// for a new pod (its node by spec.nodeName).
func (g *gpuEngine) ingestPodsJSON(codec *gpuCodec, arena []byte, offs []uint64, lens []uint32, ops []uint8,
	handles []int32) (outHandles, status []int32, nHost int, err error) {
	n := len(offs)
	outHandles, status = make([]int32, n), make([]int32, n)
	if n == 0 {
		return
	}
	arp, err := g.arBuf.get(len(arena) + 1)
	if err != nil {
		return
	}
	ar := unsafe.Slice((*byte)(arp), len(arena)+1)
	copy(ar, arena)
	resp, err := g.resBuf.get(3 * 4 * n)
	if err != nil {
		return
	}
	res := unsafe.Slice((*int32)(resp), 3*n)
	var nh C.size_t
	rc := C.kwok_ingest_pods_json(g.h, codec.c, (*C.char)(unsafe.Pointer(&ar[0])), C.size_t(len(arena)),
		(*C.uint64_t)(&offs[0]), (*C.uint32_t)(&lens[0]), (*C.uint8_t)(&ops[0]), (*C.int32_t)(&handles[0]),
		C.size_t(n), (*C.int32_t)(&res[0]), (*C.int32_t)(&res[n]), (*C.uint32_t)(unsafe.Pointer(&res[2*n])), &nh)
	if rc < 0 {
		err = fmt.Errorf("kwok_ingest_pods_json: %d: %s", int(rc), g.lastError())
		return
	}
	copy(outHandles, res[:n])
	copy(status, res[n:2*n])
	nHost = int(nh)
	return
}

// ingestNodesJSON: kwok_ingest_nodes_json - one batch of node documents decoded on
// the GPU and routed by the GPU event switch (the documents staged in page-locked
// memory).  ops[i]: Deleted -> KWOK_OP_DELETE (its status is not read), else
// KWOK_OP_UPSERT.
func (g *gpuEngine) ingestNodesJSON(codec *gpuCodec, arena []byte, offs []uint64, lens []uint32,
	ops []uint8) (handles, status []int32, nHost int, err error) {
	n := len(offs)
	handles, status = make([]int32, n), make([]int32, n)
	if n == 0 {
		return
	}
	arp, err := g.arBuf.get(len(arena) + 1)
	if err != nil {
		return
	}
	ar := unsafe.Slice((*byte)(arp), len(arena)+1)
	copy(ar, arena)
	resp, err := g.resBuf.get(2 * 4 * n)
	if err != nil {
		return
	}
	res := unsafe.Slice((*int32)(resp), 2*n)
	var nh C.size_t
	rc := C.kwok_ingest_nodes_json(g.h, codec.c, (*C.char)(unsafe.Pointer(&ar[0])), C.size_t(len(arena)),
		(*C.uint64_t)(&offs[0]), (*C.uint32_t)(&lens[0]), (*C.uint8_t)(&ops[0]), C.size_t(n),
		(*C.int32_t)(&res[0]), (*C.int32_t)(&res[n]), &nh)
	if rc < 0 {
		err = fmt.Errorf("kwok_ingest_nodes_json: %d: %s", int(rc), g.lastError())
		return
	}
	copy(handles, res[:n])
	copy(status, res[n:2*n])
	nHost = int(nh)
	return
}

// poolPut replicates IPs another rank released at ingest time (multi-GPU).
func (g *gpuEngine) poolPut(ips []uint32) error {
	if len(ips) == 0 {
		return nil
	}
	if rc := C.kwok_pool_put(g.h, (*C.uint32_t)(&ips[0]), C.size_t(len(ips))); rc != C.KWOK_OK {
		return fmt.Errorf("kwok_pool_put: %s", g.lastError())
	}
	return nil
}

func finalizerPatch() []byte {
	var n C.size_t
	p := C.kwok_finalizer_patch(&n)
	return C.GoBytes(unsafe.Pointer(p), C.int(n))
}

// tick runs one heartbeat interval and hands every body to apply.  The lists
// come first (kwok_read_outputs without an arena); then ONE heartbeat body (all
// bodies of a tick are identical, node_controller.go:393-401; the engine is
// created with KWOK_CFG_HEARTBEAT_ONCE, so the tick wrote only that one, at
// heartbeat_off, and moved the SoA state, not 1M copies) and the node-init
// / pod patches in bounded pieces (kwok_read_arena, 64-bit offsets), each copied
// once, straight into Go memory (the engine keeps no pointer past the call).  A
// steady tick at 1M nodes moves ~1 KB over PCIe, not 1 GB.  The heartbeat handle
// list is read only when its epoch changed.  Body slices stay valid after tick
// returns (each aliases its piece's buffer).
func (g *gpuEngine) tick(nowUnix int64, apply func(kind int, handle int32, body []byte)) error {
	var res C.kwok_tick_result
	if rc := C.kwok_tick(g.h, C.int64_t(nowUnix), &res); rc != C.KWOK_OK {
		return fmt.Errorf("kwok_tick: %s", g.lastError())
	}
	newEpoch := g.hb == nil || uint32(res.heartbeat_epoch) != g.hbEpoch
	if newEpoch {
		g.hb = make([]int32, res.n_heartbeat) // filled by kwok_read_outputs below
	}
	ini := make([]int32, res.n_node_init)
	iniOff := make([]uint64, res.n_node_init)
	iniLen := make([]uint32, res.n_node_init)
	pp := make([]int32, res.n_pod_patch)
	ppOff := make([]uint64, res.n_pod_patch)
	ppLen := make([]uint32, res.n_pod_patch)
	del := make([]int32, res.n_delete)
	delFin := make([]uint8, res.n_delete)
	var out C.kwok_outputs // no arena: the bytes follow through kwok_read_arena
	if len(g.hb) > 0 && newEpoch {
		out.heartbeat_nodes = (*C.int32_t)(&g.hb[0])
	}
	if len(ini) > 0 {
		out.node_init_nodes, out.node_init_off, out.node_init_len =
			(*C.int32_t)(&ini[0]), (*C.uint64_t)(&iniOff[0]), (*C.uint32_t)(&iniLen[0])
	}
	if len(pp) > 0 {
		out.pod_patch_pods, out.pod_patch_off, out.pod_patch_len =
			(*C.int32_t)(&pp[0]), (*C.uint64_t)(&ppOff[0]), (*C.uint32_t)(&ppLen[0])
	}
	if len(del) > 0 {
		out.delete_pods, out.delete_has_finalizers = (*C.int32_t)(&del[0]), (*C.uint8_t)(&delFin[0])
	}
	if rc := C.kwok_read_outputs(g.h, &out); rc != C.KWOK_OK {
		return fmt.Errorf("kwok_read_outputs: %s", g.lastError())
	}
	g.hbEpoch = uint32(res.heartbeat_epoch)
	if res.n_heartbeat > 0 {
		body := make([]byte, res.heartbeat_len) // the heartbeat body, sent to every managed node
		if err := g.readArena(uint64(out.heartbeat_off), body); err != nil {
			return err
		}
		for _, h := range g.hb {
			apply(kindHeartbeat, h, body)
		}
	}
	if err := g.applyPatches(kindNodeInit, ini, iniOff, iniLen, apply); err != nil {
		return err
	}
	if err := g.applyPatches(kindPodPatch, pp, ppOff, ppLen, apply); err != nil {
		return err
	}
	for i, h := range del { // Patch(removeFinalizers) if the pod has finalizers, then Delete(grace 0)
		if delFin[i] != 0 {
			apply(kindDeleteFin, h, nil)
		} else {
			apply(kindDelete, h, nil)
		}
	}
	return nil
}

// applyPatches: the patches at offs[i] / lens[i] (increasing offsets), read in
// pieces of at most readChunk bytes (a single larger patch is one piece)
func (g *gpuEngine) applyPatches(kind int, hs []int32, offs []uint64, lens []uint32,
	apply func(kind int, handle int32, body []byte)) error {
	for i := 0; i < len(hs); {
		lo := offs[i]
		j := i + 1
		for j < len(hs) && offs[j]+uint64(lens[j])-lo <= readChunk {
			j++
		}
		buf := make([]byte, offs[j-1]+uint64(lens[j-1])-lo)
		if err := g.readArena(lo, buf); err != nil {
			return err
		}
		for k := i; k < j; k++ {
			apply(kind, hs[k], buf[offs[k]-lo:offs[k]-lo+uint64(lens[k])])
		}
		i = j
	}
	return nil
}

// readArena copies arena bytes [off, off+len(buf)) of the collected tick into buf
func (g *gpuEngine) readArena(off uint64, buf []byte) error {
	if len(buf) == 0 {
		return nil
	}
	if rc := C.kwok_read_arena(g.h, C.uint64_t(off), C.uint64_t(len(buf)), unsafe.Pointer(&buf[0])); rc != C.KWOK_OK {
		return fmt.Errorf("kwok_read_arena: %s", g.lastError())
	}
	return nil
}

// ---- EnableCNI: configurePod's cni.Setup (pod_controller.go:383-389) ----------

// cniPending: the pods the next tick evaluates that hold no podIP, canonical order
func (g *gpuEngine) cniPending() ([]int32, error) {
	var n C.size_t
	if rc := C.kwok_cni_pending(g.h, nil, 0, &n); rc != C.KWOK_OK && n == 0 {
		return nil, fmt.Errorf("kwok_cni_pending: %s", g.lastError())
	}
	hs := make([]int32, n)
	if n == 0 {
		return hs, nil
	}
	if rc := C.kwok_cni_pending(g.h, (*C.int32_t)(&hs[0]), C.size_t(len(hs)), &n); rc != C.KWOK_OK {
		return nil, fmt.Errorf("kwok_cni_pending: %s", g.lastError())
	}
	return hs[:n], nil
}

// cniAssign: the first IP cni.Setup returned per pod (IPv4, host order)
func (g *gpuEngine) cniAssign(hs []int32, ips []uint32) error {
	if len(hs) == 0 {
		return nil
	}
	st := make([]int32, len(hs))
	if rc := C.kwok_cni_assign(g.h, (*C.int32_t)(&hs[0]), (*C.uint32_t)(&ips[0]), C.size_t(len(hs)),
		(*C.int32_t)(&st[0])); rc < 0 {
		return fmt.Errorf("kwok_cni_assign: %s", g.lastError())
	}
	return nil
}

// nodeHas / nodeSize: NodeController.Has / Size (node_controller.go:403-409)
func (g *gpuEngine) nodeHas(name string) bool {
	if name == "" {
		return false
	}
	b := []byte(name)
	return C.kwok_node_has(g.h, (*C.char)(unsafe.Pointer(&b[0])), C.size_t(len(b))) != 0
}

func (g *gpuEngine) nodeSize() int { return int(C.kwok_node_size(g.h)) }

// ---- host codec: watch objects as JSON -> records (kwok_decode_*) ----------

type gpuCodec struct{ c *C.kwok_codec }

func newGPUCodec(conf Config) (*gpuCodec, error) {
	cs := []*C.char{
		C.CString(conf.ManageNodesWithAnnotationSelector), C.CString(conf.ManageNodesWithLabelSelector),
		C.CString(conf.DisregardStatusWithAnnotationSelector), C.CString(conf.DisregardStatusWithLabelSelector),
	}
	defer func() {
		for _, p := range cs {
			C.free(unsafe.Pointer(p))
		}
	}()
	cfg := C.kwok_codec_config{
		manage_all_nodes:                          boolToC(conf.ManageAllNodes),
		manage_nodes_with_annotation_selector:     cs[0],
		manage_nodes_with_label_selector:          cs[1],
		disregard_status_with_annotation_selector: cs[2],
		disregard_status_with_label_selector:      cs[3],
	}
	var c *C.kwok_codec
	if rc := C.kwok_codec_create(&cfg, &c); rc != C.KWOK_OK { // labels.Parse errors surface here
		return nil, fmt.Errorf("kwok_codec_create: %s", C.GoString(C.kwok_codec_last_error()))
	}
	return &gpuCodec{c: c}, nil
}

func (d *gpuCodec) close() { C.kwok_codec_destroy(d.c) }

// decodeNodes / decodePods: objects at offs[i] / lens[i] of arena (their JSON,
// concatenated) -> records whose strings point into the same arena (node status
// blobs are re-serialised in place).  status[i] != KWOK_OK: outside the domain.
func (d *gpuCodec) decodeNodes(arena []byte, offs []uint64, lens []uint32, threads int) ([]C.kwok_node_event, []int32) {
	ev, st := make([]C.kwok_node_event, len(offs)), make([]int32, len(offs))
	if len(offs) > 0 {
		C.kwok_decode_nodes(d.c, arenaPtr(arena), C.size_t(len(arena)), (*C.uint64_t)(&offs[0]),
			(*C.uint32_t)(&lens[0]), C.size_t(len(offs)), C.int(threads), &ev[0], (*C.int32_t)(&st[0]))
	}
	return ev, st
}

func (d *gpuCodec) decodePods(arena []byte, offs []uint64, lens []uint32, threads int) ([]C.kwok_pod_doc, []int32) {
	docs, st := make([]C.kwok_pod_doc, len(offs)), make([]int32, len(offs))
	if len(offs) > 0 {
		C.kwok_decode_pods(d.c, arenaPtr(arena), C.size_t(len(arena)), (*C.uint64_t)(&offs[0]),
			(*C.uint32_t)(&lens[0]), C.size_t(len(offs)), C.int(threads), &docs[0], (*C.int32_t)(&st[0]))
	}
	return docs, st
}

func str(arena []byte, s C.kwok_str) string { return string(arena[s.off : s.off+s.len]) }
