// Package sketchgpu binds Go2NetSpectra's sketch aggregator to the MI355X engine
// (libgns_sketch.so, C ABI in include/gns_sketch.h) through cgo.
//
// It provides:
//   - CountMin: a statistic.Sketch (internal/engine/impl/sketch/statistic/sketch.go:5-10)
//     whose Insert/Query/HeavyHitters/Reset run on the GPU, plus InsertBatch for the
//     batched path;
//   - SuperSpread and Exact, the same way;
//   - task.go: GPUTask, a model.Task (internal/model/task.go:6-15) registered as the
//     "sketch_gpu" aggregator with factory.RegisterAggregator
//     (internal/factory/task_factory.go:24), whose ProcessPacket batches PacketInfo and
//     submits the batch with gns_{cm,ss}_insert_tuples instead of one CAS insert per
//     packet per worker.
//
// Build: CGO_CFLAGS="-I<repo>/include" CGO_LDFLAGS="-L<repo>/go2netspectra_amd -lgns_sketch".
// Not compiled in the build container (no Go toolchain there).
package sketchgpu

/*
#cgo LDFLAGS: -lgns_sketch
#include <stdlib.h>
#include "gns_sketch.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"log"
	"sync"
	"unsafe"

	"Go2NetSpectra/internal/engine/impl/sketch/statistic"
)

var fieldIDs = map[string]C.uint8_t{"SrcIP": 1, "DstIP": 2, "SrcPort": 3, "DstPort": 4, "Protocol": 5}

func lastErr(rc C.int) error {
	if rc == C.GNS_OK {
		return nil
	}
	return errors.New(C.GoString(C.gns_last_error()))
}

// CountMin mirrors statistic.CountMin (count_min.go) on one GPU.
type CountMin struct {
	h        *C.gns_cm
	keyBytes int
	err      error // first insert failure of the period (Insert has no error return)
}

// sticky keeps the first failure of a measurement period and logs it the way
// the reference logs a dropped packet (task.go:162-166).  The engine has no
// traffic-dependent failure left (its flow dictionary grows, include/gns_sketch.h),
// so this reports device / runtime errors.
func sticky(dst *error, err error) {
	if err != nil && *dst == nil {
		*dst = err
		log.Printf("sketchgpu: insert failed, packets are dropped until Reset: %v", err)
	}
}

// NewCountMin replaces statistic.NewCountMin (count_min.go:47-90); seeds are injected.
func NewCountMin(width, depth, st, ct uint32, flowFields []string, keyBytes uint32, seeds []uint32,
	maxFlows uint64, device int) (*CountMin, error) {
	var p C.gns_cm_params
	p.width, p.depth = C.uint32_t(width), C.uint32_t(depth)
	p.size_threshold, p.count_threshold = C.uint32_t(st), C.uint32_t(ct)
	p.flow.n_fields = C.uint32_t(len(flowFields))
	for i, f := range flowFields {
		p.flow.fields[i] = fieldIDs[f]
	}
	p.key_bytes = C.uint32_t(keyBytes)
	if len(seeds) > 0 {
		p.seeds = (*C.uint32_t)(unsafe.Pointer(&seeds[0]))
	}
	p.max_flows = C.uint64_t(maxFlows)
	p.device = C.int(device)
	var h *C.gns_cm
	if err := lastErr(C.gns_cm_create(&p, &h)); err != nil {
		return nil, err
	}
	return &CountMin{h: h, keyBytes: int(keyBytes)}, nil
}

// Insert implements statistic.Sketch for one packet (a batch of one; prefer InsertBatch).
func (c *CountMin) Insert(flow, elem []byte, size uint32) {
	if len(flow) == 0 {
		return
	}
	sticky(&c.err, c.InsertBatch(flow, uint32(len(flow)), []uint32{size}))
}

// Err reports the first insert failure since the last Reset (nil if none).
func (c *CountMin) Err() error { return c.err }

// InsertBatch: keys is n*stride bytes, sizes n entries, applied in order.
func (c *CountMin) InsertBatch(keys []byte, stride uint32, sizes []uint32) error {
	if len(sizes) == 0 {
		return nil
	}
	return lastErr(C.gns_cm_insert_keys(c.h, (*C.uint8_t)(unsafe.Pointer(&keys[0])), C.uint32_t(stride),
		(*C.uint32_t)(unsafe.Pointer(&sizes[0])), C.uint64_t(len(sizes)), C.GNS_MEM_HOST))
}

// InsertTuples: PacketInfo batch as SoA (task.go:156-169 for a whole batch).
func (c *CountMin) InsertTuples(src16, dst16 []byte, sport, dport []uint16, proto []uint8, length []uint32) error {
	n := len(length)
	if n == 0 {
		return nil
	}
	t := C.gns_tuples{
		src16: (*C.uint8_t)(unsafe.Pointer(&src16[0])), dst16: (*C.uint8_t)(unsafe.Pointer(&dst16[0])),
		sport: (*C.uint16_t)(unsafe.Pointer(&sport[0])), dport: (*C.uint16_t)(unsafe.Pointer(&dport[0])),
		proto: (*C.uint8_t)(unsafe.Pointer(&proto[0])), length: (*C.uint32_t)(unsafe.Pointer(&length[0])),
	}
	return lastErr(C.gns_cm_insert_tuples(c.h, &t, C.uint64_t(n), C.GNS_MEM_HOST))
}

// InsertHeaders: 64-byte header records + wire lengths (PackCapture's output),
// parsed on the GPU (pcap.Reader.ReadPackets + ParsePacketInto + ProcessPacket).
func (c *CountMin) InsertHeaders(hdr []byte, wirelen []uint32) error {
	if len(wirelen) == 0 {
		return nil
	}
	return lastErr(C.gns_cm_insert_headers(c.h, (*C.uint8_t)(unsafe.Pointer(&hdr[0])),
		(*C.uint32_t)(unsafe.Pointer(&wirelen[0])), C.uint64_t(len(wirelen)), C.GNS_MEM_HOST))
}

// PackCapture replaces pcap.NewReader + Reader.ReadPackets (pkg/pcap/reader.go:20-49)
// on the ingest side: one pass over a classic pcap or pcapng file (what libpcap's
// pcap_open_offline reads) into 64-byte header records, wire lengths and capture
// timestamps in ns, ready for InsertHeaders.
func PackCapture(path string) (hdr []byte, wirelen []uint32, tsNs []int64, err error) {
	cpath := C.CString(path)
	defer C.free(unsafe.Pointer(cpath))
	var total C.uint64_t
	if r := C.gns_pack_pcap(cpath, nil, nil, 0, &total); r < 0 {
		return nil, nil, nil, lastErr(C.int(r))
	}
	n := int(total)
	if n == 0 {
		return nil, nil, nil, nil
	}
	hdr, wirelen, tsNs = make([]byte, 64*n), make([]uint32, n), make([]int64, n)
	r := C.gns_pack_pcap_ts(cpath, (*C.uint8_t)(unsafe.Pointer(&hdr[0])), (*C.uint32_t)(unsafe.Pointer(&wirelen[0])),
		(*C.int64_t)(unsafe.Pointer(&tsNs[0])), C.uint64_t(n), &total)
	if r < 0 {
		return nil, nil, nil, lastErr(C.int(r))
	}
	return hdr[:64*int(r)], wirelen[:r], tsNs[:r], nil
}

// FrameRecord is the live-capture form of PackCapture (pcap.OpenLive feeding
// gopacket.NewPacketSource): one captured frame (packet.Data(), CaptureInfo.Length
// as wireLen) -> the 64-byte record PackCapture writes for it. kind: 0 copied
// verbatim, 1 decoded on the host into a pre-parsed record, 2 no IP layer (the
// engine drops the record, as ParsePacketInto returns "not an IP packet").
func FrameRecord(frame []byte, wireLen uint32, rec []byte) (kind int, err error) {
	if len(rec) < 64 {
		return 0, errors.New("record buffer shorter than 64 bytes")
	}
	var p *C.uint8_t
	if len(frame) > 0 {
		p = (*C.uint8_t)(unsafe.Pointer(&frame[0]))
	} else {
		p = (*C.uint8_t)(unsafe.Pointer(&rec[0])) // any non-nil pointer; caplen 0
	}
	r := C.gns_frame_record(p, C.uint32_t(len(frame)), C.uint32_t(wireLen), (*C.uint8_t)(unsafe.Pointer(&rec[0])))
	if r < 0 {
		return 0, lastErr(r)
	}
	return int(r), nil
}

// Reclaim drops flow-dictionary entries no bucket names any more (inserts also
// do it on their own when the dictionary fills); call it at a window boundary
// to take the rebuild off the ingest path.
func (c *CountMin) Reclaim() error { return lastErr(C.gns_cm_reclaim(c.h)) }

// DictStats: reclaims, dead flows dropped, live flows after the last reclaim,
// claimed slots, reclaim time (us), batches re-run after an overflow, slots, growths.
func (c *CountMin) DictStats() (out [8]uint64, err error) {
	err = lastErr(C.gns_cm_dict_stats(c.h, (*C.uint64_t)(unsafe.Pointer(&out[0]))))
	return
}

func layoutOf(fields []string) (l C.gns_layout) {
	l.n_fields = C.uint32_t(len(fields))
	for i, f := range fields {
		l.fields[i] = fieldIDs[f]
	}
	return
}

// Router shards a node's traffic over its GPUs by flow (SURVEY §8e): records are
// split on the device by owning GPU (stable per shard; exchange the runs with an
// all-to-all and insert each received run in source-rank order), and queries are
// answered by the shard that owns the flow.  The owner key is the fields every
// task keys on (gns_route_owner_fields): [SrcIP] when each task's flow key holds
// SrcIP, otherwise the fields the tasks share -- for one task its whole flow key
// (a flow key without SrcIP is legal, config.go:59).
type Router struct {
	r       *C.gns_route
	nshards int
}

// NewRouter shards by SrcIP (every task keys on SrcIP).
func NewRouter(nshards uint32, device int) (*Router, error) {
	return NewKeyedRouter(nshards, [][]string{{"SrcIP"}}, device)
}

// NewKeyedRouter derives the owner key from the tasks' flow fields (one slice per
// task: SketchTaskDef.FlowFields / exact KeyFields); it fails when the tasks share
// no field, since no GPU could then own every flow of every task.
func NewKeyedRouter(nshards uint32, taskFields [][]string, device int) (*Router, error) {
	if len(taskFields) == 0 {
		return nil, errors.New("sketchgpu: no tasks to shard")
	}
	lays := make([]C.gns_layout, len(taskFields))
	for i, f := range taskFields {
		lays[i] = layoutOf(f)
	}
	var owner C.gns_layout
	if err := lastErr(C.gns_route_owner_fields(&lays[0], C.uint32_t(len(lays)), &owner)); err != nil {
		return nil, err
	}
	var r *C.gns_route
	if err := lastErr(C.gns_route_create_keyed(C.uint32_t(nshards), &owner, C.int(device), &r)); err != nil {
		return nil, err
	}
	return &Router{r: r, nshards: int(nshards)}, nil
}

// Partition: hdr/wirelen/outHdr/outWirelen are device pointers (n records);
// counts receives the run length of every shard.
func (rt *Router) Partition(hdr, wirelen, outHdr, outWirelen unsafe.Pointer, n uint64, counts []uint64) error {
	return lastErr(C.gns_route_partition(rt.r, (*C.uint8_t)(hdr), (*C.uint32_t)(wirelen), C.uint64_t(n),
		(*C.uint8_t)(outHdr), (*C.uint32_t)(outWirelen), (*C.uint64_t)(unsafe.Pointer(&counts[0]))))
}

// Owners returns the shard owning each of the len(keys)/stride flow keys (laid out as
// keyFields, the querying task's FlowFields; they must contain every owner field).
func (rt *Router) Owners(keyFields []string, keys []byte, stride uint32) ([]uint32, error) {
	if stride == 0 {
		return nil, errors.New("sketchgpu: zero key stride")
	}
	n := len(keys) / int(stride)
	own := make([]uint32, n+1)
	if n == 0 {
		return own[:0], nil
	}
	lay := layoutOf(keyFields)
	err := lastErr(C.gns_route_owner_keys(rt.r, &lay, (*C.uint8_t)(unsafe.Pointer(&keys[0])), C.uint32_t(stride),
		C.uint64_t(n), (*C.uint32_t)(unsafe.Pointer(&own[0])), C.GNS_MEM_HOST))
	return own[:n], err
}

// BatchQuerier is a shard's batched Query (CountMin, SuperSpread, Exact).
type BatchQuerier interface {
	QueryBatch(keys []byte, stride uint32) ([]uint64, error)
}

// QueryRouted answers Query(flow) (count_min.go:160-174, super_spread.go:238-249) for
// len(keys)/stride flow keys, each from the shard owning its flow: shards[g] is the
// handle on GPU g (one process driving the node's GPUs).  The shards answer
// concurrently, every key once; the answers come back in key order.
func (rt *Router) QueryRouted(shards []BatchQuerier, keyFields []string, keys []byte, stride uint32) ([]uint64, error) {
	if len(shards) != rt.nshards {
		return nil, fmt.Errorf("sketchgpu: %d shard handles for a %d-shard router", len(shards), rt.nshards)
	}
	own, err := rt.Owners(keyFields, keys, stride)
	if err != nil {
		return nil, err
	}
	per := make([][]int, rt.nshards)
	for i, g := range own {
		per[g] = append(per[g], i)
	}
	out := make([]uint64, len(own))
	errs := make([]error, rt.nshards)
	var wg sync.WaitGroup
	for g, idx := range per {
		if len(idx) == 0 {
			continue
		}
		wg.Add(1)
		go func(g int, idx []int) {
			defer wg.Done()
			buf := make([]byte, 0, len(idx)*int(stride))
			for _, i := range idx {
				buf = append(buf, keys[i*int(stride):(i+1)*int(stride)]...)
			}
			ans, err := shards[g].QueryBatch(buf, stride)
			if err != nil {
				errs[g] = err
				return
			}
			for j, i := range idx {
				out[i] = ans[j]
			}
		}(g, idx)
	}
	wg.Wait()
	for _, e := range errs {
		if e != nil {
			return nil, e
		}
	}
	return out, nil
}

func (rt *Router) Close() { C.gns_route_destroy(rt.r) }

// Query implements statistic.Sketch (count_min.go:160-174).
func (c *CountMin) Query(flow []byte) uint64 {
	if len(flow) != c.keyBytes || len(flow) == 0 {
		return 0
	}
	var out C.uint64_t
	if C.gns_cm_query(c.h, (*C.uint8_t)(unsafe.Pointer(&flow[0])), C.uint32_t(len(flow)), 1, &out) != C.GNS_OK {
		return 0
	}
	return uint64(out)
}

// QueryBatch: Query for len(keys)/stride flows in one device call (count<<32 | size).
func (c *CountMin) QueryBatch(keys []byte, stride uint32) ([]uint64, error) {
	n := len(keys) / int(stride)
	out := make([]uint64, n+1)
	if n == 0 {
		return out[:0], nil
	}
	err := lastErr(C.gns_cm_query(c.h, (*C.uint8_t)(unsafe.Pointer(&keys[0])), C.uint32_t(stride), C.uint64_t(n),
		(*C.uint64_t)(unsafe.Pointer(&out[0]))))
	return out[:n], err
}

// HeavyHitters implements statistic.Sketch (count_min.go:178-247).
func (c *CountMin) HeavyHitters() statistic.HeavyRecord {
	return cmHeavy(c.keyBytes, func(cf *C.uint8_t, cv *C.uint32_t, nc *C.uint64_t, sf *C.uint8_t, sv *C.uint32_t,
		ns *C.uint64_t) C.int {
		return C.gns_cm_heavy_hitters(c.h, cf, cv, nc, sf, sv, ns)
	})
}

// cmHeavy runs a gns_cm_heavy_hitters-shaped call into Go buffers.  The call
// reports the full list lengths, which may exceed the buffers when the state
// changed since the sizing call (a View refreshed by its owner in between): the
// loop grows the buffers and calls again, so a list is never sliced past them.
func cmHeavy(K int, call func(cf *C.uint8_t, cv *C.uint32_t, nc *C.uint64_t, sf *C.uint8_t, sv *C.uint32_t,
	ns *C.uint64_t) C.int) statistic.HeavyRecord {
	empty := statistic.HeavyRecord{Size: []statistic.HeavySize{}, Count: []statistic.HeavyCount{}}
	capC, capS := 64, 64
	for tries := 0; tries < 8; tries++ {
		cf := make([]byte, capC*K+1)
		cv := make([]uint32, capC+1)
		sf := make([]byte, capS*K+1)
		sv := make([]uint32, capS+1)
		nc, ns := C.uint64_t(capC), C.uint64_t(capS)
		if call((*C.uint8_t)(unsafe.Pointer(&cf[0])), (*C.uint32_t)(unsafe.Pointer(&cv[0])), &nc,
			(*C.uint8_t)(unsafe.Pointer(&sf[0])), (*C.uint32_t)(unsafe.Pointer(&sv[0])), &ns) != C.GNS_OK {
			return empty
		}
		if int(nc) > capC || int(ns) > capS { // the lists outgrew the buffers: call again
			if int(nc) > capC {
				capC = 2 * int(nc)
			}
			if int(ns) > capS {
				capS = 2 * int(ns)
			}
			continue
		}
		rec := statistic.HeavyRecord{Size: make([]statistic.HeavySize, 0, int(ns)),
			Count: make([]statistic.HeavyCount, 0, int(nc))}
		for i := 0; i < int(ns); i++ {
			rec.Size = append(rec.Size, statistic.HeavySize{Flow: append([]byte(nil), sf[i*K:(i+1)*K]...), Size: sv[i]})
		}
		for i := 0; i < int(nc); i++ {
			rec.Count = append(rec.Count, statistic.HeavyCount{Flow: append([]byte(nil), cf[i*K:(i+1)*K]...), Count: cv[i]})
		}
		return rec
	}
	return empty
}

// Reset implements statistic.Sketch (count_min.go:249-265).
func (c *CountMin) Reset() {
	C.gns_cm_reset(c.h)
	c.err = nil
}

// Close releases the device sketch.
func (c *CountMin) Close() { C.gns_cm_destroy(c.h) }

var _ statistic.Sketch = (*CountMin)(nil)

// View is a snapshot of a CountMin for the snapshotter / alerter goroutines
// (manager.go:139-159 call Snapshot while the workers insert): the worker that
// owns the CountMin calls Refresh at a window boundary, and any other goroutine
// may call HeavyHitters / Query on the view meanwhile (gns_cm_view_*).
type View struct {
	v        *C.gns_cm_view
	keyBytes int
}

// NewView allocates the snapshot (16 bytes per bucket).
func (c *CountMin) NewView() (*View, error) {
	var v *C.gns_cm_view
	if err := lastErr(C.gns_cm_view_create(c.h, &v)); err != nil {
		return nil, err
	}
	return &View{v: v, keyBytes: c.keyBytes}, nil
}

// Refresh snapshots the buckets after every insert issued so far (owner goroutine only).
func (w *View) Refresh() error { return lastErr(C.gns_cm_view_refresh(w.v)) }

// HeavyHitters is CountMin.HeavyHitters at the last Refresh, safe during inserts.
func (w *View) HeavyHitters() statistic.HeavyRecord {
	return cmHeavy(w.keyBytes, func(cf *C.uint8_t, cv *C.uint32_t, nc *C.uint64_t, sf *C.uint8_t, sv *C.uint32_t,
		ns *C.uint64_t) C.int {
		return C.gns_cm_view_heavy_hitters(w.v, cf, cv, nc, sf, sv, ns)
	})
}

// Query is CountMin.Query at the last Refresh, safe during inserts.
func (w *View) Query(flow []byte) uint64 {
	if len(flow) != w.keyBytes || len(flow) == 0 {
		return 0
	}
	var out C.uint64_t
	if C.gns_cm_view_query(w.v, (*C.uint8_t)(unsafe.Pointer(&flow[0])), C.uint32_t(len(flow)), 1, &out) != C.GNS_OK {
		return 0
	}
	return uint64(out)
}

// Close releases the snapshot (before the CountMin it views).
func (w *View) Close() { C.gns_cm_view_destroy(w.v) }

// SuperSpread mirrors statistic.SuperSpread (super_spread.go) on one GPU.
type SuperSpread struct {
	h        *C.gns_ss
	flowSize int
	err      error // first insert failure of the period
}

// NewSuperSpread replaces statistic.NewSuperSpread (super_spread.go:129-149). Seeds, the
// HLL master seed and the declared generator's seed are injected (DESIGN.md §2).
func NewSuperSpread(width, depth, threshold, m, size uint32, base, b float64, flowFields, elemFields []string,
	seeds []uint32, hllMaster, rngSeed, maxFlows uint64, device int) (*SuperSpread, error) {
	var p C.gns_ss_params
	p.width, p.depth, p.threshold, p.m, p.size = C.uint32_t(width), C.uint32_t(depth), C.uint32_t(threshold),
		C.uint32_t(m), C.uint32_t(size)
	p.base, p.b = C.double(base), C.double(b)
	p.flow.n_fields = C.uint32_t(len(flowFields))
	for i, f := range flowFields {
		p.flow.fields[i] = fieldIDs[f]
	}
	p.elem.n_fields = C.uint32_t(len(elemFields))
	for i, f := range elemFields {
		p.elem.fields[i] = fieldIDs[f]
	}
	if len(seeds) > 0 {
		p.seeds = (*C.uint32_t)(unsafe.Pointer(&seeds[0]))
	}
	p.hll_master, p.rng_seed, p.device = C.uint64_t(hllMaster), C.uint64_t(rngSeed), C.int(device)
	p.max_flows = C.uint64_t(maxFlows) // 0 -> 4M
	var h *C.gns_ss
	if err := lastErr(C.gns_ss_create(&p, &h)); err != nil {
		return nil, err
	}
	fs := 0
	for _, f := range flowFields {
		fs += map[string]int{"SrcIP": 16, "DstIP": 16, "SrcPort": 2, "DstPort": 2, "Protocol": 1}[f]
	}
	return &SuperSpread{h: h, flowSize: fs}, nil
}

// InsertTuples: PacketInfo batch (task.go:156-169 for a whole batch).
func (s *SuperSpread) InsertTuples(src16, dst16 []byte, sport, dport []uint16, proto []uint8, length []uint32) error {
	n := len(length)
	if n == 0 {
		return nil
	}
	t := C.gns_tuples{
		src16: (*C.uint8_t)(unsafe.Pointer(&src16[0])), dst16: (*C.uint8_t)(unsafe.Pointer(&dst16[0])),
		sport: (*C.uint16_t)(unsafe.Pointer(&sport[0])), dport: (*C.uint16_t)(unsafe.Pointer(&dport[0])),
		proto: (*C.uint8_t)(unsafe.Pointer(&proto[0])), length: (*C.uint32_t)(unsafe.Pointer(&length[0])),
	}
	return lastErr(C.gns_ss_insert_tuples(s.h, &t, C.uint64_t(n), C.GNS_MEM_HOST))
}

// Insert implements statistic.Sketch for one packet (prefer InsertTuples).
func (s *SuperSpread) Insert(flow, elem []byte, size uint32) {
	if len(flow) == 0 {
		return
	}
	var e *C.uint8_t
	if len(elem) > 0 {
		e = (*C.uint8_t)(unsafe.Pointer(&elem[0]))
	}
	sticky(&s.err, lastErr(C.gns_ss_insert_keys(s.h, (*C.uint8_t)(unsafe.Pointer(&flow[0])),
		C.uint32_t(len(flow)), e, C.uint32_t(len(elem)), 1, C.GNS_MEM_HOST)))
}

// Err reports the first insert failure since the last Reset (nil if none).
func (s *SuperSpread) Err() error { return s.err }

// Query implements statistic.Sketch (super_spread.go:238-249).
func (s *SuperSpread) Query(flow []byte) uint64 {
	if len(flow) != s.flowSize || len(flow) == 0 {
		return 1
	}
	var out C.uint64_t
	if C.gns_ss_query(s.h, (*C.uint8_t)(unsafe.Pointer(&flow[0])), C.uint32_t(len(flow)), 1, &out) != C.GNS_OK {
		return 1
	}
	return uint64(out)
}

// QueryBatch: Query for len(keys)/stride flows in one device call.
func (s *SuperSpread) QueryBatch(keys []byte, stride uint32) ([]uint64, error) {
	n := len(keys) / int(stride)
	out := make([]uint64, n+1)
	if n == 0 {
		return out[:0], nil
	}
	err := lastErr(C.gns_ss_query(s.h, (*C.uint8_t)(unsafe.Pointer(&keys[0])), C.uint32_t(stride), C.uint64_t(n),
		(*C.uint64_t)(unsafe.Pointer(&out[0]))))
	return out[:n], err
}

// HeavyHitters implements statistic.Sketch (super_spread.go:254-294): Size is nil.
func (s *SuperSpread) HeavyHitters() statistic.HeavyRecord {
	K := s.flowSize
	capN := 64
	for tries := 0; tries < 8; tries++ {
		fl := make([]byte, capN*K+1)
		v := make([]uint32, capN+1)
		n := C.uint64_t(capN)
		if C.gns_ss_heavy_hitters(s.h, (*C.uint8_t)(unsafe.Pointer(&fl[0])), (*C.uint32_t)(unsafe.Pointer(&v[0])),
			&n) != C.GNS_OK {
			break
		}
		if int(n) > capN { // longer than the buffers: grow and call again
			capN = 2 * int(n)
			continue
		}
		rec := statistic.HeavyRecord{Count: make([]statistic.HeavyCount, 0, int(n))}
		for i := 0; i < int(n); i++ {
			rec.Count = append(rec.Count, statistic.HeavyCount{Flow: append([]byte(nil), fl[i*K:(i+1)*K]...), Count: v[i]})
		}
		return rec
	}
	return statistic.HeavyRecord{Count: []statistic.HeavyCount{}}
}

// Reset implements statistic.Sketch (super_spread.go:297-311).
func (s *SuperSpread) Reset() {
	C.gns_ss_reset(s.h)
	s.err = nil
}

// Close releases the device sketch.
func (s *SuperSpread) Close() { C.gns_ss_destroy(s.h) }

var _ statistic.Sketch = (*SuperSpread)(nil)

// Exact is the device state of one exact task (internal/engine/impl/exact/task.go).
type Exact struct {
	h        *C.gns_ex
	keyBytes int
}

// NewExact replaces exact.New's flow map (task.go:83-103).
func NewExact(keyFields []string, maxFlows uint64, device int) (*Exact, error) {
	var p C.gns_ex_params
	p.key.n_fields = C.uint32_t(len(keyFields))
	kb := 0
	for i, f := range keyFields {
		p.key.fields[i] = fieldIDs[f]
		kb += map[string]int{"SrcIP": 16, "DstIP": 16, "SrcPort": 2, "DstPort": 2, "Protocol": 1}[f]
	}
	p.max_flows, p.device = C.uint64_t(maxFlows), C.int(device)
	var h *C.gns_ex
	if err := lastErr(C.gns_ex_create(&p, &h)); err != nil {
		return nil, err
	}
	return &Exact{h: h, keyBytes: kb}, nil
}

// InsertTuples is ProcessPacket (task.go:124-149) for a batch; ipver[i] = len(IP) == 4 ? 4 : 6.
func (e *Exact) InsertTuples(src16, dst16 []byte, sport, dport []uint16, proto []uint8, length []uint32,
	ipver []uint8, tsNano []int64) error {
	n := len(length)
	if n == 0 {
		return nil
	}
	t := C.gns_tuples{
		src16: (*C.uint8_t)(unsafe.Pointer(&src16[0])), dst16: (*C.uint8_t)(unsafe.Pointer(&dst16[0])),
		sport: (*C.uint16_t)(unsafe.Pointer(&sport[0])), dport: (*C.uint16_t)(unsafe.Pointer(&dport[0])),
		proto: (*C.uint8_t)(unsafe.Pointer(&proto[0])), length: (*C.uint32_t)(unsafe.Pointer(&length[0])),
	}
	return lastErr(C.gns_ex_insert_tuples(e.h, &t, (*C.uint8_t)(unsafe.Pointer(&ipver[0])),
		(*C.int64_t)(unsafe.Pointer(&tsNano[0])), C.uint64_t(n), C.GNS_MEM_HOST))
}

// Query is exact.Task.Query (task.go:298-326).
func (e *Exact) Query(flow []byte) uint64 {
	if len(flow) != e.keyBytes || len(flow) == 0 {
		return 0
	}
	var out C.uint64_t
	if C.gns_ex_query(e.h, (*C.uint8_t)(unsafe.Pointer(&flow[0])), C.uint32_t(len(flow)), 1, &out) != C.GNS_OK {
		return 0
	}
	return uint64(out)
}

// QueryBatch: Query for len(keys)/stride flows in one device call (PacketCount<<32 | ByteCount).
func (e *Exact) QueryBatch(keys []byte, stride uint32) ([]uint64, error) {
	n := len(keys) / int(stride)
	out := make([]uint64, n+1)
	if n == 0 {
		return out[:0], nil
	}
	err := lastErr(C.gns_ex_query(e.h, (*C.uint8_t)(unsafe.Pointer(&keys[0])), C.uint32_t(stride), C.uint64_t(n),
		(*C.uint64_t)(unsafe.Pointer(&out[0]))))
	return out[:n], err
}

// Flows returns the snapshot arrays; the task rebuilds statistic.Flow (Key string via
// net.IP(key[i:i+16]).String(), Fields, StartTime = time.Unix(0, start[i]), ...).
func (e *Exact) Flows() (keys []byte, start, end []int64, pkts, bytes []uint64, err error) {
	var n C.uint64_t
	if err = lastErr(C.gns_ex_snapshot(e.h, nil, nil, nil, nil, nil, &n)); err != nil {
		return
	}
	m := int(n)
	keys = make([]byte, m*e.keyBytes+1)
	start, end = make([]int64, m+1), make([]int64, m+1)
	pkts, bytes = make([]uint64, m+1), make([]uint64, m+1)
	err = lastErr(C.gns_ex_snapshot(e.h, (*C.uint8_t)(unsafe.Pointer(&keys[0])), (*C.int64_t)(unsafe.Pointer(&start[0])),
		(*C.int64_t)(unsafe.Pointer(&end[0])), (*C.uint64_t)(unsafe.Pointer(&pkts[0])),
		(*C.uint64_t)(unsafe.Pointer(&bytes[0])), &n))
	m = int(n)
	return keys[:m*e.keyBytes], start[:m], end[:m], pkts[:m], bytes[:m], err
}

// Reset is exact.Task.Reset (task.go:194-210).
func (e *Exact) Reset() { C.gns_ex_reset(e.h) }

// Close releases the device state.
func (e *Exact) Close() { C.gns_ex_destroy(e.h) }

// ThriftDecoder holds the device buffers one batch of NATS messages decodes into
// (ns-engine's live path: stream_aggregator.go:85 decodes one PacketInfo message
// at a time with probe.UnmarshalPacketInfo, packetcodec.go:97-108; here a whole
// batch is decoded on the GPU into the engine's pre-parsed records).
type ThriftDecoder struct {
	rec, wirelen, ts unsafe.Pointer
	capacity         int
	device           int
}

// NewThriftDecoder allocates room for `capacity` messages per batch on `device`.
func NewThriftDecoder(capacity, device int) (*ThriftDecoder, error) {
	d := &ThriftDecoder{capacity: capacity, device: device}
	for _, b := range []struct {
		p     *unsafe.Pointer
		bytes int
	}{{&d.rec, 64 * capacity}, {&d.wirelen, 4 * capacity}, {&d.ts, 8 * capacity}} {
		if err := lastErr(C.gns_device_alloc(C.uint64_t(b.bytes), C.int(device), b.p)); err != nil {
			d.Close()
			return nil, err
		}
	}
	return d, nil
}

// decode turns msgs (back to back; offs[i] = start of message i, offs[n] = len(msgs))
// into device records; bad counts the messages the reference would reject.
func (d *ThriftDecoder) decode(msgs []byte, offs []uint64) (n int, bad uint64, err error) {
	n = len(offs) - 1
	if n <= 0 {
		return 0, 0, nil
	}
	if n > d.capacity {
		return 0, 0, fmt.Errorf("sketchgpu: %d messages for a %d-message decoder", n, d.capacity)
	}
	var nb C.uint64_t
	err = lastErr(C.gns_thrift_decode((*C.uint8_t)(unsafe.Pointer(&msgs[0])), C.uint64_t(len(msgs)),
		(*C.uint64_t)(unsafe.Pointer(&offs[0])), C.uint64_t(n), (*C.uint8_t)(d.rec), (*C.uint32_t)(d.wirelen),
		(*C.int64_t)(d.ts), &nb, C.GNS_MEM_HOST, C.int(d.device)))
	return n, uint64(nb), err
}

// Close frees the device buffers.
func (d *ThriftDecoder) Close() {
	for _, p := range []unsafe.Pointer{d.rec, d.wirelen, d.ts} {
		if p != nil {
			C.gns_device_free(p, C.int(d.device))
		}
	}
	d.rec, d.wirelen, d.ts = nil, nil, nil
}

// InsertThriftBatch decodes a batch of PacketInfo messages on the GPU and inserts
// the packets (ProcessPacket for each message, task.go:156-169).  It returns once
// the decoder's buffers are free again.
func (c *CountMin) InsertThriftBatch(d *ThriftDecoder, msgs []byte, offs []uint64) (bad uint64, err error) {
	n, bad, err := d.decode(msgs, offs)
	if err != nil || n == 0 {
		return bad, err
	}
	if err = lastErr(C.gns_cm_insert_headers(c.h, (*C.uint8_t)(d.rec), (*C.uint32_t)(d.wirelen), C.uint64_t(n),
		C.GNS_MEM_DEVICE)); err != nil {
		return bad, err
	}
	return bad, lastErr(C.gns_cm_flush(c.h))
}

// InsertThriftBatch for SuperSpread (see CountMin.InsertThriftBatch).
func (s *SuperSpread) InsertThriftBatch(d *ThriftDecoder, msgs []byte, offs []uint64) (bad uint64, err error) {
	n, bad, err := d.decode(msgs, offs)
	if err != nil || n == 0 {
		return bad, err
	}
	if err = lastErr(C.gns_ss_insert_headers(s.h, (*C.uint8_t)(d.rec), (*C.uint32_t)(d.wirelen), C.uint64_t(n),
		C.GNS_MEM_DEVICE)); err != nil {
		return bad, err
	}
	return bad, lastErr(C.gns_ss_flush(s.h))
}

// InsertThriftBatch for the exact aggregator (the messages' TimestampUnixNano kept).
func (e *Exact) InsertThriftBatch(d *ThriftDecoder, msgs []byte, offs []uint64) (bad uint64, err error) {
	n, bad, err := d.decode(msgs, offs)
	if err != nil || n == 0 {
		return bad, err
	}
	if err = lastErr(C.gns_ex_insert_headers(e.h, (*C.uint8_t)(d.rec), (*C.uint32_t)(d.wirelen), (*C.int64_t)(d.ts),
		C.uint64_t(n), C.GNS_MEM_DEVICE)); err != nil {
		return bad, err
	}
	return bad, lastErr(C.gns_ex_flush(e.h))
}
