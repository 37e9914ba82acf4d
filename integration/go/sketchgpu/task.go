// GPUTask: the model.Task (internal/model/task.go:6-15) a maintainer registers
// next to the reference's "sketch" aggregator.  It has the reference sketch.Task's
// surface (internal/engine/impl/sketch/task.go:91-243) -- same SketchTaskDef keys,
// same Snapshot payload (statistic.HeavyRecord), same Query / Fields /
// DecodeFlowFunc / AlerterMsg -- but ProcessPacket appends the packet to a host
// batch instead of inserting it.  The Manager's workers (manager.go:218-244) keep
// calling ProcessPacket concurrently, as they call the reference's lock-free
// ProcessPacket (task.go:156-169):
//   - under the task's mutex a worker only appends to the current batch and, when
//     it is full, hands it to the submitter (a channel send) and takes an empty
//     one from the free list -- no device work is done under the lock;
//   - ONE submitter goroutine per task owns the device handle: it inserts the full
//     batches in the order they were handed over (gns_{cm,ss}_insert_tuples, where
//     EncodeFlow, task.go:265-300, and the d seeded MurmurHash3 updates run), so
//     the stream the GPU applies is the order in which packets reached the batch
//     (the reference's workers race on the buckets instead, SURVEY.md §0.2);
//   - Query / Snapshot / Reset hand over the pending packets, then run on the
//     submitter behind every batch handed over before them, and wait for it: they
//     see every packet processed before the call, and the handle is only ever
//     used from one goroutine (include/gns_sketch.h rules).
// The workers stall only when the GPU is `Inflight` batches behind.
//
// Registration (the "sketch_gpu" aggregator type, configs' aggregator.types):
//
//	import _ "Go2NetSpectra/integration/go/sketchgpu"   // in manager.go, beside the sketch import
//
// Not compiled in the build container (no Go toolchain there); tests/test_gputask_replay_gpu.py
// replays this file's call sequence through the C ABI (integration/c/gputask_replay.c).
package sketchgpu

import (
	"fmt"
	"log"
	"strings"
	"sync"
	"time"

	"Go2NetSpectra/internal/config"
	"Go2NetSpectra/internal/engine/impl/sketch"
	"Go2NetSpectra/internal/engine/impl/sketch/statistic"
	"Go2NetSpectra/internal/factory"
	"Go2NetSpectra/internal/model"
)

// BatchPackets is the host batch handed to the GPU in one insert.
var BatchPackets = 1 << 16

// Inflight is the number of full batches that may wait for the submitter before
// ProcessPacket blocks (host memory: Inflight+2 batches per task).
var Inflight = 2

// Device is the HIP device ordinal the tasks of this process use.
var Device = 0

func init() {
	factory.RegisterAggregator("sketch_gpu", newTaskGroup)
}

// newTaskGroup is the TaskFactory (task_factory.go:18) of "sketch_gpu": the
// sketch aggregator's writers (task.go:22-56) and one GPUTask per SketchTaskDef.
func newTaskGroup(cfg *config.Config) (*factory.TaskGroup, error) {
	sketchCfg := cfg.Aggregator.Sketch
	writers := make([]model.Writer, 0, len(sketchCfg.Writers))
	for _, wd := range sketchCfg.Writers {
		if !wd.Enabled {
			continue
		}
		interval, err := time.ParseDuration(wd.SnapshotInterval)
		if err != nil {
			log.Printf("sketch_gpu: invalid snapshot_interval for writer '%s': %v, skipping", wd.Type, err)
			continue
		}
		switch wd.Type {
		case "text":
			writers = append(writers, sketch.NewTextWriter(wd.Text.RootPath, interval))
		case "clickhouse":
			w, err := sketch.NewClickHouseWriter(wd.ClickHouse, interval)
			if err != nil {
				log.Printf("sketch_gpu: clickhouse writer: %v, skipping", err)
				continue
			}
			writers = append(writers, w)
		default:
			log.Printf("sketch_gpu: unknown writer type '%s', skipping", wd.Type)
		}
	}
	tasks := make([]model.Task, 0, len(sketchCfg.Tasks))
	for _, tc := range sketchCfg.Tasks {
		t, err := NewGPUTask(tc)
		if err != nil {
			return nil, fmt.Errorf("task %s: %w", tc.Name, err)
		}
		tasks = append(tasks, t)
	}
	return &factory.TaskGroup{Tasks: tasks, Writers: writers}, nil
}

func fieldBytes(fields []string) uint32 {
	n := uint32(0)
	for _, f := range fields {
		n += map[string]uint32{"SrcIP": 16, "DstIP": 16, "SrcPort": 2, "DstPort": 2, "Protocol": 1}[f]
	}
	return n
}

// pktBatch is one host batch of PacketInfo as SoA (the layout gns_tuples reads).
type pktBatch struct {
	src16, dst16 []byte
	sport, dport []uint16
	proto        []uint8
	length       []uint32
}

func newPktBatch(b int) *pktBatch {
	return &pktBatch{src16: make([]byte, 0, 16*b), dst16: make([]byte, 0, 16*b), sport: make([]uint16, 0, b),
		dport: make([]uint16, 0, b), proto: make([]uint8, 0, b), length: make([]uint32, 0, b)}
}

func (b *pktBatch) clear() {
	b.src16, b.dst16 = b.src16[:0], b.dst16[:0]
	b.sport, b.dport, b.proto, b.length = b.sport[:0], b.dport[:0], b.proto[:0], b.length[:0]
}

// job is one unit of the submitter's queue: a batch to insert, or a call on the
// handle (fn) whose caller waits on done.
type job struct {
	b    *pktBatch
	fn   func()
	done chan struct{}
}

// GPUTask implements model.Task on a GPU Count-Min (skt_type 0) or SuperSpread (1).
type GPUTask struct {
	name       string
	flowFields []string
	elemFields []string
	cm         *CountMin
	ss         *SuperSpread

	mu   sync.Mutex // guards cur and the order of sends on work
	cur  *pktBatch
	work chan job       // to the submitter, in hand-over order
	free chan *pktBatch // empty batches back from the submitter
	quit chan struct{}  // closed by Close after the last job

	errMu sync.Mutex
	err   error // first failed insert of the period
}

// NewGPUTask replaces sketch.New (task.go:106-138).  Row seeds: NewCountMin's
// rand.Uint32 draws (count_min.go:61-64) become the engine's default seed stream.
func NewGPUTask(cfg config.SketchTaskDef) (*GPUTask, error) {
	t := &GPUTask{name: cfg.Name, flowFields: cfg.FlowFields, elemFields: cfg.ElementFields}
	flowSize := fieldBytes(cfg.FlowFields)
	var err error
	switch cfg.SketchType {
	case 0:
		t.cm, err = NewCountMin(cfg.Width, cfg.Depth, cfg.SizeThreshold, cfg.CountThreshold, cfg.FlowFields, flowSize,
			nil, 0, Device)
	case 1:
		t.ss, err = NewSuperSpread(cfg.Width, cfg.Depth, cfg.CountThreshold, cfg.M, cfg.Size, cfg.Base, cfg.B,
			cfg.FlowFields, cfg.ElementFields, nil, uint64(time.Now().UnixNano()), uint64(time.Now().UnixNano())^0x9E3779B97F4A7C15, 0, Device)
	default:
		log.Fatalf("Unknown sketch type: %d for task %s", cfg.SketchType, cfg.Name) // task.go:126-127
	}
	if err != nil {
		return nil, err
	}
	t.cur = newPktBatch(BatchPackets)
	t.work = make(chan job, Inflight)
	t.free = make(chan *pktBatch, Inflight+1)
	for i := 0; i < Inflight+1; i++ {
		t.free <- newPktBatch(BatchPackets)
	}
	t.quit = make(chan struct{})
	go t.submitter()
	return t, nil
}

// submitter owns the device handle: batches and calls in hand-over order.
func (t *GPUTask) submitter() {
	defer close(t.quit)
	for j := range t.work {
		if j.b != nil {
			t.insert(j.b)
			j.b.clear()
			t.free <- j.b
		}
		if j.fn != nil {
			j.fn()
		}
		if j.done != nil {
			close(j.done)
		}
	}
}

// insert submits one batch.  The reference logs a packet it cannot insert and
// goes on (task.go:162-166); a failed batch is logged the same way and kept for Err().
func (t *GPUTask) insert(b *pktBatch) {
	var err error
	if t.cm != nil {
		err = t.cm.InsertTuples(b.src16, b.dst16, b.sport, b.dport, b.proto, b.length)
	} else {
		err = t.ss.InsertTuples(b.src16, b.dst16, b.sport, b.dport, b.proto, b.length)
	}
	if err != nil {
		t.errMu.Lock()
		if t.err == nil {
			t.err = err
		}
		t.errMu.Unlock()
		log.Printf("Error inserting a batch for task '%s': %v", t.name, err)
	}
}

// ProcessPacket (task.go:156-169) for the GPU: the PacketInfo joins the batch;
// EncodeFlow and the sketch update run on the device when the batch is submitted.
func (t *GPUTask) ProcessPacket(p *model.PacketInfo) {
	var s, d [16]byte
	copy(s[:], p.FiveTuple.SrcIP) // 4-byte IPv4 left-aligned, zero padded (task.go:281-286)
	copy(d[:], p.FiveTuple.DstIP)
	t.mu.Lock()
	b := t.cur
	b.src16 = append(b.src16, s[:]...)
	b.dst16 = append(b.dst16, d[:]...)
	b.sport = append(b.sport, p.FiveTuple.SrcPort)
	b.dport = append(b.dport, p.FiveTuple.DstPort)
	b.proto = append(b.proto, p.FiveTuple.Protocol)
	b.length = append(b.length, uint32(p.Length)) // task.go:168
	if len(b.length) >= BatchPackets {
		t.handOverLocked()
	}
	t.mu.Unlock()
}

// handOverLocked queues the current batch (mutex held, so batches keep their order)
// and starts an empty one.
func (t *GPUTask) handOverLocked() {
	if len(t.cur.length) == 0 {
		return
	}
	t.work <- job{b: t.cur}
	t.cur = <-t.free
}

// call runs fn on the submitter after every packet processed so far, and waits.
func (t *GPUTask) call(fn func()) {
	done := make(chan struct{})
	t.mu.Lock()
	t.handOverLocked()
	t.work <- job{fn: fn, done: done}
	t.mu.Unlock()
	<-done
}

// Flush submits the pending batch and waits until the GPU has it (e.g. at the end of a capture).
func (t *GPUTask) Flush() { t.call(nil) }

// Close drains the queue and stops the submitter; the task is unusable afterwards.
func (t *GPUTask) Close() {
	t.Flush()
	t.mu.Lock()
	close(t.work)
	t.mu.Unlock()
	<-t.quit
}

// Err reports the first failed batch since the last Reset.
func (t *GPUTask) Err() error {
	t.errMu.Lock()
	defer t.errMu.Unlock()
	return t.err
}

func (t *GPUTask) Name() string       { return t.name }
func (t *GPUTask) Fields() []string   { return t.flowFields }
func (t *GPUTask) sk() statistic.Sketch {
	if t.cm != nil {
		return t.cm
	}
	return t.ss
}

// Query (task.go:171-174) of the state after every packet processed so far.
func (t *GPUTask) Query(flow []byte) uint64 {
	var v uint64
	t.call(func() { v = t.sk().Query(flow) })
	return v
}

// Snapshot (task.go:176-179): the heavy hitters of every packet processed so far.
func (t *GPUTask) Snapshot() interface{} {
	var rec statistic.HeavyRecord
	t.call(func() { rec = t.sk().HeavyHitters() })
	return rec
}

// Reset (task.go:181-184): the packets processed before the call belong to the period that ends.
func (t *GPUTask) Reset() {
	t.call(func() {
		t.sk().Reset()
		t.errMu.Lock()
		t.err = nil
		t.errMu.Unlock()
	})
}

// DecodeFlowFunc (task.go:150-153): the reference's DecodeFlow (it reads no task state).
func (t *GPUTask) DecodeFlowFunc() func(flow []byte, fields []string) string {
	return (&sketch.Task{}).DecodeFlow
}

// AlerterMsg (task.go:186-243) over this task's Snapshot, same rules and markup.
func (t *GPUTask) AlerterMsg(rules []config.AlerterRule) string {
	snap, ok := t.Snapshot().(statistic.HeavyRecord)
	if !ok {
		return ""
	}
	decode := t.DecodeFlowFunc()
	var msgs []string
	for _, rule := range rules {
		if rule.TaskName != t.name {
			continue
		}
		var rows []string
		switch rule.Metric {
		case "heavy_hitter_count":
			for _, h := range snap.Count {
				if compare(float64(h.Count), rule.Threshold, rule.Operator) {
					rows = append(rows, fmt.Sprintf("<tr><td><code>%s</code></td><td>%d</td></tr>", decode(h.Flow, t.flowFields), h.Count))
				}
			}
		case "heavy_hitter_size":
			for _, h := range snap.Size {
				if compare(float64(h.Size), rule.Threshold, rule.Operator) {
					rows = append(rows, fmt.Sprintf("<tr><td><code>%s</code></td><td>%d bytes</td></tr>", decode(h.Flow, t.flowFields), h.Size))
				}
			}
		case "super_spreader_spread":
			if snap.Size == nil {
				for _, h := range snap.Count {
					if compare(float64(h.Count), rule.Threshold, rule.Operator) {
						rows = append(rows, fmt.Sprintf("<tr><td><code>%s</code></td><td>%d</td></tr>", decode(h.Flow, t.flowFields), h.Count))
					}
				}
			}
		}
		if len(rows) == 0 {
			continue
		}
		table := fmt.Sprintf("<table border=\"1\" cellpadding=\"5\" cellspacing=\"0\">"+
			"<tr><th>Flow/Source</th><th>Value</th></tr>%s</table>", strings.Join(rows, ""))
		msgs = append(msgs, fmt.Sprintf("<h3>Alert: %s</h3><ul><li><b>Task:</b> <code>%s</code></li>"+
			"<li><b>Metric:</b> <code>%s</code></li><li><b>Condition:</b> <code>%s %.2f</code></li></ul>"+
			"<p><b>Triggering Items:</b></p>%s", rule.Name, rule.TaskName, rule.Metric, rule.Operator, rule.Threshold, table))
	}
	return strings.Join(msgs, "<br><hr><br>")
}

// compare restates task.go's check (unexported there).
func compare(v, threshold float64, op string) bool {
	switch op {
	case ">":
		return v > threshold
	case "<":
		return v < threshold
	case "=":
		return v == threshold
	case ">=":
		return v >= threshold
	case "<=":
		return v <= threshold
	}
	log.Printf("Warning: unknown operator '%s' in alerter rule", op)
	return false
}

var _ model.Task = (*GPUTask)(nil)
