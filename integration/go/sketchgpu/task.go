package sketchgpu

// GPUTask: the model.Task (internal/model/task.go:6-15) a maintainer registers
// next to the reference's "sketch" aggregator.  It has the reference sketch.Task's
// surface (internal/engine/impl/sketch/task.go:91-243) -- same SketchTaskDef keys,
// same Snapshot payload (statistic.HeavyRecord), same Query / Fields /
// DecodeFlowFunc / AlerterMsg -- but ProcessPacket appends the packet to a host
// batch instead of inserting it: every `BatchPackets` packets (and before every
// Snapshot, Query and Reset) the batch goes to the GPU in one
// gns_{cm,ss}_insert_tuples call, where EncodeFlow (task.go:265-300) and the d
// seeded MurmurHash3 updates run.  The Manager's workers (manager.go:218-244)
// keep calling ProcessPacket concurrently; the batch is filled under a mutex, so
// the stream order the GPU applies is the order in which packets reached it (the
// reference's workers race on the buckets, SURVEY.md §0.2).
//
// Registration (the "sketch_gpu" aggregator type, configs' aggregator.types):
//
//	import _ "Go2NetSpectra/integration/go/sketchgpu"   // in manager.go, beside the sketch import
//
// Not compiled in the build container (no Go toolchain there).

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

// GPUTask implements model.Task on a GPU Count-Min (skt_type 0) or SuperSpread (1).
type GPUTask struct {
	name       string
	flowFields []string
	elemFields []string
	cm         *CountMin
	ss         *SuperSpread

	mu     sync.Mutex
	src16  []byte
	dst16  []byte
	sport  []uint16
	dport  []uint16
	proto  []uint8
	length []uint32
	err    error // first failed insert of the period
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
	t.reserve()
	return t, nil
}

func (t *GPUTask) reserve() {
	b := BatchPackets
	t.src16, t.dst16 = make([]byte, 0, 16*b), make([]byte, 0, 16*b)
	t.sport, t.dport = make([]uint16, 0, b), make([]uint16, 0, b)
	t.proto, t.length = make([]uint8, 0, b), make([]uint32, 0, b)
}

// ProcessPacket (task.go:156-169) for the GPU: the PacketInfo joins the batch;
// EncodeFlow and the sketch update run on the device at the next flush.
func (t *GPUTask) ProcessPacket(p *model.PacketInfo) {
	var s, d [16]byte
	copy(s[:], p.FiveTuple.SrcIP) // 4-byte IPv4 left-aligned, zero padded (task.go:281-286)
	copy(d[:], p.FiveTuple.DstIP)
	t.mu.Lock()
	t.src16 = append(t.src16, s[:]...)
	t.dst16 = append(t.dst16, d[:]...)
	t.sport = append(t.sport, p.FiveTuple.SrcPort)
	t.dport = append(t.dport, p.FiveTuple.DstPort)
	t.proto = append(t.proto, p.FiveTuple.Protocol)
	t.length = append(t.length, uint32(p.Length)) // task.go:168
	if len(t.length) >= BatchPackets {
		t.flushLocked()
	}
	t.mu.Unlock()
}

// flushLocked submits the pending batch (mutex held).  The reference logs a
// packet it cannot insert and goes on (task.go:162-166); a failed batch is
// logged the same way and kept for Err().
func (t *GPUTask) flushLocked() {
	if len(t.length) == 0 {
		return
	}
	var err error
	if t.cm != nil {
		err = t.cm.InsertTuples(t.src16, t.dst16, t.sport, t.dport, t.proto, t.length)
	} else {
		err = t.ss.InsertTuples(t.src16, t.dst16, t.sport, t.dport, t.proto, t.length)
	}
	if err != nil {
		if t.err == nil {
			t.err = err
		}
		log.Printf("Error inserting a batch for task '%s': %v", t.name, err)
	}
	t.src16, t.dst16 = t.src16[:0], t.dst16[:0]
	t.sport, t.dport, t.proto, t.length = t.sport[:0], t.dport[:0], t.proto[:0], t.length[:0]
}

// Flush submits the pending batch now (e.g. at the end of a capture).
func (t *GPUTask) Flush() {
	t.mu.Lock()
	t.flushLocked()
	t.mu.Unlock()
}

// Err reports the first failed batch since the last Reset.
func (t *GPUTask) Err() error {
	t.mu.Lock()
	defer t.mu.Unlock()
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
	t.mu.Lock()
	defer t.mu.Unlock()
	t.flushLocked()
	return t.sk().Query(flow)
}

// Snapshot (task.go:176-179): the heavy hitters of every packet processed so far.
func (t *GPUTask) Snapshot() interface{} {
	t.mu.Lock()
	defer t.mu.Unlock()
	t.flushLocked()
	return t.sk().HeavyHitters()
}

// Reset (task.go:181-184): the pending batch belongs to the period that ends.
func (t *GPUTask) Reset() {
	t.mu.Lock()
	defer t.mu.Unlock()
	t.flushLocked()
	t.sk().Reset()
	t.err = nil
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
