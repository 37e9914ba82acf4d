/*
 * gns_sketch.h -- C ABI of the MI355X sketch engine (libgns_sketch.so).
 *
 * Drop-in boundary for Go2NetSpectra's sketch hot path.  Each entry point names
 * the reference interface it replaces (paths relative to the reference repo):
 *
 *   statistic.Sketch.Insert(flow, elem, size)  internal/engine/impl/sketch/statistic/sketch.go:6
 *       -> gns_cm_insert_keys / gns_ss_insert_keys           (batched, stream-ordered)
 *   sketch.Task.ProcessPacket(*PacketInfo)     internal/engine/impl/sketch/task.go:156-169
 *       -> gns_cm_insert_tuples / gns_ss_insert_tuples       (EncodeFlow fused on device)
 *   pcap.Reader.ReadPackets + ParsePacketInto  pkg/pcap/reader.go:35-49, internal/protocol/parser.go:23-67
 *       -> gns_cm_insert_headers / gns_ss_insert_headers     (64-byte records, parse fused)
 *   statistic.Sketch.Query(flow)               sketch.go:7; count_min.go:160-174; super_spread.go:238-249
 *       -> gns_cm_query / gns_ss_query
 *   statistic.Sketch.HeavyHitters()            sketch.go:8; count_min.go:178-247; super_spread.go:254-294
 *       -> gns_cm_heavy_hitters / gns_ss_heavy_hitters
 *   statistic.Sketch.Reset()                   sketch.go:9; count_min.go:249-265; super_spread.go:297-311
 *       -> gns_cm_reset / gns_ss_reset
 *   statistic.NewCountMin / NewSuperSpread     count_min.go:47-90; super_spread.go:127-179
 *       -> gns_cm_create / gns_ss_create (seeds injected, see below)
 *
 * Rules:
 *   - Every call returns GNS_OK (0) or a negative gns_status; gns_last_error()
 *     returns the thread-local message of the last failure.
 *   - Calls on one handle must be serialized by the caller (one goroutine per
 *     handle).  Inserts are applied in call order, packets in array order:
 *     the device state equals the reference sketch fed the same stream by ONE
 *     worker (num_workers: 1) with the same seeds.
 *   - Pointers flagged GNS_MEM_HOST are read before the call returns (the
 *     caller keeps ownership).  GNS_MEM_DEVICE pointers must be device memory
 *     of the handle's device and stay valid until gns_*_flush() returns.
 *   - Flow keys are the reference EncodeFlow bytes (task.go:279-300): IP slots
 *     of 16 bytes with IPv4 left-aligned and zero padded, ports big-endian,
 *     protocol one byte; key_bytes <= 37 (task.go:74).
 *   - Flow dictionary (fingerprints are dense flow ids): the
 *     reference's buckets hold key bytes (count_min.go:66-81), so Insert has no
 *     failure mode whatever the traffic (count_min.go:94-157).  Here a bucket
 *     names a dictionary slot; between device batches the sketches reclaim the
 *     flows no bucket names any more and the table DOUBLES while the live flows
 *     exceed a quarter of it (live ids are at most 2*depth*width for Count-Min,
 *     depth*width for SuperSpread).  A batch whose new flows overflow the table
 *     is not applied: the dictionary is rebuilt and the batch re-run (in
 *     halves; a piece of 16K packets that still does not fit grows the table).
 *     max_flows is only the INITIAL capacity.  GNS_E_FULL is left only for a
 *     table of 2^30 slots (64 GB of 64-byte records) that cannot take one 16K
 *     piece next to its live flows -- beyond any sketch with depth*width <=
 *     2^27 -- and then holds until gns_*_reset() (the period reset,
 *     manager.go:179-193).  The exact aggregator's table grows the same way.
 *   - Sizes >= 2^16-1 take an overflow side table that grows with the batch
 *     (no per-batch limit).
 *   - Deviations from NewCountMin (count_min.go:47-60), which accepts any
 *     geometry: depth <= 8 (GNS_E_ARG) and width < 2^25 (GNS_E_RANGE; at depth
 *     8 also width <= 2^25 / bins limit, see gns_cm_create's message).  Batches
 *     are capped at 2^31 / depth packets (longer inserts are split).
  */
#ifndef GNS_SKETCH_H
#define GNS_SKETCH_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum gns_status {
    GNS_OK = 0,
    GNS_E_ARG = -1,    /* bad argument (log.Fatalf / panic sites in the reference) */
    GNS_E_HIP = -2,    /* HIP runtime error */
    GNS_E_OOM = -3,    /* device allocation failed */
    GNS_E_FULL = -4,   /* flow dictionary at its 2^30-slot limit (see the rules above) */
    GNS_E_RANGE = -5,  /* geometry beyond a documented limit (see message) */
    GNS_E_NODEV = -6   /* no usable HIP device */
} gns_status;

typedef enum gns_mem { GNS_MEM_HOST = 0, GNS_MEM_DEVICE = 1 } gns_mem;

/* gns_*_set_timing(h, GNS_TIMING_MASK | stage bits): time only those stages */
#define GNS_TIMING_MASK 0x100

/* task.go:279-300 field names -> ids; fieldByteSize task.go:327-338 */
typedef enum gns_field {
    GNS_F_NONE = 0, GNS_F_SRCIP = 1, GNS_F_DSTIP = 2, GNS_F_SRCPORT = 3, GNS_F_DSTPORT = 4,
    GNS_F_PROTO = 5
} gns_field;

typedef struct gns_layout {
    uint32_t n_fields;
    uint8_t fields[8]; /* gns_field, in configured order (SketchTaskDef.FlowFields) */
} gns_layout;

/* Pre-parsed packets: model.PacketInfo (internal/model/packet.go:9-22) as SoA.
 * src16/dst16 hold the 16-byte slots exactly as EncodeFlow lays them out. */
typedef struct gns_tuples {
    const uint8_t *src16;   /* n*16 */
    const uint8_t *dst16;   /* n*16 */
    const uint16_t *sport;  /* n */
    const uint16_t *dport;  /* n */
    const uint8_t *proto;   /* n */
    const uint32_t *length; /* n, uint32(PacketInfo.Length) (task.go:168) */
} gns_tuples;

/* ------------------------------------------------------------------ */
/* Count-Min (count_min.go)                                           */
/* ------------------------------------------------------------------ */
typedef struct gns_cm gns_cm;

typedef struct gns_cm_params {
    uint32_t width, depth;                    /* 0 -> 2^20 / 3 (count_min.go:48-53) */
    uint32_t size_threshold, count_threshold; /* 0 -> 512 KiB / 512 (count_min.go:54-59) */
    gns_layout flow;                          /* flow key layout (for tuples/headers input) */
    uint32_t key_bytes;                       /* FS; must equal the layout's byte size when
                                                 n_fields > 0; used alone for keys input */
    const uint32_t *seeds;                    /* depth row seeds (count_min.go:61-64 draws
                                                 them with rand.Uint32; here injected).
                                                 NULL -> splitmix64(0x9747B28C) stream */
    uint64_t max_flows;                       /* INITIAL flow dictionary capacity (it grows with
                                                 the live flows; dead flows are reclaimed); 0 -> 4M */
    uint64_t batch_packets;                   /* device batch size; 0 -> 16M packets */
    int device;                               /* HIP device ordinal */
    uint32_t bucket_lo, bucket_hi;            /* bucket-range slice (SURVEY §8e exact global
                                                 mode): only updates whose row bucket lies in
                                                 [bucket_lo, bucket_hi) are applied, so G handles
                                                 fed the same stream with disjoint ranges hold,
                                                 between them, exactly the state of one handle.
                                                 0, 0 -> the whole row */
} gns_cm_params;

int gns_cm_create(const gns_cm_params *p, gns_cm **out);
int gns_cm_destroy(gns_cm *cm);
/* statistic.Sketch.Insert batch: keys[n*stride] (first key_bytes used), sizes[n] */
int gns_cm_insert_keys(gns_cm *cm, const uint8_t *keys, uint32_t stride, const uint32_t *sizes,
                       uint64_t n, gns_mem where);
/* Task.ProcessPacket batch over pre-parsed PacketInfo */
int gns_cm_insert_tuples(gns_cm *cm, const gns_tuples *t, uint64_t n, gns_mem where);
/* fused parse: hdr[n*64] = first 64 bytes of each frame (zero padded),
 * wirelen[n] = capture orig_len (= PacketInfo.Length, parser.go:30-33).
 * Records outside the device parser's subset (gns_device.cuh parse_record:
 * Ethernet II, <= 2 VLAN tags, IPv4 without options, IPv6 without extension
 * headers, TCP/UDP, no tunnels) are skipped and counted (gns_cm_stats [2]);
 * the host packer (gns_pack_pcap) never emits them: it decodes such frames
 * itself (gns_frame_record). */
int gns_cm_insert_headers(gns_cm *cm, const uint8_t *hdr, const uint32_t *wirelen, uint64_t n,
                          gns_mem where);
/* Compact records (the PCIe-bound host-inclusive path): rec16[n*16]
 * = the canonical tuple the device parser derives from a 64-byte record, in 16
 * bytes + wirelen[n] (20 B/packet instead of 68):
 *   word 0 IPv4 source, word 1 IPv4 destination (the left-aligned slots' first
 *   4 bytes), word 2 ports (big-endian bytes), word 3 = protocol | class << 8 |
 *   destination IP version << 16 | source IP version << 24;
 *   class 0 = that tuple, 1 = no IP layer (not counted, parser.go:48-49),
 *   2 = escape: word 0 indexes side64[n_side*64], a 64-byte record parsed as
 *   gns_cm_insert_headers parses it (IPv6 tuples, unsupported shapes).
 * The insert equals gns_cm_insert_headers of the records the compact form was
 * made from.  Producers: gns_pack_pcap_compact (host), gns_compact_headers (device).
 * wirelen == NULL: the 16-byte form (16 B/packet over the bus): word 3 bits 16..31
 * hold the wire length instead of the IP versions, a class-0 record is an IPv4
 * tuple both ways (any other tuple escapes to side64), so no wire lengths above
 * 65535; producers gns_pack_pcap_compact16, gns_compact_headers16. */
int gns_cm_insert_compact(gns_cm *cm, const uint8_t *rec16, const uint32_t *wirelen, uint64_t n,
                          const uint8_t *side64, uint64_t n_side, gns_mem where);
int gns_cm_flush(gns_cm *cm);
/* out[i] = count<<32 | size, count_min.go:160-174 */
int gns_cm_query(gns_cm *cm, const uint8_t *keys, uint32_t stride, uint64_t n, uint64_t *out);
/* gns_cm_query with keys and out in DEVICE memory of the handle's GPU (out 8-byte
 * aligned): the owner-routed query path keeps keys and answers on the GPU between
 * its all-to-alls.  The keys must be complete when called; returns once out is written. */
int gns_cm_query_device(gns_cm *cm, const uint8_t *keys, uint32_t stride, uint64_t n, uint64_t *out);
/* HeavyHitters, count_min.go:178-247.  Lists are sorted value-descending with
 * ties broken by flow bytes ascending (the reference leaves ties unordered).
 * On input *n_count / *n_size hold the capacities (entries); on output the
 * full list lengths (call again with larger buffers if they exceed the
 * capacities).  flows_* are n*key_bytes. */
int gns_cm_heavy_hitters(gns_cm *cm, uint8_t *count_flows, uint32_t *counts, uint64_t *n_count,
                         uint8_t *size_flows, uint32_t *sizes, uint64_t *n_size);
/* HeavyHitters into DEVICE memory, for the multi-GPU window exchange (the lists
 * stay on the device through the all-gather and the merge): packed rows
 * [flow (key_bytes) | value (u32, little-endian)], in the order above;
 * *n_count / *n_size in/out as for gns_cm_heavy_hitters (capacities in rows; a
 * list longer than its buffer is reported and not written). */
int gns_cm_heavy_rows(gns_cm *cm, uint8_t *count_rows, uint64_t *n_count, uint8_t *size_rows, uint64_t *n_size);
/* The canonical order (value desc, flow bytes asc) of n DEVICE rows of the form
 * above -- the union of flow-disjoint per-shard lists after an all-gather
 *  -- written to out_rows (device).  Runs on the device's null
 * stream, ordered after the caller's earlier work on it; returns when done. */
int gns_hh_order_rows(const uint8_t *rows, uint32_t key_bytes, uint64_t n, uint8_t *out_rows, int device);
int gns_cm_reset(gns_cm *cm);
/* Full state for parity: C/S [depth*width], FPc/FPs [depth*width*key_bytes]
 * (any pointer may be NULL). */
int gns_cm_export_state(gns_cm *cm, uint32_t *C, uint32_t *S, uint8_t *FPc, uint8_t *FPs);
/* stats[0]=packets inserted, [1]=records dropped (not IP), [2]=records outside
 * the fast-parse subset, [3]=distinct flows in the dictionary */
int gns_cm_stats(gns_cm *cm, uint64_t stats[4]);
/* Per-stage device time (ms, HIP events on the handle's stream), accumulated
 * since the last call with reset != 0.  Stages: 0 extract, 1 resolve, 2 scan,
 * 3 scatter, 4 apply, 5 total insert, 6 hot-bucket aggregate/decide/fallback,
 * 7 hot-bucket designation.  Enabled by gns_cm_set_timing(cm, 1) (every stage) or
 * gns_cm_set_timing(cm, GNS_TIMING_MASK | bits) (only the stages whose bits are set: each
 * timed stage puts two events into the batch's stream). */
/* raw engine counters: [0] inserted, [1] dropped, [2] unsupported, [3] dictionary
 * full, [4] size-overflow full, [5] tile updates replayed sequentially,
 * [6] tile chunks, [7] tile chunks with a replay */
int gns_cm_counters(gns_cm *cm, uint64_t out[8]);
/* flow dictionary: [0] reclaims, [1] dead flows dropped, [2] live flows after the
 * last reclaim, [3] claimed slots now, [4] reclaim time (us, host clock incl. the
 * rebuild's device work), [5] batches re-run after a dictionary overflow,
 * [6] dictionary slots now, [7] table growths */
int gns_cm_dict_stats(gns_cm *cm, uint64_t out[8]);
/* reclaim now (e.g. at a window boundary; inserts also reclaim on their own) */
int gns_cm_reclaim(gns_cm *cm);
int gns_cm_set_timing(gns_cm *cm, int on);
int gns_cm_stage_times(gns_cm *cm, double ms[8], uint64_t launches[8], int reset);
void *gns_cm_stream(gns_cm *cm); /* hipStream_t the handle launches on */

/* Snapshot view: heavy hitters and queries CONCURRENT with ingest (BASELINE
 * configs[4]; the reference's snapshotter and alerter call Task.Snapshot ->
 * HeavyHitters while the workers insert, manager.go:139-159, task.go:177).
 *   - gns_cm_view_refresh is an ingest-side call (serialized with the handle's
 *     other calls): it copies the bucket state, in insert order, at the current
 *     end of the insert stream (a window boundary), asynchronously on the
 *     handle's stream.
 *   - gns_cm_view_heavy_hitters / gns_cm_view_query may run on any other
 *     thread while the handle keeps inserting; they run on the view's own
 *     stream and see exactly the state at the last refresh (same results as
 *     gns_cm_heavy_hitters / gns_cm_query called at that point).
 *   - A refresh waits for a view call in progress; after gns_cm_reset the view
 *     answers GNS_E_ARG until it is refreshed.  Destroy views before their handle.
 * Memory: 16 bytes per bucket (depth*width) for the snapshot. */
typedef struct gns_cm_view gns_cm_view;
int gns_cm_view_create(gns_cm *cm, gns_cm_view **out);
int gns_cm_view_destroy(gns_cm_view *v);
int gns_cm_view_refresh(gns_cm_view *v);
int gns_cm_view_heavy_hitters(gns_cm_view *v, uint8_t *count_flows, uint32_t *counts, uint64_t *n_count,
                              uint8_t *size_flows, uint32_t *sizes, uint64_t *n_size);
int gns_cm_view_query(gns_cm_view *v, const uint8_t *keys, uint32_t stride, uint64_t n, uint64_t *out);

/* ------------------------------------------------------------------ */
/* SuperSpread (super_spread.go)                                      */
/* ------------------------------------------------------------------ */
typedef struct gns_ss gns_ss;

typedef struct gns_ss_params {
    uint32_t width, depth, threshold;  /* 0 -> 2^20 / 3 / 4096 (super_spread.go:12-20) */
    uint32_t m, size;                  /* 0 -> 128 / 5; size <= 8 */
    double base, b;                    /* 0 -> 0.5 / 1.08 */
    gns_layout flow, elem;             /* FlowFields / ElementFields */
    uint32_t flow_bytes, elem_bytes;
    const uint32_t *seeds;             /* depth row seeds (super_spread.go:175); NULL -> default */
    uint64_t hll_master;               /* derives each GeneralHLL's seeds[0..1] */
    uint64_t rng_seed;                 /* keys the declared generator replacing rand.Float64 */
    uint64_t batch_packets;
    uint64_t max_flows;                /* initial flow dictionary capacity (grows); 0 -> 4M */
    int device;
} gns_ss_params;

/* The SuperSpread flow dictionary holds the flows that own a cell (only they
 * can be named by a key, a query or a heavy hitter); it is reclaimed and grows
 * like Count-Min's (see the rules above), so inserts do not fail on it.
 * Deviations (GNS_E_ARG at create): depth <= 8, m <= 256, size <= 8, merged
 * key <= 74 bytes, depth * width <= 2^25 cells.  A device batch in which one
 * cell gets more than 8192 encodes (possible with m = 256 only) is undone before
 * any state write and re-run in halves (a cell takes at most one encode per
 * record), so inserts do not fail on it. */
int gns_ss_create(const gns_ss_params *p, gns_ss **out);
int gns_ss_destroy(gns_ss *ss);
int gns_ss_insert_keys(gns_ss *ss, const uint8_t *flows, uint32_t fstride, const uint8_t *elems,
                       uint32_t estride, uint64_t n, gns_mem where);
int gns_ss_insert_tuples(gns_ss *ss, const gns_tuples *t, uint64_t n, gns_mem where);
int gns_ss_insert_headers(gns_ss *ss, const uint8_t *hdr, const uint32_t *wirelen, uint64_t n,
                          gns_mem where);
int gns_ss_flush(gns_ss *ss);
int gns_ss_query(gns_ss *ss, const uint8_t *flows, uint32_t stride, uint64_t n, uint64_t *out);
/* device keys / answers, as gns_cm_query_device */
int gns_ss_query_device(gns_ss *ss, const uint8_t *flows, uint32_t stride, uint64_t n, uint64_t *out);
int gns_ss_heavy_hitters(gns_ss *ss, uint8_t *flows, uint32_t *spreads, uint64_t *n);
int gns_ss_reset(gns_ss *ss);
/* values[d*w], keys[d*w*flow_bytes], regs[d*w*m] (u8), pbits[d*w] */
int gns_ss_export_state(gns_ss *ss, uint32_t *values, uint8_t *keys, uint8_t *regs, double *pbits);
int gns_ss_stats(gns_ss *ss, uint64_t stats[4]);
/* out[8]: inserted, dropped, unsupported, dictionary full, HLL candidates
 * (lz above the batch-entry register), HLL encodes, records, device batches */
int gns_ss_counters(gns_ss *ss, uint64_t out[8]);
int gns_ss_dict_stats(gns_ss *ss, uint64_t out[8]);  /* as gns_cm_dict_stats */
int gns_ss_reclaim(gns_ss *ss);
int gns_ss_set_timing(gns_ss *ss, int on);
int gns_ss_stage_times(gns_ss *ss, double ms[8], uint64_t launches[8], int reset);

/* ------------------------------------------------------------------ */
/* Inputs: synthetic traffic and the pcap packer           */
/* ------------------------------------------------------------------ */
typedef struct gns_synth gns_synth;
typedef struct gns_synth_params {
    uint32_t flows;        /* flow universe F (default 2^20) */
    double zipf_s;         /* default 1.1 */
    uint64_t tuple_seed;   /* default 0x5EED0001 */
    uint64_t rank_seed;    /* default 0x5EED0002 */
    uint64_t len_seed;     /* default 0x5EED0003 */
    uint32_t shard, nshards; /* keep only flows whose src slot hashes to `shard` */
    int device;
    uint32_t fanout;       /* > 0: each packet's DstIP is drawn Zipf(zipf_s) over `fanout`
                              destinations instead of the flow's own (SuperSpread C3 shape) */
} gns_synth_params;
int gns_synth_create(const gns_synth_params *p, gns_synth **out);
int gns_synth_destroy(gns_synth *s);
/* Fill device buffers hdr[n*64], wirelen[n] with packets first..first+n-1 of
 * the (shard's) stream.  Deterministic, counter-based. */
int gns_synth_fill(gns_synth *s, uint8_t *hdr_dev, uint32_t *wirelen_dev, uint64_t first,
                   uint64_t n);
/* flow tuple of each shard-local flow (for tests): src16,dst16 [flows*16] etc */
int gns_synth_flows(gns_synth *s, uint32_t *n_flows);

/* capture file -> 64-byte records + wirelen (pkg/pcap/reader.go:35-49, which
 * opens it with libpcap's pcap_open_offline: classic pcap in either byte order
 * and time unit, or pcapng with any number of sections and interfaces;
 * Ethernet link type only).  Returns the number of records written (<= cap) or
 * a negative status; *total = packets in the file. */
int64_t gns_pack_pcap(const char *path, uint8_t *hdr, uint32_t *wirelen, uint64_t cap,
                      uint64_t *total);

/* as gns_pack_pcap, into compact records (see gns_cm_insert_compact): frames whose
 * tuple is not an IPv4 one go to side64 (side_cap records; *n_side = the number
 * written, or needed: GNS_E_RANGE when it exceeds side_cap) */
int64_t gns_pack_pcap_compact(const char *path, uint8_t *rec16, uint32_t *wirelen, uint64_t cap,
                              uint8_t *side64, uint64_t side_cap, uint64_t *n_side, uint64_t *total);
/* 64-byte records -> compact records on the device (all pointers DEVICE memory of
 * `device`; inputs complete before the call); *n_side as above */
int gns_compact_headers(const uint8_t *hdr, const uint32_t *wirelen, uint64_t n, uint8_t *rec16,
                        uint8_t *side64, uint64_t side_cap, uint64_t *n_side, int device);
/* the 16-byte forms (gns_cm_insert_compact with wirelen == NULL): GNS_E_RANGE when a
 * wire length exceeds 65535 */
int64_t gns_pack_pcap_compact16(const char *path, uint8_t *rec16, uint64_t cap, uint8_t *side64,
                                uint64_t side_cap, uint64_t *n_side, uint64_t *total);
int gns_compact_headers16(const uint8_t *hdr, const uint32_t *wirelen, uint64_t n, uint8_t *rec16,
                          uint8_t *side64, uint64_t side_cap, uint64_t *n_side, int device);

/* [0] frames copied verbatim, [1] frames decoded on the host into 0x88B5
 * records, [2] frames without an IP layer, of the calling thread's last
 * gns_pack_pcap[_ts] call (records written only) */
int gns_pack_counts(uint64_t out[3]);

/* One captured frame -> one 64-byte record (what gns_pack_pcap writes for it):
 * a frame of the device fast-path shape (untagged IPv4, IHL 5, not a fragment,
 * TCP or non-tunnel UDP, by both caplen and wirelen) is copied verbatim;
 * any other frame is decoded here the way gopacket v1.1.19 + parser.go:23-67
 * decode it -- Ethernet/LLC/SNAP, any number of 802.1Q tags, IPv4 options,
 * IPv6 extension chains, IP-in-IP, GRE, VXLAN, Geneve, GTP-U, MPLS, PPPoE/PPP,
 * EtherIP; first IPv4 layer else first IPv6, first TCP layer else first UDP --
 * into a pre-parsed 0x88B5 record, or into a record the device drops when the
 * frame has no IP layer ("not an IP packet", parser.go:48-49).
 * Returns 0 verbatim, 1 decoded, 2 no IP layer, < 0 on a bad argument.
 * Replaces the per-packet gopacket.NewPacket decode of reader.go:35-49. */
int gns_frame_record(const uint8_t *frame, uint32_t caplen, uint32_t wirelen, uint8_t *rec64);

/* as gns_pack_pcap, plus ts_ns[n] = capture timestamp in ns (PacketInfo.Timestamp,
 * parser.go:30-33; gopacket opens captures with nanosecond precision) */
int64_t gns_pack_pcap_ts(const char *path, uint8_t *hdr, uint32_t *wirelen, int64_t *ts_ns, uint64_t cap,
                         uint64_t *total);

/* Thrift live path: decode n binary-protocol PacketInfo messages
 * (api/thrift/v1/traffic.thrift; packetcodec.go:97-108 UnmarshalPacketInfo over
 * apache/thrift v0.22.0) laid out back to back in buf, message i =
 * buf[offsets[i], offsets[i+1]), into DEVICE buffers hdr_out[n*64] (pre-parsed
 * 0x88B5 records), wirelen_out[n] = uint32(Length), ts_out[n] =
 * TimestampUnixNano.  A message the reference rejects becomes a record the
 * parser drops (*n_bad counts them).  buf/offsets live in `where`.  The records
 * feed gns_{cm,ss,ex}_insert_headers unchanged. */
int gns_thrift_decode(const uint8_t *buf, uint64_t buf_bytes, const uint64_t *offsets, uint64_t n,
                      uint8_t *hdr_out, uint32_t *wirelen_out, int64_t *ts_out, uint64_t *n_bad,
                      gns_mem where, int device);

/* ------------------------------------------------------------------ */
/* Flow routing for the multi-GPU path (BASELINE configs[3]) */
/* ------------------------------------------------------------------ */
/* Replaces the per-packet host split of the sharded deployment (SURVEY §8e:
 * "sharded by src-IP ... use the full key when SrcIP is not in the key";
 * go2netspectra_amd/dist.py owner_fields / owner_of_* are the host form).
 *
 * Every flow of every task must be owned by ONE shard, so that each shard's
 * sketch is exact for its sub-stream.  A router hashes an OWNER KEY made of
 * fields that every task's flow key contains (a flow key is the configured
 * fields, task.go:265-300; any non-empty field list is legal, config.go:59):
 * shard = mm3(owner key, 0xA5A5A5A5) % nshards.  IP slots enter the owner key
 * with an IPv4-mapped IPv6 slot folded to its IPv4 slot, so the owner is a
 * function of the EncodeFlow bytes and of the exact aggregator's To16 key alike.
 *
 * gns_route_owner_fields: the owner key of a set of tasks (a Manager's tasks,
 * manager.go:139-159 runs them on every packet): [SrcIP] when every task's key
 * holds SrcIP (configs[3]), else the fields common to all tasks in canonical
 * order (SrcIP, DstIP, SrcPort, DstPort, Protocol) -- for one task its whole
 * flow key.  GNS_E_ARG (with a message) when the tasks share no field: no
 * single owner exists for such a set.  Host logic only (no device needed). */
int gns_route_owner_fields(const gns_layout *tasks, uint32_t n_tasks, gns_layout *owner);
typedef struct gns_route gns_route;
/* nshards <= 64; owner = gns_route_owner_fields' result (or any non-empty field set) */
int gns_route_create_keyed(uint32_t nshards, const gns_layout *owner, int device, gns_route **out);
/* = gns_route_create_keyed with owner [SrcIP] */
int gns_route_create(uint32_t nshards, int device, gns_route **out);
int gns_route_destroy(gns_route *r);
int gns_route_owner_layout(gns_route *r, gns_layout *owner);
/* gns_route_partition reorders n DEVICE-resident 64-byte records (+ wire
 * lengths) into nshards runs, shard by shard, keeping packet order inside each
 * run (stable); counts[g] (host) = length of run g.  Records the parser drops
 * or does not support go to shard 0.  The call returns after the device work.
 * An all-to-all of run g to rank g, received runs concatenated in source-rank
 * order, delivers to every GPU exactly its stable filter of the stream. */
int gns_route_partition(gns_route *r, const uint8_t *hdr, const uint32_t *wirelen, uint64_t n,
                        uint8_t *out_hdr, uint32_t *out_wirelen, uint64_t *counts);
/* The same partition queued on `stream` (a hipStream_t; NULL = the router's own)
 * without waiting: counts_dev[g] (DEVICE int64) = length of run g once the stream
 * reaches it -- the all-to-all's split sizes stay on the device until the one
 * host read the exchange needs (dist.exchange_runs).  Partitions of one router
 * are ordered after each other whatever streams they are queued on (they share
 * its scratch). */
int gns_route_partition_async(gns_route *r, const uint8_t *hdr, const uint32_t *wirelen, uint64_t n,
                              uint8_t *out_hdr, uint32_t *out_wirelen, int64_t *counts_dev, void *stream);
/* Owner-routed queries (SURVEY §8e "queries are routed to the owner shard";
 * Sketch.Query, count_min.go:160-174 / super_spread.go:238-249, answers from the
 * shard that holds the flow): owner[i] = the shard owning flow key i, keys laid
 * out as key_layout (the querying task's FlowFields; it must contain every owner
 * field, else GNS_E_ARG).  keys and owner both in `where`; returns after the
 * device work.  dist.routed_query / the Go Router's QueryRouted exchange the
 * keys by owner, query each shard's handle and return the answers in order. */
int gns_route_owner_keys(gns_route *r, const gns_layout *key_layout, const uint8_t *keys, uint32_t stride,
                         uint64_t n, uint32_t *owner, gns_mem where);

/* ------------------------------------------------------------------ */
/* Exact aggregator (internal/engine/impl/exact/task.go)               */
/* ------------------------------------------------------------------ */
/* Replaces exact.New (task.go:83-103), Task.ProcessPacket (:124-149),
 * Task.Query (:298-326), Task.Snapshot (:153-191) and Task.Reset (:194-210).
 * Flows are keyed like the reference's string key strings.Join(fields, "-")
 * with IPs printed by net.IP.String(): the engine stores each IP field as its
 * 16-byte form (IPv4 and IPv4-mapped IPv6 -> ::ffff:a.b.c.d, other IPv6 as
 * is), which is equal exactly when the printed strings are equal. */
typedef struct gns_ex gns_ex;
typedef struct gns_ex_params {
    gns_layout key;          /* key_fields (task.go:330-366) */
    uint64_t max_flows;      /* initial flow dictionary capacity (default 4M; the table grows) */
    uint64_t batch_packets;  /* device batch (default 16M) */
    int device;
} gns_ex_params;
int gns_ex_create(const gns_ex_params *p, gns_ex **out);
int gns_ex_destroy(gns_ex *ex);
/* ProcessPacket over PacketInfo batches.  ipver[n]: 4 (net.IP of 4 bytes, IPv4
 * left-aligned in the 16-byte slots) or 6 (16-byte net.IP); ts_ns[n] =
 * PacketInfo.Timestamp.UnixNano(); t->length = ByteCount increment. */
int gns_ex_insert_tuples(gns_ex *ex, const gns_tuples *t, const uint8_t *ipver, const int64_t *ts_ns,
                         uint64_t n, gns_mem where);
/* fused parse of 64-byte records (as gns_cm_insert_headers) + timestamps */
int gns_ex_insert_headers(gns_ex *ex, const uint8_t *hdr, const uint32_t *wirelen, const int64_t *ts_ns,
                          uint64_t n, gns_mem where);
int gns_ex_flush(gns_ex *ex);
/* out[i] = PacketCount << 32 | ByteCount (task.go:323); IP fields of the
 * encoded flow are read as 16-byte net.IPs, as the reference does; 0 if absent */
int gns_ex_query(gns_ex *ex, const uint8_t *flows, uint32_t stride, uint64_t n, uint64_t *out);
/* device keys / answers, as gns_cm_query_device */
int gns_ex_query_device(gns_ex *ex, const uint8_t *flows, uint32_t stride, uint64_t n, uint64_t *out);
/* Snapshot: *n_io = capacity in, number of flows out.  keys[n*key_bytes] in the
 * canonical 16-byte-IP layout; start/end = first/last packet timestamps
 * (stream order), pkts/bytes = PacketCount/ByteCount.  Any pointer may be NULL. */
int gns_ex_snapshot(gns_ex *ex, uint8_t *keys, int64_t *start_ns, int64_t *end_ns, uint64_t *pkts,
                    uint64_t *bytes, uint64_t *n_io);
int gns_ex_reset(gns_ex *ex);
/* out[8]: inserted, dropped, unsupported, dictionary full, flows, records, batches, 0 */
int gns_ex_counters(gns_ex *ex, uint64_t out[8]);
/* [0] table growths, [1] 0, [2] slots, [3] claimed slots, [4] growth time (us),
 * [5] batches re-run after a dictionary overflow, [6] slots, [7] growths */
int gns_ex_dict_stats(gns_ex *ex, uint64_t out[8]);
int gns_ex_set_timing(gns_ex *ex, int on);
/* stages: 0 extract, 1 resolve, 2 aggregate, 3 timestamps, 5 total */
int gns_ex_stage_times(gns_ex *ex, double ms[8], uint64_t launches[8], int reset);

/* Device buffers for callers without a device allocator of their own (the cgo
 * binding's ThriftDecoder: gns_thrift_decode writes device records that
 * gns_*_insert_headers then reads with GNS_MEM_DEVICE). */
int gns_device_alloc(uint64_t bytes, int device, void **out);
int gns_device_free(void *p, int device);

const char *gns_last_error(void);
const char *gns_version(void);

#ifdef __cplusplus
}
#endif
#endif
