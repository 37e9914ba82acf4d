/*
 * gns_oracle.h -- CPU ORACLE (test infrastructure, never product code).
 *
 * A plain-C sequential restatement of the reference's sketch hot path
 * (Decade-qiu/Go2NetSpectra @ 2026-04-24, read-only at /root/reference):
 *   - MurmurHash3_x86_32            internal/engine/impl/sketch/statistic/hash.go:13-53
 *   - flow-key encoding             internal/engine/impl/sketch/task.go:265-300,327-338
 *   - packet -> 5-tuple             internal/protocol/parser.go:23-67 (+ gopacket v1.1.19 subset)
 *   - fingerprinted "CountMin"      internal/engine/impl/sketch/statistic/count_min.go:47-265
 *   - SuperSpread (+ GeneralHLL)    internal/engine/impl/sketch/statistic/super_spread.go:24-311
 *   - math.Pow integer path         Go stdlib math/pow.go (restated; not vendored)
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library, and only as the checker / the timed CPU baseline.  The product
 * (go2netspectra_amd) never links or calls it.
 *
 * Determinism contract (the reference itself is not deterministic, see
 * SURVEY.md §0.2): row seeds and SuperSpread HLL seeds are injected, the packet
 * stream is applied in order by ONE worker, and SuperSpread's rand.Float64()
 * draws are replaced by the declared counter-based generator or_ss_uniform().
 *
 * Parity status: MurmurHash3 is pinned by public KATs (tests/golden/mm3_kat.json).
 * The bucket state machines are pinned only by hand-derived traces from
 * count_min.go / super_spread.go (the reference ships no counter fixtures and Go
 * is not installed), i.e. "parity unpinned" against an executed reference.
 */
#ifndef GNS_ORACLE_H
#define GNS_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- hash.go:13-53 ---- */
uint32_t or_mm3(const uint8_t *data, uint32_t len, uint32_t seed);

/* ---- model.FiveTuple (internal/model/packet.go:9-22), IP slots already laid
 * out as EncodeFlow copies them (IPv4 left-aligned, 12 zero bytes). ---- */
typedef struct or_tuple {
    uint8_t src[16];
    uint8_t dst[16];
    uint16_t sport, dport;
    uint8_t proto;
    uint8_t ipver;     /* source net.IP: 4 (4 bytes) or 6 (16 bytes); 0 other (Thrift path) */
    uint8_t dst_ipver; /* destination, same coding */
} or_tuple;

enum { OR_PARSE_OK = 0, OR_PARSE_DROP = 1, OR_PARSE_UNSUPPORTED = 2 };

/* parser.go:23-67 restricted to the 64-byte record subset. */
int or_parse_hdr64(const uint8_t *rec, or_tuple *out);

/* field ids: task.go:279-300 */
enum { OR_F_SRCIP = 1, OR_F_DSTIP = 2, OR_F_SRCPORT = 3, OR_F_DSTPORT = 4, OR_F_PROTO = 5 };
uint32_t or_field_size(uint8_t field);                       /* task.go:327-338 */
uint32_t or_encode_key(const uint8_t *fields, uint32_t nfields, const or_tuple *t,
                       uint8_t *out);                        /* task.go:265-300 */

/* ---- count_min.go ---- */
typedef struct or_cm or_cm;
or_cm *or_cm_new(uint32_t width, uint32_t depth, uint32_t st, uint32_t ct, uint32_t key_bytes,
                 const uint32_t *seeds);
void or_cm_free(or_cm *cm);
void or_cm_params(const or_cm *cm, uint32_t *w, uint32_t *d, uint32_t *st, uint32_t *ct);
void or_cm_insert(or_cm *cm, const uint8_t *key, uint32_t size);
void or_cm_insert_batch(or_cm *cm, const uint8_t *keys, uint32_t stride, const uint32_t *sizes,
                        uint64_t n);
/* parse + encode + insert, the reference worker loop (manager.go:232-244 ->
 * task.go:156-169) over 64-byte records; returns packets inserted. */
uint64_t or_cm_insert_hdr64(or_cm *cm, const uint8_t *hdr, const uint32_t *wirelen, uint64_t n,
                            const uint8_t *fields, uint32_t nfields);
/* Same work as a restatement of the Go worker pool: nthreads workers pull
 * packets from a shared cursor (stand-in for the Go channel, manager.go:218-244)
 * and run count_min.go:100-155's CAS loops on the shared sketch.
 * Non-deterministic by design (like the reference) -> timed, never compared. */
uint64_t or_cm_insert_hdr64_pool(or_cm *cm, const uint8_t *hdr, const uint32_t *wirelen,
                                 uint64_t n, const uint8_t *fields, uint32_t nfields,
                                 int nthreads);
uint64_t or_cm_query(const or_cm *cm, const uint8_t *key);
void or_cm_export(const or_cm *cm, uint32_t *C, uint32_t *S, uint8_t *FPc, uint8_t *FPs);
void or_cm_import(or_cm *cm, const uint32_t *C, const uint32_t *S, const uint8_t *FPc,
                  const uint8_t *FPs);
/* HeavyHitters (count_min.go:178-246), canonicalised: value desc, flow bytes asc.
 * which = 0 -> Count list, 1 -> Size list.  Returns the list length; writes up
 * to cap entries. */
uint32_t or_cm_heavy(const or_cm *cm, int which, uint8_t *flows, uint32_t *vals, uint32_t cap);
void or_cm_reset(or_cm *cm);

/* ---- super_spread.go ---- */
typedef struct or_ss or_ss;
/* hll_master derives each GeneralHLL's seeds[0..1] (super_spread.go:47-49 draws
 * m+1 random seeds, only the first two are ever used), rng_seed keys the
 * declared generator that replaces rand.Float64() (super_spread.go:201,223). */
or_ss *or_ss_new(uint32_t width, uint32_t depth, uint32_t threshold, uint32_t m, uint32_t size,
                 double base, double b, uint32_t flow_bytes, uint32_t elem_bytes,
                 const uint32_t *seeds, uint64_t hll_master, uint64_t rng_seed);
void or_ss_free(or_ss *ss);
void or_ss_insert(or_ss *ss, const uint8_t *flow, const uint8_t *elem);
void or_ss_insert_batch(or_ss *ss, const uint8_t *flows, uint32_t fstride, const uint8_t *elems,
                        uint32_t estride, uint64_t n);
uint64_t or_ss_insert_hdr64(or_ss *ss, const uint8_t *hdr, const uint32_t *wirelen, uint64_t n,
                            const uint8_t *ffields, uint32_t nff, const uint8_t *efields, uint32_t nef);
uint64_t or_ss_query(const or_ss *ss, const uint8_t *flow);
uint32_t or_ss_heavy(const or_ss *ss, uint8_t *flows, uint32_t *vals, uint32_t cap);
void or_ss_export(const or_ss *ss, uint32_t *values, uint8_t *keys, uint8_t *regs, double *pbits);
void or_ss_reset(or_ss *ss);
uint64_t or_ss_packets(const or_ss *ss);

/* declared generator + Go helpers (exposed for tests) */
uint64_t or_mix64(uint64_t x);
double or_ss_uniform(uint64_t rng_seed, uint64_t pkt, uint32_t row, uint32_t draw);
void or_ss_hll_seeds(uint64_t hll_master, uint64_t cell, uint32_t *s0, uint32_t *s1);
double or_go_pow(double x, double y);
double or_det_log(double x);    /* deterministic log, x in (0, 1] */
double or_det_log1m(double p);  /* log(1 - p), 0 < p < 1 */
double or_go_ldexp(double frac, int e);

/* splitmix64 stream (BASELINE/SURVEY §8d seeds) */
uint64_t or_splitmix64_next(uint64_t *state);

/* ---- exact aggregator, internal/engine/impl/exact/task.go (gns_oracle_exact.c) ---- */
typedef struct or_ex or_ex;
or_ex *or_ex_new(const uint8_t *fields, uint32_t nfields);
void or_ex_free(or_ex *ex);
void or_ex_reset(or_ex *ex);
void or_ex_insert(or_ex *ex, const or_tuple *t, int64_t ts, uint64_t length);
void or_ex_insert_tuples(or_ex *ex, const uint8_t *src16, const uint8_t *dst16, const uint16_t *sport,
                         const uint16_t *dport, const uint8_t *proto, const uint8_t *ipver,
                         const uint32_t *length, const int64_t *ts, uint64_t n);
uint64_t or_ex_insert_hdr64(or_ex *ex, const uint8_t *hdr, const uint32_t *wirelen, const int64_t *ts,
                            uint64_t n);
uint64_t or_ex_query(const or_ex *ex, const uint8_t *flow);
uint64_t or_ex_count(const or_ex *ex);
uint64_t or_ex_export(const or_ex *ex, char *keys_out, uint64_t keys_cap, int64_t *start, int64_t *end,
                      uint64_t *pkts, uint64_t *bytes);
int or_parse_hdr64_len(const uint8_t *rec, uint32_t wirelen, or_tuple *out);

/* ---- Thrift PacketInfo decode, packetcodec.go:97-108 (gns_oracle_thrift.c) ---- */
int or_thrift_decode_one(const uint8_t *msg, uint64_t len, or_tuple *t, uint8_t *dst_ver, int64_t *length,
                         int64_t *ts);
uint64_t or_thrift_decode(const uint8_t *buf, const uint64_t *offsets, uint64_t n, uint8_t *ok, uint8_t *src16,
                          uint8_t *dst16, uint16_t *sport, uint16_t *dport, uint8_t *proto, uint8_t *sver,
                          uint8_t *dver, int64_t *length, int64_t *ts);

#ifdef __cplusplus
}
#endif
#endif
