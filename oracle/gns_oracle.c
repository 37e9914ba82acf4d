/*
 * gns_oracle.c -- CPU ORACLE (test infrastructure only; see gns_oracle.h).
 *
 * Sequential restatement of the reference's sketch path.  Every function cites
 * the reference file:line it restates (paths relative to /root/reference).
 * Built with -O2 -ffp-contract=off so the float64 steps of SuperSpread round
 * exactly like Go's (no fused multiply-add).
 */
#define _GNU_SOURCE
#include "gns_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* hash.go:13-53 -- MurmurHash3_x86_32                                        */
/* ------------------------------------------------------------------------- */
static inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

uint32_t or_mm3(const uint8_t *data, uint32_t len, uint32_t seed) {
    const uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u; /* hash.go:7-10 */
    uint32_t h1 = seed;
    uint32_t nblocks = len / 4;
    for (uint32_t i = 0; i < nblocks; i++) { /* hash.go:16-27 */
        const uint8_t *p = data + 4 * i;
        uint32_t k1 = (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 |
                      (uint32_t)p[3] << 24;
        k1 *= c1;
        k1 = rotl32(k1, 15);
        k1 *= c2;
        h1 ^= k1;
        h1 = rotl32(h1, 13);
        h1 = h1 * 5 + 0xe6546b64u;
    }
    const uint8_t *tail = data + 4 * nblocks;
    uint32_t k1 = 0;
    switch (len & 3) { /* hash.go:28-42 */
    case 3: k1 ^= (uint32_t)tail[2] << 16; /* fallthrough */
    case 2: k1 ^= (uint32_t)tail[1] << 8;  /* fallthrough */
    case 1:
        k1 ^= (uint32_t)tail[0];
        k1 *= c1;
        k1 = rotl32(k1, 15);
        k1 *= c2;
        h1 ^= k1;
    }
    h1 ^= len; /* hash.go:44-50 fmix32 */
    h1 ^= h1 >> 16;
    h1 *= 0x85ebca6bu;
    h1 ^= h1 >> 13;
    h1 *= 0xc2b2ae35u;
    h1 ^= h1 >> 16;
    return h1;
}

/* ------------------------------------------------------------------------- */
/* 64-byte record -> FiveTuple.  parser.go:23-67 over gopacket v1.1.19 layers,  */
/* restricted to the record contract in DESIGN.md §"Header records".          */
/* ------------------------------------------------------------------------- */
static inline uint16_t be16(const uint8_t *p) { return (uint16_t)(p[0] << 8 | p[1]); }

static int udp_tunnel_port(uint16_t p) { return p == 4789 || p == 6081 || p == 2152; }

int or_parse_hdr64_len(const uint8_t *r, uint32_t wirelen, or_tuple *t);

int or_parse_hdr64(const uint8_t *r, or_tuple *t) { return or_parse_hdr64_len(r, 0xFFFFFFFFu, t); }

int or_parse_hdr64_len(const uint8_t *r, uint32_t wirelen, or_tuple *t) {
    memset(t, 0, sizeof(*t));
    uint32_t type = be16(r + 12);
    uint32_t off = 14;
    if (type == 0x88B5) { /* pre-parsed record written by the host packer */
        if (r[14] != 1) return OR_PARSE_UNSUPPORTED;
        t->ipver = r[15];
        t->dst_ipver = r[53] ? r[53] : r[15];
        memcpy(t->src, r + 16, 16);
        memcpy(t->dst, r + 32, 16);
        t->sport = be16(r + 48);
        t->dport = be16(r + 50);
        t->proto = r[52];
        return OR_PARSE_OK;
    }
    for (int nv = 0; type == 0x8100 || type == 0x88A8; nv++) { /* gopacket Dot1Q */
        if (nv == 2) return OR_PARSE_UNSUPPORTED;
        type = be16(r + off + 2);
        off += 4;
    }
    uint32_t l2len = wirelen > off ? wirelen - off : 0; /* bytes after the L2 header */
    /* gopacket v1.1.19 decodeIPv4 / decodeIPv6 / decodeTCP / decodeUDP add the
     * layer before returning a decode error, with the fields DecodeFromBytes set
     * before the failing check; parser.go:38-61 reads those fields. */
    if (type == 0x0800) { /* gopacket IPv4.DecodeFromBytes */
        const uint8_t *ip = r + off;
        if (l2len < 20) return OR_PARSE_OK; /* "Invalid ip4 header": nil IPs, Protocol 0 */
        uint32_t ihl = ip[0] & 15u;
        uint32_t tot = be16(ip + 2);
        if (tot == 0) tot = l2len; /* TSO: Length := len(data) */
        t->ipver = 4;
        t->dst_ipver = 4;
        t->proto = ip[9];                        /* parser.go:42 */
        memcpy(t->src, ip + 12, 4);               /* parser.go:40-41; task.go:281-286 */
        memcpy(t->dst, ip + 16, 4);
        if (tot < 20 || ihl < 5 || ihl * 4 > tot) return OR_PARSE_OK; /* error: no next layer */
        if (ihl > 5) return OR_PARSE_UNSUPPORTED; /* options: host packer */
        uint32_t frag = be16(ip + 6);
        if ((frag & 0x2000u) || (frag & 0x1FFFu)) return OR_PARSE_OK; /* LayerTypeFragment */
        uint32_t avail = (tot < l2len ? tot : l2len) - 20;
        if (avail == 0) return OR_PARSE_OK; /* NextDecoder on an empty payload: no layer */
        const uint8_t *l4 = ip + 20;
        switch (t->proto) {
        case 6: /* decodeTCP: ports are read before the data-offset checks */
            if (avail < 20) return OR_PARSE_OK;
            t->sport = be16(l4);
            t->dport = be16(l4 + 2);
            return OR_PARSE_OK;
        case 17: /* gopacket UDP.DecodeFromBytes */
            if (avail < 8) return OR_PARSE_OK;
            if (udp_tunnel_port(be16(l4)) || udp_tunnel_port(be16(l4 + 2)))
                return OR_PARSE_UNSUPPORTED;
            t->sport = be16(l4);
            t->dport = be16(l4 + 2);
            return OR_PARSE_OK;
        case 0: case 4: case 41: case 43: case 47: case 51: case 60: case 137:
            return OR_PARSE_UNSUPPORTED; /* inner layers could hold IPv4/TCP/UDP */
        default:
            return OR_PARSE_OK; /* ICMP etc.: ports stay 0 (parser.go:62) */
        }
    }
    if (type == 0x86DD) { /* gopacket IPv6.DecodeFromBytes */
        const uint8_t *ip = r + off;
        if (l2len < 40) return OR_PARSE_OK; /* nil IPs, NextHeader 0 */
        uint32_t plen = be16(ip + 4);
        uint32_t nh = ip[6];
        t->ipver = 6;
        t->dst_ipver = 6;
        t->proto = (uint8_t)nh; /* parser.go:47: first NextHeader */
        memcpy(t->src, ip + 8, 16);
        memcpy(t->dst, ip + 24, 16);
        if (nh == 0) return OR_PARSE_UNSUPPORTED; /* hop-by-hop / jumbogram: host packer */
        if (plen == 0) return OR_PARSE_OK;        /* "IPv6 length 0, but next header is ..." */
        uint32_t cap = l2len - 40;
        uint32_t avail = plen < cap ? plen : cap;
        if (avail == 0) return OR_PARSE_OK;
        const uint8_t *l4 = ip + 40;
        uint32_t l4off = off + 40;
        switch (nh) {
        case 4: case 41: case 43: case 47: case 51: case 60: case 137:
            return OR_PARSE_UNSUPPORTED; /* extension headers / encapsulation */
        case 6:
            if (avail < 20) return OR_PARSE_OK;
            if (l4off + 4 > 64) return OR_PARSE_UNSUPPORTED;
            t->sport = be16(l4);
            t->dport = be16(l4 + 2);
            return OR_PARSE_OK;
        case 17:
            if (avail < 8) return OR_PARSE_OK;
            if (l4off + 4 > 64) return OR_PARSE_UNSUPPORTED;
            if (udp_tunnel_port(be16(l4)) || udp_tunnel_port(be16(l4 + 2)))
                return OR_PARSE_UNSUPPORTED;
            t->sport = be16(l4);
            t->dport = be16(l4 + 2);
            return OR_PARSE_OK;
        default:
            return OR_PARSE_OK;
        }
    }
    switch (type) { /* well-known non-IP ethertypes: parser.go:48-49 "not an IP packet" */
    case 0x0806: case 0x8035: case 0x88CC: case 0x8808: case 0x888E: case 0x88F7: case 0x8863:
        return OR_PARSE_DROP;
    default:
        return OR_PARSE_UNSUPPORTED; /* 802.3/LLC, MPLS, PPPoE, ...: host packer decides */
    }
}

/* ------------------------------------------------------------------------- */
/* task.go:265-300 (EncodeFlow) and :327-338 (fieldByteSize)                   */
/* ------------------------------------------------------------------------- */
uint32_t or_field_size(uint8_t f) {
    switch (f) {
    case OR_F_SRCIP: case OR_F_DSTIP: return 16;
    case OR_F_SRCPORT: case OR_F_DSTPORT: return 2;
    case OR_F_PROTO: return 1;
    default: return 0;
    }
}

uint32_t or_encode_key(const uint8_t *fields, uint32_t nfields, const or_tuple *t, uint8_t *out) {
    uint32_t off = 0;
    for (uint32_t i = 0; i < nfields; i++) {
        switch (fields[i]) {
        case OR_F_SRCIP: memcpy(out + off, t->src, 16); off += 16; break;
        case OR_F_DSTIP: memcpy(out + off, t->dst, 16); off += 16; break;
        case OR_F_SRCPORT: out[off] = t->sport >> 8; out[off + 1] = t->sport & 0xFF; off += 2; break;
        case OR_F_DSTPORT: out[off] = t->dport >> 8; out[off + 1] = t->dport & 0xFF; off += 2; break;
        case OR_F_PROTO: out[off] = t->proto; off += 1; break;
        default: break;
        }
    }
    return off;
}

/* ------------------------------------------------------------------------- */
/* count_min.go                                                               */
/* ------------------------------------------------------------------------- */
struct or_cm {
    uint32_t w, d, st, ct, K;
    uint32_t *seed;
    uint32_t *C, *S; /* [d*w]      PacketCount.C / PacketSize.S */
    uint8_t *FPc, *FPs; /* [d*w*K] PacketCount.FP / PacketSize.FP */
};

or_cm *or_cm_new(uint32_t width, uint32_t depth, uint32_t st, uint32_t ct, uint32_t K,
                 const uint32_t *seeds) {
    /* defaults: count_min.go:11-16,47-59 */
    if (width == 0) width = 1u << 20;
    if (depth == 0) depth = 3;
    if (st == 0) st = 512 * 1024;
    if (ct == 0) ct = 512;
    or_cm *cm = (or_cm *)calloc(1, sizeof(or_cm));
    cm->w = width; cm->d = depth; cm->st = st; cm->ct = ct; cm->K = K;
    cm->seed = (uint32_t *)malloc(sizeof(uint32_t) * depth);
    for (uint32_t i = 0; i < depth; i++) cm->seed[i] = seeds[i]; /* injected (count_min.go:61-64) */
    size_t cells = (size_t)depth * width;
    cm->C = (uint32_t *)calloc(cells, 4);
    cm->S = (uint32_t *)calloc(cells, 4);
    cm->FPc = (uint8_t *)calloc(cells * (K ? K : 1), 1);
    cm->FPs = (uint8_t *)calloc(cells * (K ? K : 1), 1);
    return cm;
}

void or_cm_free(or_cm *cm) {
    if (!cm) return;
    free(cm->seed); free(cm->C); free(cm->S); free(cm->FPc); free(cm->FPs); free(cm);
}

void or_cm_params(const or_cm *cm, uint32_t *w, uint32_t *d, uint32_t *st, uint32_t *ct) {
    *w = cm->w; *d = cm->d; *st = cm->st; *ct = cm->ct;
}

/* count_min.go:94-157, one worker (no CAS races). */
void or_cm_insert(or_cm *cm, const uint8_t *key, uint32_t size) {
    const uint32_t K = cm->K;
    for (uint32_t i = 0; i < cm->d; i++) {
        size_t cell = (size_t)i * cm->w + or_mm3(key, K, cm->seed[i]) % cm->w; /* :96 */
        uint8_t *fs = cm->FPs + cell * K, *fc = cm->FPc + cell * K;
        /* size half :99-128 */
        uint32_t S = cm->S[cell];
        if (S == 0) { cm->S[cell] = size; memcpy(fs, key, K); }
        else if (memcmp(fs, key, K) == 0) cm->S[cell] = S + size; /* u32 wrap */
        else if (size > S) { cm->S[cell] = size; memcpy(fs, key, K); }
        else cm->S[cell] = S - size;
        /* count half :130-155 */
        uint32_t C = cm->C[cell];
        if (C == 0) { cm->C[cell] = 1; memcpy(fc, key, K); }
        else if (memcmp(fc, key, K) == 0) cm->C[cell] = C + 1;
        else { cm->C[cell] = C - 1; if (C - 1 == 0) memcpy(fc, key, K); }
    }
}

void or_cm_insert_batch(or_cm *cm, const uint8_t *keys, uint32_t stride, const uint32_t *sizes,
                        uint64_t n) {
    for (uint64_t p = 0; p < n; p++) or_cm_insert(cm, keys + p * stride, sizes[p]);
}

uint64_t or_cm_insert_hdr64(or_cm *cm, const uint8_t *hdr, const uint32_t *wirelen, uint64_t n,
                            const uint8_t *fields, uint32_t nfields) {
    uint8_t key[64];
    uint64_t done = 0;
    for (uint64_t p = 0; p < n; p++) {
        or_tuple t;
        if (or_parse_hdr64_len(hdr + p * 64, wirelen[p], &t) != OR_PARSE_OK) continue;
        or_encode_key(fields, nfields, &t, key);
        or_cm_insert(cm, key, wirelen[p]); /* task.go:168 uint32(Length) */
        done++;
    }
    return done;
}

/* --- worker-pool restatement (timed CPU baseline, never compared) --- */
typedef struct {
    or_cm *cm;
    const uint8_t *hdr;
    const uint32_t *wirelen;
    uint64_t n;
    const uint8_t *fields;
    uint32_t nfields;
    uint64_t *cursor;
    uint64_t done;
} pool_arg;

static void cas_insert(or_cm *cm, const uint8_t *key, uint32_t size) {
    const uint32_t K = cm->K;
    for (uint32_t i = 0; i < cm->d; i++) {
        size_t cell = (size_t)i * cm->w + or_mm3(key, K, cm->seed[i]) % cm->w;
        uint32_t *Sp = &cm->S[cell], *Cp = &cm->C[cell];
        uint8_t *fs = cm->FPs + cell * K, *fc = cm->FPc + cell * K;
        for (;;) { /* count_min.go:99-128 */
            uint32_t cur = __atomic_load_n(Sp, __ATOMIC_SEQ_CST);
            if (cur == 0) {
                if (__atomic_compare_exchange_n(Sp, &cur, size, 0, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST)) {
                    memcpy(fs, key, K); break;
                }
            } else if (memcmp(fs, key, K) == 0) {
                if (__atomic_compare_exchange_n(Sp, &cur, cur + size, 0, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST)) break;
            } else if (size > cur) {
                if (__atomic_compare_exchange_n(Sp, &cur, size, 0, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST)) {
                    memcpy(fs, key, K); break;
                }
            } else {
                if (__atomic_compare_exchange_n(Sp, &cur, cur - size, 0, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST)) break;
            }
        }
        for (;;) { /* count_min.go:130-155 */
            uint32_t cur = __atomic_load_n(Cp, __ATOMIC_SEQ_CST);
            if (cur == 0) {
                if (__atomic_compare_exchange_n(Cp, &cur, 1, 0, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST)) {
                    memcpy(fc, key, K); break;
                }
            } else if (memcmp(fc, key, K) == 0) {
                if (__atomic_compare_exchange_n(Cp, &cur, cur + 1, 0, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST)) break;
            } else {
                if (__atomic_compare_exchange_n(Cp, &cur, cur - 1, 0, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST)) {
                    if (cur - 1 == 0) memcpy(fc, key, K);
                    break;
                }
            }
        }
    }
}

static void *pool_worker(void *vp) {
    pool_arg *a = (pool_arg *)vp;
    uint8_t key[64];
    for (;;) {
        /* one shared cursor, one packet per hand-off: the Go channel stand-in */
        uint64_t p = __atomic_fetch_add(a->cursor, 1, __ATOMIC_RELAXED);
        if (p >= a->n) break;
        or_tuple t;
        if (or_parse_hdr64_len(a->hdr + p * 64, a->wirelen[p], &t) != OR_PARSE_OK) continue;
        or_encode_key(a->fields, a->nfields, &t, key);
        cas_insert(a->cm, key, a->wirelen[p]);
        a->done++;
    }
    return NULL;
}

uint64_t or_cm_insert_hdr64_pool(or_cm *cm, const uint8_t *hdr, const uint32_t *wirelen,
                                 uint64_t n, const uint8_t *fields, uint32_t nfields,
                                 int nthreads) {
    if (nthreads < 1) nthreads = 1;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * nthreads);
    pool_arg *args = (pool_arg *)calloc(nthreads, sizeof(pool_arg));
    uint64_t cursor = 0;
    for (int i = 0; i < nthreads; i++) {
        args[i] = (pool_arg){cm, hdr, wirelen, n, fields, nfields, &cursor, 0};
        pthread_create(&th[i], NULL, pool_worker, &args[i]);
    }
    uint64_t done = 0;
    for (int i = 0; i < nthreads; i++) { pthread_join(th[i], NULL); done += args[i].done; }
    free(th); free(args);
    return done;
}

/* count_min.go:160-174 */
uint64_t or_cm_query(const or_cm *cm, const uint8_t *key) {
    uint32_t sz = 0, ct = 0;
    for (uint32_t i = 0; i < cm->d; i++) {
        size_t cell = (size_t)i * cm->w + or_mm3(key, cm->K, cm->seed[i]) % cm->w;
        if (memcmp(cm->FPs + cell * cm->K, key, cm->K) == 0 && cm->S[cell] > sz) sz = cm->S[cell];
        if (memcmp(cm->FPc + cell * cm->K, key, cm->K) == 0 && cm->C[cell] > ct) ct = cm->C[cell];
    }
    return (uint64_t)ct << 32 | sz;
}

void or_cm_export(const or_cm *cm, uint32_t *C, uint32_t *S, uint8_t *FPc, uint8_t *FPs) {
    size_t cells = (size_t)cm->d * cm->w;
    if (C) memcpy(C, cm->C, cells * 4);
    if (S) memcpy(S, cm->S, cells * 4);
    if (FPc) memcpy(FPc, cm->FPc, cells * cm->K);
    if (FPs) memcpy(FPs, cm->FPs, cells * cm->K);
}

void or_cm_import(or_cm *cm, const uint32_t *C, const uint32_t *S, const uint8_t *FPc,
                  const uint8_t *FPs) {
    size_t cells = (size_t)cm->d * cm->w;
    memcpy(cm->C, C, cells * 4);
    memcpy(cm->S, S, cells * 4);
    memcpy(cm->FPc, FPc, cells * cm->K);
    memcpy(cm->FPs, FPs, cells * cm->K);
}

/* heavy-hitter extraction shared by CM and SS */
typedef struct { const uint8_t *fp; uint32_t v; } hh_item;
static uint32_t hh_K;
static int hh_cmp_fp(const void *a, const void *b) {
    const hh_item *x = (const hh_item *)a, *y = (const hh_item *)b;
    int c = memcmp(x->fp, y->fp, hh_K);
    if (c) return c;
    return x->v > y->v ? -1 : x->v < y->v ? 1 : 0;
}
static int hh_cmp_val(const void *a, const void *b) {
    const hh_item *x = (const hh_item *)a, *y = (const hh_item *)b;
    if (x->v != y->v) return x->v > y->v ? -1 : 1;
    return memcmp(x->fp, y->fp, hh_K);
}
static pthread_mutex_t hh_mu = PTHREAD_MUTEX_INITIALIZER;

/* dedupe by fingerprint keeping the max, keep >= thr, sort value desc
 * (count_min.go:178-247); ties ordered by flow bytes (canonical). */
static uint32_t hh_finish(hh_item *it, size_t n, uint32_t K, uint32_t thr, uint8_t *flows,
                          uint32_t *vals, uint32_t cap) {
    pthread_mutex_lock(&hh_mu);
    hh_K = K;
    qsort(it, n, sizeof(hh_item), hh_cmp_fp);
    size_t m = 0;
    for (size_t i = 0; i < n; i++) {
        if (m > 0 && memcmp(it[m - 1].fp, it[i].fp, K) == 0) continue; /* first = max */
        it[m++] = it[i];
    }
    size_t k = 0;
    for (size_t i = 0; i < m; i++)
        if (it[i].v >= thr) it[k++] = it[i];
    qsort(it, k, sizeof(hh_item), hh_cmp_val);
    pthread_mutex_unlock(&hh_mu);
    for (size_t i = 0; i < k && i < cap; i++) {
        if (flows) memcpy(flows + i * K, it[i].fp, K);
        if (vals) vals[i] = it[i].v;
    }
    return (uint32_t)k;
}

uint32_t or_cm_heavy(const or_cm *cm, int which, uint8_t *flows, uint32_t *vals, uint32_t cap) {
    size_t cells = (size_t)cm->d * cm->w;
    hh_item *it = (hh_item *)malloc(sizeof(hh_item) * (cells ? cells : 1));
    size_t n = 0;
    for (size_t c = 0; c < cells; c++) {
        uint32_t v = which ? cm->S[c] : cm->C[c];
        if (v > 0) { /* :188, :198 */
            it[n].fp = (which ? cm->FPs : cm->FPc) + c * cm->K;
            it[n].v = v;
            n++;
        }
    }
    uint32_t r = hh_finish(it, n, cm->K, which ? cm->st : cm->ct, flows, vals, cap);
    free(it);
    return r;
}

/* count_min.go:249-265 */
void or_cm_reset(or_cm *cm) {
    size_t cells = (size_t)cm->d * cm->w;
    memset(cm->C, 0, cells * 4);
    memset(cm->S, 0, cells * 4);
    memset(cm->FPc, 0, cells * cm->K);
    memset(cm->FPs, 0, cells * cm->K);
}

/* ------------------------------------------------------------------------- */
/* Declared generators (replace Go's unseedable global RNGs)     */
/* ------------------------------------------------------------------------- */
uint64_t or_mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

uint64_t or_splitmix64_next(uint64_t *state) {
    *state += 0x9E3779B97F4A7C15ull;
    return or_mix64(*state);
}

double or_ss_uniform(uint64_t rng_seed, uint64_t pkt, uint32_t row, uint32_t draw) {
    uint64_t x = or_mix64(rng_seed + pkt * 0x9E3779B97F4A7C15ull);
    x = or_mix64(x ^ ((uint64_t)row << 32 | draw) ^ 0xD1B54A32D192ED03ull);
    return (double)(x >> 11) * 0x1.0p-53;
}

void or_ss_hll_seeds(uint64_t hll_master, uint64_t cell, uint32_t *s0, uint32_t *s1) {
    uint64_t x = or_mix64(hll_master + cell * 0x9E3779B97F4A7C15ull);
    *s0 = (uint32_t)x;
    *s1 = (uint32_t)(x >> 32);
}

/* Go math.Ldexp (src/math/ldexp.go), bit-level restatement. */
double or_go_ldexp(double frac, int e) {
    if (frac == 0 || isinf(frac) || isnan(frac)) return frac;
    /* normalize */
    int ne = 0;
    if (fabs(frac) < 2.2250738585072014e-308) { frac *= (double)(1ull << 52); ne = -52; }
    e += ne;
    uint64_t x;
    memcpy(&x, &frac, 8);
    e += (int)((x >> 52) & 0x7FF) - 1023;
    if (e < -1075) return copysign(0.0, frac);
    if (e > 1023) return frac < 0 ? -INFINITY : INFINITY;
    double m = 1.0;
    if (e < -1022) { e += 53; m = 1.0 / (double)(1ull << 53); }
    x &= ~(0x7FFull << 52);
    x |= (uint64_t)(e + 1023) << 52;
    double r;
    memcpy(&r, &x, 8);
    return m * r;
}

/* Go math.Pow (src/math/pow.go) for the cases SuperSpread reaches: integer y
 * (float64 of a u32), x > 0.  Non-integer y falls back to libm (unused). */
double or_go_pow(double x, double y) {
    if (y == 0 || x == 1) return 1;
    if (y == 1) return x;
    if (isnan(x) || isnan(y)) return NAN;
    if (x == 0) return y < 0 ? INFINITY : 0;
    if (isinf(y)) {
        if (x == -1) return 1;
        if ((fabs(x) < 1) == (y > 0)) return 0;
        return INFINITY;
    }
    if (isinf(x)) return y < 0 ? 0 : INFINITY; /* x = +Inf only (x > 0) */
    if (y == 0.5) return sqrt(x);
    if (y == -0.5) return 1 / sqrt(x);
    double yi, yf = modf(fabs(y), &yi);
    if (yf != 0) return pow(x, y); /* not reached by super_spread.go */
    if (yi >= 9223372036854775808.0) return 0; /* unreachable for u32 exponents */
    double a1 = 1.0;
    int ae = 0;
    int xe;
    double x1 = frexp(x, &xe);
    for (int64_t i = (int64_t)yi; i != 0; i >>= 1) {
        if (xe < -(1 << 12) || (1 << 12) < xe) { ae += xe; break; }
        if (i & 1) { a1 *= x1; ae += xe; }
        x1 *= x1;
        xe <<= 1;
        if (x1 < .5) { x1 += x1; xe--; }
    }
    if (y < 0) { a1 = 1 / a1; ae = -ae; }
    return or_go_ldexp(a1, ae);
}

/* ------------------------------------------------------------------------- */
/* super_spread.go                                                            */
/* ------------------------------------------------------------------------- */
/* Deterministic natural log for x in (0, 1]: the fdlibm reduction and
 * polynomial (as in Go's math.Log), plain IEEE double operations only, so the
 * device (gns_gomath.cuh gm_log) rounds identically. */
double or_det_log(double x) {
    const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10;
    const double L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01;
    const double L3 = 2.857142874366239149e-01, L4 = 2.222219843214978396e-01;
    const double L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01;
    const double L7 = 1.479819860511658591e-01;
    int ki;
    double f1 = frexp(x, &ki);
    if (f1 < 0.70710678118654752440) { f1 *= 2; ki--; }
    double f = f1 - 1;
    double k = (double)ki;
    double s = f / (2 + f);
    double s2 = s * s;
    double s4 = s2 * s2;
    double t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)));
    double t2 = s4 * (L2 + s4 * (L4 + s4 * L6));
    double R = t1 + t2;
    double hfsq = 0.5 * f * f;
    return k * Ln2Hi - ((hfsq - (s * (hfsq + R) + k * Ln2Lo)) - f);
}

/* log(1 - p) for 0 < p < 1 (series below 1e-4). */
double or_det_log1m(double p) {
    if (p < 1e-4) {
        double t = p * p;
        double r = p + t * 0.5;
        r = r + t * p * (1.0 / 3.0);
        return -r;
    }
    return or_det_log(1.0 - p);
}

/* super_spread.go:207-233 for one (packet, row) after sampling passed.
 * Owner (or empty) counter: every remaining iteration increments (:211-220).
 * Foreign counter: iteration t decrements with probability b^-val (:222-227);
 * the declared generator draws the number of failed iterations before the
 * next decrement as a geometric waiting time (one uniform per decrement,
 * draw = 1, 2, ...), the same law as one uniform per iteration. */
static void ss_mv(uint32_t *val, uint8_t *key, const uint8_t *flow, uint32_t K, int64_t vv, double b,
                  uint64_t rng_seed, uint64_t pkt, uint32_t row) {
    uint32_t draw = 1;
    while (vv > 0) {
        if (*val == 0 || memcmp(key, flow, K) == 0) {
            if (*val == 0) memcpy(key, flow, K);
            *val = (uint32_t)((uint64_t)*val + (uint64_t)vv);
            return;
        }
        double ppp = or_go_pow(b, -(double)*val); /* :222 */
        if (!(ppp > 0)) return;                   /* underflow: no decrement can happen */
        if (ppp >= 1) {                           /* b <= 1: every iteration decrements */
            int64_t k = (int64_t)*val < vv ? (int64_t)*val : vv;
            *val -= (uint32_t)k;
            vv -= k;
            continue;
        }
        double u = or_ss_uniform(rng_seed, pkt, row, draw++);
        double q = or_det_log(1.0 - u) / or_det_log1m(ppp); /* failures before the decrement */
        if (!(q < (double)vv)) return;
        vv -= (int64_t)floor(q) + 1;
        *val -= 1;
    }
}

struct or_ss {
    uint32_t d, w, thr, m, size, maxv, Kf, Ke;
    double base, b;
    uint32_t *seed;
    uint64_t hll_master, rng_seed, pkt;
    uint8_t *regs;    /* [d*w*m] GeneralHLL.hll (values <= maxValue <= 255) */
    double *pbits;    /* [d*w]   GeneralHLL.pbits */
    uint32_t *values; /* [d*w]   SuperSpread.values */
    uint8_t *keys;    /* [d*w*Kf] SuperSpread.keys */
};

or_ss *or_ss_new(uint32_t width, uint32_t depth, uint32_t threshold, uint32_t m, uint32_t size,
                 double base, double b, uint32_t Kf, uint32_t Ke, const uint32_t *seeds,
                 uint64_t hll_master, uint64_t rng_seed) {
    /* defaults: super_spread.go:12-20,129-149 */
    if (width == 0) width = 1u << 20;
    if (depth == 0) depth = 3;
    if (threshold == 0) threshold = 4096;
    if (m == 0) m = 128;
    if (size == 0) size = 5;
    if (base == 0) base = 0.5;
    if (b == 0) b = 1.08;
    if (size > 8) return NULL;
    or_ss *ss = (or_ss *)calloc(1, sizeof(or_ss));
    ss->d = depth; ss->w = width; ss->thr = threshold; ss->m = m; ss->size = size;
    ss->maxv = (1u << size) - 1; /* :41 */
    ss->base = base; ss->b = b; ss->Kf = Kf; ss->Ke = Ke;
    ss->seed = (uint32_t *)malloc(4 * depth);
    memcpy(ss->seed, seeds, 4 * depth);
    ss->hll_master = hll_master; ss->rng_seed = rng_seed;
    size_t cells = (size_t)depth * width;
    ss->regs = (uint8_t *)calloc(cells * m, 1);
    ss->pbits = (double *)malloc(sizeof(double) * cells);
    for (size_t c = 0; c < cells; c++) ss->pbits[c] = 1.0; /* :44 */
    ss->values = (uint32_t *)calloc(cells, 4);
    ss->keys = (uint8_t *)calloc(cells * (Kf ? Kf : 1), 1);
    return ss;
}

void or_ss_free(or_ss *ss) {
    if (!ss) return;
    free(ss->seed); free(ss->regs); free(ss->pbits); free(ss->values); free(ss->keys); free(ss);
}

uint64_t or_ss_packets(const or_ss *ss) { return ss->pkt; }

static inline uint32_t clz32_go(uint32_t x) { return x ? (uint32_t)__builtin_clz(x) : 32; } /* :54-64 */

/* super_spread.go:84-111: returns p_before or -1 */
static double ss_encode(or_ss *ss, size_t cell, const uint8_t *merged, uint32_t mlen) {
    uint32_t s0, s1;
    or_ss_hll_seeds(ss->hll_master, cell, &s0, &s1);
    uint32_t lz = clz32_go(or_mm3(merged, mlen, s0)) + 1; /* :66-70 geometricHash */
    if (lz > ss->maxv) lz = ss->maxv;
    uint32_t idx = or_mm3(merged, mlen, s1) % ss->m; /* :87-88 */
    uint8_t *reg = ss->regs + cell * ss->m + idx;
    uint32_t old = *reg;
    if (lz <= old) return -1.0; /* :91-93 */
    *reg = (uint8_t)lz;          /* :95-103 */
    double result = ss->pbits[cell]; /* :105 */
    ss->pbits[cell] = ss->pbits[cell] + (-or_go_pow(ss->base, (double)old) / (double)ss->m); /* :106 */
    if (lz < ss->maxv)
        ss->pbits[cell] = ss->pbits[cell] + or_go_pow(ss->base, (double)lz) / (double)ss->m; /* :107-109 */
    return result;
}

/* super_spread.go:182-235, one worker; rand.Float64() -> or_ss_uniform(). */
void or_ss_insert(or_ss *ss, const uint8_t *flow, const uint8_t *elem) {
    uint8_t merged[160];
    uint32_t mlen = ss->Kf + ss->Ke;
    memcpy(merged, flow, ss->Kf);
    memcpy(merged + ss->Kf, elem, ss->Ke);
    uint64_t pkt = ss->pkt++;
    for (uint32_t i = 0; i < ss->d; i++) {
        size_t cell = (size_t)i * ss->w + or_mm3(flow, ss->Kf, ss->seed[i]) % ss->w; /* :193 */
        double tempP = ss_encode(ss, cell, merged, mlen);
        if (tempP == -1.0) continue; /* :196-198 */
        double inv = 1.0 / tempP;
        double pCU = inv / ceil(inv); /* :200 */
        if (or_ss_uniform(ss->rng_seed, pkt, i, 0) >= pCU) continue; /* :201-204 */
        double cv = ceil(inv);
        /* :206 int(math.Ceil(1.0/tempP)); amd64 maps out-of-range to MinInt64 */
        int64_t tempVV = (cv < 9223372036854775808.0) ? (int64_t)cv : INT64_MIN;
        ss_mv(&ss->values[cell], ss->keys + cell * ss->Kf, flow, ss->Kf, tempVV, ss->b, ss->rng_seed, pkt, i);
    }
}

void or_ss_insert_batch(or_ss *ss, const uint8_t *flows, uint32_t fstride, const uint8_t *elems,
                        uint32_t estride, uint64_t n) {
    for (uint64_t p = 0; p < n; p++) or_ss_insert(ss, flows + p * fstride, elems + p * estride);
}

/* Task.ProcessPacket over 64-byte records (task.go:156-169, parser.go:23-67).
 * Every record advances the declared generator's packet index, also the ones
 * the parser drops (the engine's convention). */
uint64_t or_ss_insert_hdr64(or_ss *ss, const uint8_t *hdr, const uint32_t *wirelen, uint64_t n,
                            const uint8_t *ffields, uint32_t nff, const uint8_t *efields, uint32_t nef) {
    uint8_t fk[64], ek[64];
    uint64_t done = 0;
    for (uint64_t p = 0; p < n; p++) {
        or_tuple t;
        if (or_parse_hdr64_len(hdr + p * 64, wirelen[p], &t) != OR_PARSE_OK) {
            ss->pkt++;
            continue;
        }
        or_encode_key(ffields, nff, &t, fk);
        or_encode_key(efields, nef, &t, ek);
        or_ss_insert(ss, fk, ek);
        done++;
    }
    return done;
}

static uint32_t ss_estimate(const or_ss *ss, const uint8_t *flow) {
    uint32_t est = 0;
    for (uint32_t i = 0; i < ss->d; i++) {
        size_t cell = (size_t)i * ss->w + or_mm3(flow, ss->Kf, ss->seed[i]) % ss->w;
        if (memcmp(ss->keys + cell * ss->Kf, flow, ss->Kf) == 0 && ss->values[cell] > est)
            est = ss->values[cell];
    }
    return est;
}

/* super_spread.go:238-249 */
uint64_t or_ss_query(const or_ss *ss, const uint8_t *flow) {
    uint32_t e = ss_estimate(ss, flow);
    return e > 1 ? e : 1;
}

/* super_spread.go:254-294 */
uint32_t or_ss_heavy(const or_ss *ss, uint8_t *flows, uint32_t *vals, uint32_t cap) {
    size_t cells = (size_t)ss->d * ss->w;
    hh_item *it = (hh_item *)malloc(sizeof(hh_item) * (cells ? cells : 1));
    size_t n = 0;
    for (size_t c = 0; c < cells; c++) {
        if (ss->values[c] > 0) {
            it[n].fp = ss->keys + c * ss->Kf;
            it[n].v = ss_estimate(ss, it[n].fp); /* re-query (:266-276) */
            n++;
        }
    }
    uint32_t r = hh_finish(it, n, ss->Kf, ss->thr, flows, vals, cap);
    free(it);
    return r;
}

void or_ss_export(const or_ss *ss, uint32_t *values, uint8_t *keys, uint8_t *regs, double *pbits) {
    size_t cells = (size_t)ss->d * ss->w;
    if (values) memcpy(values, ss->values, cells * 4);
    if (keys) memcpy(keys, ss->keys, cells * ss->Kf);
    if (regs) memcpy(regs, ss->regs, cells * ss->m);
    if (pbits) memcpy(pbits, ss->pbits, cells * sizeof(double));
}

/* super_spread.go:297-311 (pbits is not reset by the reference either) */
void or_ss_reset(or_ss *ss) {
    size_t cells = (size_t)ss->d * ss->w;
    memset(ss->regs, 0, cells * ss->m);
    memset(ss->keys, 0, cells * ss->Kf);
    memset(ss->values, 0, cells * 4);
}
