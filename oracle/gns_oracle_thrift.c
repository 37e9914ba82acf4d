/*
 * gns_oracle_thrift.c -- CPU ORACLE (test infrastructure, never product code)
 * for the NATS live path's message decode: internal/probe/packetcodec.go:97-108
 * (UnmarshalPacketInfo) over the generated readers in
 * api/gen/thrift/v1/traffic.go:71-160 (FiveTuple.Read) and :399-470
 * (PacketInfo.Read), with apache/thrift v0.22.0 lib/go TBinaryProtocol and the
 * recursive Skip(ctx, prot, type, maxDepth = 64) (protocol.go), which is not
 * vendored in the reference and is restated here from its published source.
 *
 * Written as the Go code is structured (recursive Skip, one reader per struct),
 * independently of the engine's iterative decoder (gns_thrift.cuh).
 */
#include "gns_oracle.h"

#include <string.h>

typedef struct {
    const uint8_t *p;
    uint64_t n, off;
    int err;
} rd;

static int rd_bytes(rd *r, uint64_t k, const uint8_t **out) {
    if (r->err || r->n - r->off < k) { r->err = 1; return 0; }
    if (out) *out = r->p + r->off;
    r->off += k;
    return 1;
}
static uint32_t rd_byte(rd *r) { const uint8_t *b; return rd_bytes(r, 1, &b) ? b[0] : 0; }
static uint32_t rd_i16(rd *r) { const uint8_t *b; return rd_bytes(r, 2, &b) ? (uint32_t)(b[0] << 8 | b[1]) : 0; }
static uint32_t rd_i32(rd *r) {
    const uint8_t *b;
    if (!rd_bytes(r, 4, &b)) return 0;
    return (uint32_t)b[0] << 24 | (uint32_t)b[1] << 16 | (uint32_t)b[2] << 8 | b[3];
}
static uint64_t rd_i64(rd *r) { uint64_t hi = rd_i32(r); return hi << 32 | rd_i32(r); }

/* TBinaryProtocol.ReadBinary / ReadString: i32 size, negative or past the end -> error */
static int rd_binary(rd *r, const uint8_t **b, uint32_t *len) {
    int32_t sz = (int32_t)rd_i32(r);
    if (r->err || sz < 0) { r->err = 1; return 0; }
    *len = (uint32_t)sz;
    return rd_bytes(r, (uint64_t)sz, b);
}

enum { T_STOP = 0, T_BOOL = 2, T_BYTE = 3, T_DOUBLE = 4, T_I16 = 6, T_I32 = 8, T_I64 = 10, T_STRING = 11,
       T_STRUCT = 12, T_MAP = 13, T_SET = 14, T_LIST = 15, T_UUID = 16 };

/* protocol.go Skip(ctx, self, fieldType, maxDepth) */
static int skip(rd *r, uint32_t t, int max_depth) {
    if (max_depth <= 0) return 0;
    switch (t) {
    case T_BOOL: case T_BYTE: rd_bytes(r, 1, NULL); return !r->err;
    case T_I16: rd_bytes(r, 2, NULL); return !r->err;
    case T_I32: rd_bytes(r, 4, NULL); return !r->err;
    case T_I64: case T_DOUBLE: rd_bytes(r, 8, NULL); return !r->err;
    case T_UUID: rd_bytes(r, 16, NULL); return !r->err;
    case T_STRING: { const uint8_t *b; uint32_t l; return rd_binary(r, &b, &l); }
    case T_STRUCT:
        for (;;) {
            uint32_t ft = rd_byte(r);
            if (r->err) return 0;
            if (ft == T_STOP) return 1;
            rd_i16(r);
            if (r->err) return 0;
            if (!skip(r, ft, max_depth - 1)) return 0;
        }
    case T_MAP: {
        uint32_t kt = rd_byte(r), vt = rd_byte(r);
        int32_t sz = (int32_t)rd_i32(r);
        if (r->err || sz < 0) return 0;
        for (int32_t i = 0; i < sz; i++) {
            if (!skip(r, kt, max_depth - 1)) return 0;
            if (!skip(r, vt, max_depth - 1)) return 0;
        }
        return 1;
    }
    case T_SET: case T_LIST: {
        uint32_t et = rd_byte(r);
        int32_t sz = (int32_t)rd_i32(r);
        if (r->err || sz < 0) return 0;
        for (int32_t i = 0; i < sz; i++)
            if (!skip(r, et, max_depth - 1)) return 0;
        return 1;
    }
    default:
        return 0; /* unknown data type */
    }
}

typedef struct {
    const uint8_t *src, *dst;
    uint32_t src_len, dst_len;
    int32_t sport, dport, proto;
} five_tuple;

/* traffic.go:71-160 */
static int read_five_tuple(rd *r, five_tuple *ft) {
    int s1 = 0, s2 = 0, s3 = 0, s4 = 0, s5 = 0;
    memset(ft, 0, sizeof(*ft));
    for (;;) {
        uint32_t t = rd_byte(r);
        if (r->err) return 0;
        if (t == T_STOP) break;
        uint32_t id = rd_i16(r);
        if (r->err) return 0;
        switch (id) {
        case 1:
            if (t == T_STRING) { if (!rd_binary(r, &ft->src, &ft->src_len)) return 0; s1 = 1; }
            else if (!skip(r, t, 64)) return 0;
            break;
        case 2:
            if (t == T_STRING) { if (!rd_binary(r, &ft->dst, &ft->dst_len)) return 0; s2 = 1; }
            else if (!skip(r, t, 64)) return 0;
            break;
        case 3:
            if (t == T_I32) { ft->sport = (int32_t)rd_i32(r); if (r->err) return 0; s3 = 1; }
            else if (!skip(r, t, 64)) return 0;
            break;
        case 4:
            if (t == T_I32) { ft->dport = (int32_t)rd_i32(r); if (r->err) return 0; s4 = 1; }
            else if (!skip(r, t, 64)) return 0;
            break;
        case 5:
            if (t == T_I32) { ft->proto = (int32_t)rd_i32(r); if (r->err) return 0; s5 = 1; }
            else if (!skip(r, t, 64)) return 0;
            break;
        default:
            if (!skip(r, t, 64)) return 0;
        }
    }
    return s1 && s2 && s3 && s4 && s5;
}

/* PacketInfo.Read (traffic.go:399-470) + packetInfoFromThrift (packetcodec.go:76-95).
 * On success fills the tuple (IP slots as EncodeFlow copies them: min(len,16)
 * bytes), the version code of each IP (4: 4 bytes, 6: 16 bytes, 0: other),
 * the wire length (i64) and the timestamp.  Returns 1 ok, 0 rejected. */
int or_thrift_decode_one(const uint8_t *msg, uint64_t len, or_tuple *t, uint8_t *dst_ver, int64_t *length,
                         int64_t *ts) {
    rd r = {msg, len, 0, 0};
    int s1 = 0, s2 = 0, s3 = 0;
    five_tuple ft;
    memset(&ft, 0, sizeof(ft));
    for (;;) {
        uint32_t ty = rd_byte(&r);
        if (r.err) return 0;
        if (ty == T_STOP) break;
        uint32_t id = rd_i16(&r);
        if (r.err) return 0;
        switch (id) {
        case 1:
            if (ty == T_I64) { *ts = (int64_t)rd_i64(&r); if (r.err) return 0; s1 = 1; }
            else if (!skip(&r, ty, 64)) return 0;
            break;
        case 2:
            if (ty == T_STRUCT) { if (!read_five_tuple(&r, &ft)) return 0; s2 = 1; }
            else if (!skip(&r, ty, 64)) return 0;
            break;
        case 3:
            if (ty == T_I64) { *length = (int64_t)rd_i64(&r); if (r.err) return 0; s3 = 1; }
            else if (!skip(&r, ty, 64)) return 0;
            break;
        default:
            if (!skip(&r, ty, 64)) return 0;
        }
    }
    if (!(s1 && s2 && s3)) return 0;
    memset(t, 0, sizeof(*t));
    memcpy(t->src, ft.src, ft.src_len < 16 ? ft.src_len : 16);
    memcpy(t->dst, ft.dst, ft.dst_len < 16 ? ft.dst_len : 16);
    t->sport = (uint16_t)ft.sport;
    t->dport = (uint16_t)ft.dport;
    t->proto = (uint8_t)ft.proto;
    t->ipver = ft.src_len == 4 ? 4 : (ft.src_len == 16 ? 6 : 0);
    t->dst_ipver = ft.dst_len == 4 ? 4 : (ft.dst_len == 16 ? 6 : 0);
    *dst_ver = t->dst_ipver;
    return 1;
}

/* batch: ok[i], tuple arrays, lengths, timestamps; returns messages accepted */
uint64_t or_thrift_decode(const uint8_t *buf, const uint64_t *offsets, uint64_t n, uint8_t *ok, uint8_t *src16,
                          uint8_t *dst16, uint16_t *sport, uint16_t *dport, uint8_t *proto, uint8_t *sver,
                          uint8_t *dver, int64_t *length, int64_t *ts) {
    uint64_t good = 0;
    for (uint64_t i = 0; i < n; i++) {
        or_tuple t;
        int64_t ln = 0, tv = 0;
        uint8_t dv = 0;
        ok[i] = (uint8_t)or_thrift_decode_one(buf + offsets[i], offsets[i + 1] - offsets[i], &t, &dv, &ln, &tv);
        if (!ok[i]) memset(&t, 0, sizeof(t));
        memcpy(src16 + 16 * i, t.src, 16);
        memcpy(dst16 + 16 * i, t.dst, 16);
        sport[i] = t.sport; dport[i] = t.dport; proto[i] = t.proto;
        sver[i] = ok[i] ? t.ipver : 0;
        dver[i] = ok[i] ? dv : 0;
        length[i] = ok[i] ? ln : 0;
        ts[i] = ok[i] ? tv : 0;
        good += ok[i];
    }
    return good;
}
