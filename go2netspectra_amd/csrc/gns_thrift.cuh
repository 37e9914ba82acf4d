// gns_thrift.cuh -- Thrift binary-protocol decode of traffic.thrift PacketInfo
// messages (the NATS live path: internal/probe/packetcodec.go:97-108,
// UnmarshalPacketInfo; api/gen/thrift/v1/traffic.go:71-160,399-470 generated
// readers; apache/thrift v0.22.0 lib/go TBinaryProtocol + Skip).
//
// Shared by the device decoder (gns_thrift.hip); written against a byte
// pointer and a length so one thread decodes one message.
//   PacketInfo { 1: i64 timestamp_unix_nano, 2: FiveTuple five_tuple, 3: i64 length }
//   FiveTuple  { 1: binary src_ip, 2: binary dst_ip, 3: i32 src_port,
//                4: i32 dst_port, 5: i32 protocol }      (all required)
// Decode rules restated from the generated code and the library:
//   * fields in any order; a field whose id is known but whose wire type
//     differs is skipped; unknown ids are skipped; the last occurrence wins,
//     and a repeated five_tuple starts from an empty FiveTuple;
//   * Skip handles every wire type with a depth budget of 64 per Skip call;
//     unknown wire types, negative sizes and reads past the end are errors;
//   * missing required fields are errors; bytes after the final STOP are
//     ignored (TDeserializer does not check for trailing data).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gns {

enum TType : uint32_t {
    TT_STOP = 0, TT_VOID = 1, TT_BOOL = 2, TT_BYTE = 3, TT_DOUBLE = 4, TT_I16 = 6, TT_I32 = 8,
    TT_I64 = 10, TT_STRING = 11, TT_STRUCT = 12, TT_MAP = 13, TT_SET = 14, TT_LIST = 15, TT_UUID = 16
};

struct TReader {
    const uint8_t *p;
    uint32_t n, off;
    bool ok;

    __host__ __device__ bool need(uint32_t k) {
        if (!ok || n - off < k) { ok = false; return false; }
        return true;
    }
    __host__ __device__ uint32_t u8() {
        if (!need(1)) return 0;
        return p[off++];
    }
    __host__ __device__ uint32_t be16() {
        if (!need(2)) return 0;
        const uint32_t v = (uint32_t)p[off] << 8 | p[off + 1];
        off += 2;
        return v;
    }
    __host__ __device__ uint32_t be32() {
        if (!need(4)) return 0;
        const uint32_t v = (uint32_t)p[off] << 24 | (uint32_t)p[off + 1] << 16 | (uint32_t)p[off + 2] << 8 | p[off + 3];
        off += 4;
        return v;
    }
    __host__ __device__ uint64_t be64() {
        const uint64_t hi = be32();
        return hi << 32 | be32();
    }
    __host__ __device__ void skip(uint32_t k) {
        if (need(k)) off += k;
    }
};

// Skip one value of wire type t (thrift lib/go protocol.go Skip, depth 64).
__host__ __device__ inline bool thrift_skip(TReader &r, uint32_t t) {
    struct Frame { uint8_t kind, a, b, pad; int32_t left; };  // kind 0 struct, 1 list/set, 2 map
    Frame st[64];
    int sp = 0;
    uint32_t cur = t;
    for (;;) {
        // value of type cur at nesting sp: Skip(..., 64 - sp)
        if (sp >= 64) return false;
        switch (cur) {
        case TT_BOOL: case TT_BYTE: r.skip(1); break;
        case TT_I16: r.skip(2); break;
        case TT_I32: r.skip(4); break;
        case TT_I64: case TT_DOUBLE: r.skip(8); break;
        case TT_UUID: r.skip(16); break;
        case TT_STRING: {
            const int32_t sz = (int32_t)r.be32();
            if (!r.ok || sz < 0) return false;
            r.skip((uint32_t)sz);
            break;
        }
        case TT_STRUCT: st[sp++] = Frame{0, 0, 0, 0, 0}; break;
        case TT_LIST: case TT_SET: {
            const uint32_t et = r.u8();
            const int32_t sz = (int32_t)r.be32();
            if (!r.ok || sz < 0) return false;
            st[sp++] = Frame{1, (uint8_t)et, 0, 0, sz};
            break;
        }
        case TT_MAP: {
            const uint32_t kt = r.u8(), vt = r.u8();
            const int32_t sz = (int32_t)r.be32();
            if (!r.ok || sz < 0) return false;
            // 2*sz items, alternating key / value; sz < 2^31 so 2*sz fits u32
            st[sp++] = Frame{2, (uint8_t)kt, (uint8_t)vt, 0, sz};
            st[sp - 1].pad = 0;  // 0: next is a key, 1: next is a value
            break;
        }
        default: return false;  // unknown data type
        }
        if (!r.ok) return false;
        // next value inside the innermost open frame
        for (;;) {
            if (sp == 0) return true;
            Frame &f = st[sp - 1];
            if (f.kind == 0) {
                const uint32_t ft = r.u8();
                if (!r.ok) return false;
                if (ft == TT_STOP) { sp--; continue; }
                r.be16();
                if (!r.ok) return false;
                cur = ft;
                break;
            }
            if (f.kind == 1) {
                if (f.left == 0) { sp--; continue; }
                f.left--;
                cur = f.a;
                break;
            }
            if (f.left == 0) { sp--; continue; }  // map
            if (f.pad == 0) { cur = f.a; f.pad = 1; }
            else { cur = f.b; f.pad = 0; f.left--; }
            break;
        }
    }
}

struct ThriftPacket {
    int64_t ts, length;
    uint32_t src_off, src_len, dst_off, dst_len;
    int32_t sport, dport, proto;
};

// FiveTuple.Read (traffic.go:71-160)
__host__ __device__ inline bool thrift_five_tuple(TReader &r, ThriftPacket &pk) {
    bool s1 = false, s2 = false, s3 = false, s4 = false, s5 = false;
    pk.src_off = pk.dst_off = 0; pk.src_len = pk.dst_len = 0;
    pk.sport = pk.dport = pk.proto = 0;
    for (;;) {
        const uint32_t t = r.u8();
        if (!r.ok) return false;
        if (t == TT_STOP) break;
        const uint32_t id = r.be16();
        if (!r.ok) return false;
        if ((id == 1 || id == 2) && t == TT_STRING) {
            const int32_t sz = (int32_t)r.be32();
            if (!r.ok || sz < 0) return false;
            const uint32_t o = r.off;
            r.skip((uint32_t)sz);
            if (!r.ok) return false;
            if (id == 1) { pk.src_off = o; pk.src_len = (uint32_t)sz; s1 = true; }
            else { pk.dst_off = o; pk.dst_len = (uint32_t)sz; s2 = true; }
        } else if (id >= 3 && id <= 5 && t == TT_I32) {
            const int32_t v = (int32_t)r.be32();
            if (!r.ok) return false;
            if (id == 3) { pk.sport = v; s3 = true; }
            else if (id == 4) { pk.dport = v; s4 = true; }
            else { pk.proto = v; s5 = true; }
        } else if (!thrift_skip(r, t)) {
            return false;
        }
    }
    return s1 && s2 && s3 && s4 && s5;
}

// UnmarshalPacketInfo (packetcodec.go:97-108) + packetInfoFromThrift (:76-95)
__host__ __device__ inline bool thrift_packet_info(const uint8_t *msg, uint32_t len, ThriftPacket &pk) {
    TReader r{msg, len, 0, true};
    bool s1 = false, s2 = false, s3 = false;
    pk.ts = 0; pk.length = 0;
    for (;;) {
        const uint32_t t = r.u8();
        if (!r.ok) return false;
        if (t == TT_STOP) break;
        const uint32_t id = r.be16();
        if (!r.ok) return false;
        if ((id == 1 || id == 3) && t == TT_I64) {
            const int64_t v = (int64_t)r.be64();
            if (!r.ok) return false;
            if (id == 1) { pk.ts = v; s1 = true; }
            else { pk.length = v; s3 = true; }
        } else if (id == 2 && t == TT_STRUCT) {
            if (!thrift_five_tuple(r, pk)) return false;  // ReadField2: a fresh FiveTuple
            s2 = true;
        } else if (!thrift_skip(r, t)) {
            return false;
        }
    }
    return s1 && s2 && s3;
}

}  // namespace gns
