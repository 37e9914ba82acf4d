// gns_thrift.hip -- device decode of Thrift PacketInfo batches (the NATS live
// path) into the 64-byte pre-parsed record format that every
// engine's fused-parse entry point consumes (ethertype 0x88B5).
// One thread decodes one message (gns_thrift.cuh).  A message the reference
// would reject (UnmarshalPacketInfo error -> logged and dropped,
// stream_aggregator.go:84-90) becomes a record with ethertype 0x0806, which
// the parser drops and counts like any other non-IP record.
#include <algorithm>

#include "gns_common.hpp"
#include "gns_thrift.cuh"

namespace gns {

// record byte 15 / 53: 4 for a 4-byte net.IP, 6 for 16 bytes, 0 otherwise
__device__ __forceinline__ uint32_t ip_code(uint32_t len) { return len == 4u ? 4u : (len == 16u ? 6u : 0u); }

__global__ __launch_bounds__(256) void k_thrift_decode(const uint8_t *buf, uint64_t buf_bytes, const uint64_t *offs,
                                                       uint64_t n, uint32_t *hdr, uint32_t *wirelen, int64_t *ts,
                                                       unsigned long long *bad) {
    const uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= n) return;
    const uint64_t o0 = offs[p], o1 = offs[p + 1];
    ThriftPacket pk{};
    bool ok = o0 <= o1 && o1 <= buf_bytes && o1 - o0 <= 0xFFFFFFFFull;
    const uint8_t *msg = buf + (ok ? o0 : 0);
    uint8_t b[64];
#pragma unroll
    for (int i = 0; i < 64; i++) b[i] = 0;
    // Fast path: the 70-byte message MarshalPacketInfo writes for an IPv4
    // PacketInfo (fields in id order, 4-byte IPs).  Aligned word loads +
    // v_alignbyte realignment; every header byte of the layout is checked, so
    // a message takes this path only if the full decoder would read exactly
    // these fields from it (anything else falls through to thrift_packet_info).
    bool fast = ok && o1 - o0 == 70 && (o0 & ~3ull) + 76 <= ((buf_bytes + 15) & ~15ull);
    if (fast) {
        const uint32_t *wp = reinterpret_cast<const uint32_t *>(buf + (o0 & ~3ull));
        const uint32_t sh = (uint32_t)(o0 & 3u);
        uint32_t w[19], m[18];
#pragma unroll
        for (int i = 0; i < 19; i++) w[i] = wp[i];
#pragma unroll
        for (int i = 0; i < 18; i++) m[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], sh);
        auto B = [&](int k) -> uint32_t { return (m[k >> 2] >> (8 * (k & 3))) & 0xFFu; };
        auto be32 = [&](int k) -> uint32_t { return B(k) << 24 | B(k + 1) << 16 | B(k + 2) << 8 | B(k + 3); };
        const uint32_t hdrs = (B(0) ^ 0x0A) | B(1) | (B(2) ^ 1) | (B(11) ^ 0x0C) | B(12) | (B(13) ^ 2) |
                              (B(14) ^ 0x0B) | B(15) | (B(16) ^ 1) | (be32(17) ^ 4) |
                              (B(25) ^ 0x0B) | B(26) | (B(27) ^ 2) | (be32(28) ^ 4) |
                              (B(36) ^ 8) | B(37) | (B(38) ^ 3) | (B(43) ^ 8) | B(44) | (B(45) ^ 4) |
                              (B(50) ^ 8) | B(51) | (B(52) ^ 5) | B(57) | (B(58) ^ 0x0A) | B(59) | (B(60) ^ 3) | B(69);
        fast = hdrs == 0;
        if (fast) {
            pk.ts = (int64_t)((uint64_t)be32(3) << 32 | be32(7));
            pk.length = (int64_t)((uint64_t)be32(61) << 32 | be32(65));
            pk.src_len = 4; pk.dst_len = 4;
            pk.sport = (int32_t)be32(39); pk.dport = (int32_t)be32(46); pk.proto = (int32_t)be32(53);
#pragma unroll
            for (int i = 0; i < 4; i++) { b[16 + i] = (uint8_t)B(21 + i); b[32 + i] = (uint8_t)B(32 + i); }
        }
    }
    if (ok && !fast) ok = thrift_packet_info(msg, (uint32_t)(o1 - o0), pk);
    if (ok) {
        b[12] = 0x88; b[13] = 0xB5; b[14] = 1;
        b[15] = (uint8_t)ip_code(pk.src_len);
        b[53] = (uint8_t)ip_code(pk.dst_len);
        // EncodeFlow copies min(len, 16) bytes of each net.IP into its slot (task.go:281-286)
        if (!fast) {
            const uint32_t ls = min(pk.src_len, 16u), ld = min(pk.dst_len, 16u);
            for (uint32_t i = 0; i < ls; i++) b[16 + i] = msg[pk.src_off + i];
            for (uint32_t i = 0; i < ld; i++) b[32 + i] = msg[pk.dst_off + i];
        }
        const uint32_t sp = (uint16_t)pk.sport, dp = (uint16_t)pk.dport;  // uint16(int32), packetcodec.go:90-91
        b[48] = (uint8_t)(sp >> 8); b[49] = (uint8_t)sp;
        b[50] = (uint8_t)(dp >> 8); b[51] = (uint8_t)dp;
        b[52] = (uint8_t)pk.proto;  // uint8(int32)
    } else {
        b[12] = 0x08; b[13] = 0x06;  // not an IP packet: dropped
        atomicAdd(bad, 1ull);
    }
    uint4 *o = reinterpret_cast<uint4 *>(hdr + p * 16);
#pragma unroll
    for (int q = 0; q < 4; q++) {
        uint32_t w[4];
#pragma unroll
        for (int k = 0; k < 4; k++)
            w[k] = (uint32_t)b[16 * q + 4 * k] | (uint32_t)b[16 * q + 4 * k + 1] << 8 |
                   (uint32_t)b[16 * q + 4 * k + 2] << 16 | (uint32_t)b[16 * q + 4 * k + 3] << 24;
        o[q] = make_uint4(w[0], w[1], w[2], w[3]);
    }
    wirelen[p] = ok ? (uint32_t)(uint64_t)pk.length : 0u;  // uint32(int(Length)), task.go:168
    ts[p] = ok ? pk.ts : 0;
}

}  // namespace gns

using namespace gns;

extern "C" int gns_thrift_decode(const uint8_t *buf, uint64_t buf_bytes, const uint64_t *offsets, uint64_t n,
                                 uint8_t *hdr_out, uint32_t *wirelen_out, int64_t *ts_out, uint64_t *n_bad,
                                 gns_mem where, int device) {
    if (n && (!buf || !offsets || !hdr_out || !wirelen_out || !ts_out)) { set_error("null argument"); return GNS_E_ARG; }
    (void)hipGetLastError();  // clear a stale error of an earlier runtime call on this thread
    GNS_HIP(hipSetDevice(device));
    if (n == 0) { if (n_bad) *n_bad = 0; return GNS_OK; }
    const uint8_t *dbuf = buf;
    const uint64_t *doff = offsets;
    uint8_t *tmp = nullptr;
    unsigned long long *dbad = nullptr;
    if (where == GNS_MEM_HOST) {
        if (offsets[n] > buf_bytes) { set_error("offsets[n] = %llu beyond the %llu-byte buffer",
                                                (unsigned long long)offsets[n], (unsigned long long)buf_bytes);
                                      return GNS_E_ARG; }
        const size_t ob = (n + 1) * 8, bb = (buf_bytes + 15) & ~uint64_t(15);
        GNS_TRY(dalloc(reinterpret_cast<void **>(&tmp), ob + bb));
        if (hipMemcpy(tmp, offsets, ob, hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(tmp + ob, buf, buf_bytes, hipMemcpyHostToDevice) != hipSuccess) {
            dfree(tmp);
            set_error("thrift decode: H2D copy failed");
            return GNS_E_HIP;
        }
        doff = reinterpret_cast<const uint64_t *>(tmp);
        dbuf = tmp + ob;
    }
    int rc = dalloc(reinterpret_cast<void **>(&dbad), 8);
    if (rc) { dfree(tmp); return rc; }
    hipError_t e = hipMemset(dbad, 0, 8);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_thrift_decode, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, nullptr, dbuf, buf_bytes,
                           doff, n, reinterpret_cast<uint32_t *>(hdr_out), wirelen_out, ts_out, dbad);
        e = hipGetLastError();
    }
    unsigned long long hb = 0;
    if (e == hipSuccess) e = hipMemcpy(&hb, dbad, 8, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    dfree(tmp);
    dfree(dbad);
    if (e != hipSuccess) { set_error("thrift decode: %s", hipGetErrorString(e)); return GNS_E_HIP; }
    if (n_bad) *n_bad = hb;
    return GNS_OK;
}
