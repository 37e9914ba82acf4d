// gns_records.hip -- 64-byte header records -> compact 16-byte records
// (IN_REC16, gns_keys.cuh) on the device.
//
// The host-inclusive path is PCIe-bound: a 64-byte record plus
// the wire length is 68 bytes per packet over the bus, while the device parser
// reads 26 of them.  A compact record carries exactly the canonical tuple the
// parser derives (the IPv4 slots, the ports, protocol and IP versions: tw[0],
// tw[4], tw[8], tw[9]) in 16 bytes, 20 with the wire length.  Records whose
// tuple does not fit (IPv6 addresses, shapes the device parser leaves
// unsupported) escape to a side array of the original 64-byte records, which
// the insert parses exactly as gns_*_insert_headers would; records without an
// IP layer become the drop class.  So an insert of the compact form is the same
// stream as the insert of the 64-byte form, packet for packet.
//
// The capture packer builds the same format on the host (gns_pack_pcap_compact);
// this kernel converts records that already sit in device memory (the
// synthetic stream, a decoded Thrift batch) -- the bench stages its
// host-resident windows with it.
#include "gns_common.hpp"

namespace gns {

// emb: the 16-byte form (wire length in word 3 bits 16..31; a tuple record is IPv4 both
// ways, any other tuple escapes); a wire length above 65535 raises *big
__global__ __launch_bounds__(256) void k_compact(const uint32_t *hdr, const uint32_t *wl, uint64_t n, uint4 *rec,
                                                 uint32_t *side, uint64_t side_cap, unsigned long long *nside,
                                                 int emb, unsigned long long *big) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t p0 = (uint64_t)blockIdx.x * 256; p0 < n; p0 += stride) {  // wave-uniform trip count
        const uint64_t p = p0 + threadIdx.x;
        const bool valid = p < n;
        uint32_t w[16];
        const uint64_t pc = valid ? p : n - 1;
        const uint4 *r = reinterpret_cast<const uint4 *>(hdr + pc * 16);
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint4 v = r[i];
            w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
        }
        uint32_t tw[10];
        const int st = parse_record_fast(w, wl[pc], valid, tw);
        const bool narrow = (tw[1] | tw[2] | tw[3] | tw[5] | tw[6] | tw[7]) == 0;
        const bool v4 = !emb || (tw[9] >> 16) == 0x0404u;
        const uint32_t cls = st == PARSE_DROP ? kRecDrop : ((st == PARSE_OK && narrow && v4) ? kRecTuple : kRecSide);
        const uint32_t wlp = wl[pc];
        if (emb && valid && wlp > 0xFFFFu) atomicAdd(big, 1ull);
        const uint32_t hi = emb ? wlp << 16 : 0u;  // the wire length in word 3 (16-byte form)
        // side slots: one global atomic per wave
        const uint64_t m = __ballot(valid && cls == kRecSide);
        unsigned long long base = 0;
        if (m) {
            const int leader = __ffsll((unsigned long long)m) - 1;
            if ((int)__lane_id() == leader) base = atomicAdd(nside, (unsigned long long)__popcll(m));
            base = __shfl(base, leader);
        }
        if (!valid) continue;
        uint4 o;
        if (cls == kRecTuple) {
            o = make_uint4(tw[0], tw[4], tw[8], emb ? ((tw[9] & 0xFFu) | hi) : tw[9]);
        } else if (cls == kRecDrop) {
            o = make_uint4(0u, 0u, 0u, kRecDrop << 8 | hi);
        } else {
            const uint64_t idx = base + __popcll(m & ((1ull << __lane_id()) - 1ull));
            o = make_uint4((uint32_t)idx, 0u, 0u, kRecSide << 8 | hi);
            if (idx < side_cap) {
                uint4 *q = reinterpret_cast<uint4 *>(side + idx * 16);
#pragma unroll
                for (int i = 0; i < 4; i++) q[i] = make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]);
            }
        }
        rec[p] = o;
    }
}

}  // namespace gns

using namespace gns;

static int compact_headers(const uint8_t *hdr, const uint32_t *wirelen, uint64_t n, uint8_t *rec16,
                           uint8_t *side64, uint64_t side_cap, uint64_t *n_side, int device, int emb) {
    if ((n && (!hdr || !wirelen || !rec16)) || (side_cap && !side64) || !n_side) {
        set_error("null argument");
        return GNS_E_ARG;
    }
    (void)hipGetLastError();
    GNS_HIP(hipSetDevice(device));
    *n_side = 0;
    if (n == 0) return GNS_OK;
    unsigned long long *cnt = nullptr;
    GNS_TRY(dalloc_t(&cnt, 2));
    unsigned long long h[2] = {0, 0};
    hipError_t e = hipMemsetAsync(cnt, 0, 16, 0);
    if (e == hipSuccess) {
        const unsigned grid = (unsigned)std::min<uint64_t>((n + 255) / 256, 8192);
        hipLaunchKernelGGL(k_compact, dim3(grid), dim3(256), 0, 0, reinterpret_cast<const uint32_t *>(hdr), wirelen, n,
                           reinterpret_cast<uint4 *>(rec16), reinterpret_cast<uint32_t *>(side64), side_cap, cnt,
                           emb, cnt + 1);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(h, cnt, 16, hipMemcpyDeviceToHost);
    dfree(cnt);
    if (e != hipSuccess) {
        set_error("gns_compact_headers: %s", hipGetErrorString(e));
        return GNS_E_HIP;
    }
    *n_side = h[0];
    if (h[1]) {
        set_error("%llu wire lengths above 65535: the 16-byte form cannot hold them (use the 20-byte form)", h[1]);
        return GNS_E_RANGE;
    }
    if (h[0] > side_cap) {
        set_error("%llu side records needed, room for %llu", h[0], (unsigned long long)side_cap);
        return GNS_E_RANGE;
    }
    return GNS_OK;
}

extern "C" int gns_compact_headers(const uint8_t *hdr, const uint32_t *wirelen, uint64_t n, uint8_t *rec16,
                                   uint8_t *side64, uint64_t side_cap, uint64_t *n_side, int device) {
    return compact_headers(hdr, wirelen, n, rec16, side64, side_cap, n_side, device, 0);
}

extern "C" int gns_compact_headers16(const uint8_t *hdr, const uint32_t *wirelen, uint64_t n, uint8_t *rec16,
                                     uint8_t *side64, uint64_t side_cap, uint64_t *n_side, int device) {
    return compact_headers(hdr, wirelen, n, rec16, side64, side_cap, n_side, device, 1);
}
