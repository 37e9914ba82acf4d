// gns_synth.hip -- synthetic traffic for the benchmark and the parity tests
// (SURVEY.md §8d): a universe of F flows (splitmix64 5-tuples), Zipf(s) packet
// ranks over a random rank->flow permutation, wire lengths uniform 64..1518,
// 64-byte Ethernet/IPv4/TCP|UDP header records shaped like scripts/pcapgen
// (scripts/pcapgen/main.go:43-93).  Packet i is a pure function of
// (seeds, shard, i), so any sub-range can be regenerated on host or device.
//
// Sharding (multi-GPU): shard g of G keeps the flows whose SrcIP
// slot hashes to g (mm3(slot16, 0xA5A5A5A5) % G); its packet stream samples
// the Zipf law conditioned on those flows, i.e. exactly the sub-stream a
// flow-hash splitter would route to GPU g.
#include <algorithm>
#include <cmath>
#include <vector>

#include "gns_common.hpp"

namespace gns {

static inline uint64_t mix64_h(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t mix64_d(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static uint32_t mm3_host(const uint8_t *d, uint32_t len, uint32_t seed) {
    uint32_t h = seed;
    const uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
    auto rotl = [](uint32_t x, int r) { return (x << r) | (x >> (32 - r)); };
    uint32_t nb = len / 4;
    for (uint32_t i = 0; i < nb; i++) {
        uint32_t k;
        memcpy(&k, d + 4 * i, 4);
        k *= c1; k = rotl(k, 15); k *= c2;
        h ^= k; h = rotl(h, 13); h = h * 5 + 0xe6546b64u;
    }
    uint32_t k = 0;
    const uint8_t *t = d + 4 * nb;
    switch (len & 3) {
    case 3: k ^= (uint32_t)t[2] << 16; [[fallthrough]];
    case 2: k ^= (uint32_t)t[1] << 8; [[fallthrough]];
    case 1: k ^= t[0]; k *= c1; k = rotl(k, 15); k *= c2; h ^= k;
    }
    h ^= len;
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
    return h;
}

struct SynthDev {
    const uint32_t *src, *dst, *ports;  // ports = sport<<16 | dport
    const uint8_t *proto;
    const double *cdf;                   // inclusive CDF over shard flows (rank order)
    uint32_t nf;
    uint64_t rank_key, len_key;
    const double *dcdf;                  // fan-out mode: CDF over destinations (nd > 0)
    uint32_t nd;
    uint64_t dst_key;
};

__device__ __forceinline__ uint32_t cdf_search(const double *cdf, uint32_t n, double u) {
    uint32_t lo = 0, hi = n - 1;  // first j with cdf[j] > u
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (cdf[mid] > u) hi = mid; else lo = mid + 1;
    }
    return lo;
}

__global__ __launch_bounds__(256) void k_synth(SynthDev s, uint32_t *hdr, uint32_t *wirelen,
                                               uint64_t first, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint64_t pk = first + i;
    const double u = (double)(mix64_d(s.rank_key + pk * 0x9E3779B97F4A7C15ull) >> 11) * 0x1.0p-53;
    const uint32_t f = cdf_search(s.cdf, s.nf, u);
    const uint32_t len = 64u + (uint32_t)(mix64_d(s.len_key + pk * 0x9E3779B97F4A7C15ull) % 1455u);
    const uint32_t src = s.src[f], ports = s.ports[f];
    uint32_t dst = s.dst[f];
    if (s.nd) {  // per-packet destination: Zipf rank -> hashed address
        const uint64_t dk = mix64_d(s.dst_key + pk * 0x9E3779B97F4A7C15ull);
        const uint32_t r = cdf_search(s.dcdf, s.nd, (double)(dk >> 11) * 0x1.0p-53);
        dst = (uint32_t)mix64_d(0xD57D57ull + r);
    }
    const uint32_t proto = s.proto[f];
    uint8_t b[64];
#pragma unroll
    for (int j = 0; j < 64; j++) b[j] = 0;
    // Ethernet (pcapgen MACs)
    b[0] = 0x00; b[1] = 0x66; b[2] = 0x77; b[3] = 0x88; b[4] = 0x99; b[5] = 0xAA;
    b[6] = 0x00; b[7] = 0x11; b[8] = 0x22; b[9] = 0x33; b[10] = 0x44; b[11] = 0x55;
    b[12] = 0x08; b[13] = 0x00;
    // IPv4, IHL 5, DF
    const uint32_t tot = len - 14u;
    b[14] = 0x45; b[16] = tot >> 8; b[17] = tot & 0xFF;
    b[18] = (pk >> 8) & 0xFF; b[19] = pk & 0xFF; b[20] = 0x40; b[22] = 64; b[23] = (uint8_t)proto;
    b[26] = src >> 24; b[27] = src >> 16; b[28] = src >> 8; b[29] = src;
    b[30] = dst >> 24; b[31] = dst >> 16; b[32] = dst >> 8; b[33] = dst;
    const uint32_t sp = ports >> 16, dp = ports & 0xFFFF;
    b[34] = sp >> 8; b[35] = sp & 0xFF; b[36] = dp >> 8; b[37] = dp & 0xFF;
    if (proto == 6) {
        const uint32_t seq = (uint32_t)mix64_d(pk ^ 0xC0FFEEull);
        b[38] = seq >> 24; b[39] = seq >> 16; b[40] = seq >> 8; b[41] = seq;
        b[46] = 0x50; b[47] = 0x02; b[48] = 14600 >> 8; b[49] = 14600 & 0xFF;
    } else {
        const uint32_t ul = tot - 20u;
        b[38] = ul >> 8; b[39] = ul & 0xFF;
    }
    uint4 *o = reinterpret_cast<uint4 *>(hdr + i * 16);
#pragma unroll
    for (int q = 0; q < 4; q++) {
        uint32_t w[4];
#pragma unroll
        for (int k = 0; k < 4; k++)
            w[k] = (uint32_t)b[16 * q + 4 * k] | (uint32_t)b[16 * q + 4 * k + 1] << 8 |
                   (uint32_t)b[16 * q + 4 * k + 2] << 16 | (uint32_t)b[16 * q + 4 * k + 3] << 24;
        o[q] = make_uint4(w[0], w[1], w[2], w[3]);
    }
    wirelen[i] = len;
}

}  // namespace gns

using namespace gns;

struct gns_synth {
    int device = 0;
    SynthDev dev{};
    uint32_t *src = nullptr, *dst = nullptr, *ports = nullptr;
    uint8_t *proto = nullptr;
    double *cdf = nullptr, *dcdf = nullptr;
};

extern "C" {

int gns_synth_create(const gns_synth_params *p, gns_synth **out) {
    if (!p || !out) { set_error("null argument"); return GNS_E_ARG; }
    *out = nullptr;
    const uint32_t F = p->flows ? p->flows : (1u << 20);
    const double s = p->zipf_s != 0 ? p->zipf_s : 1.1;
    const uint64_t tseed = p->tuple_seed ? p->tuple_seed : 0x5EED0001ull;
    const uint64_t rseed = p->rank_seed ? p->rank_seed : 0x5EED0002ull;
    const uint64_t lseed = p->len_seed ? p->len_seed : 0x5EED0003ull;
    const uint32_t G = p->nshards ? p->nshards : 1, shard = p->shard;
    if (shard >= G) { set_error("shard %u >= nshards %u", shard, G); return GNS_E_ARG; }
    // flow universe
    std::vector<uint32_t> fsrc(F), fdst(F), fports(F);
    std::vector<uint8_t> fproto(F);
    uint64_t st = tseed;
    for (uint32_t f = 0; f < F; f++) {
        st += 0x9E3779B97F4A7C15ull; const uint64_t r1 = mix64_h(st);
        st += 0x9E3779B97F4A7C15ull; const uint64_t r2 = mix64_h(st);
        fsrc[f] = (uint32_t)r1; fdst[f] = (uint32_t)(r1 >> 32);
        uint32_t sp = (uint32_t)(r2 >> 16) & 0xFFFFu, dp = (uint32_t)r2 & 0xFFFFu;
        fproto[f] = ((r2 >> 32) % 10) < 8 ? 6 : 17;
        if (fproto[f] == 17) {  // keep UDP off the tunnel ports gopacket decodes further
            auto tun = [](uint32_t p) { return p == 4789u || p == 6081u || p == 2152u; };
            if (tun(sp)) sp += 1;
            if (tun(dp)) dp += 1;
        }
        fports[f] = sp << 16 | dp;
    }
    // rank -> flow permutation (Fisher-Yates)
    std::vector<uint32_t> perm(F);
    for (uint32_t i = 0; i < F; i++) perm[i] = i;
    uint64_t ps = rseed ^ 0xA0761D6478BD642Full;
    for (uint32_t i = F - 1; i > 0; i--) {
        ps += 0x9E3779B97F4A7C15ull;
        const uint32_t j = (uint32_t)(mix64_h(ps) % (uint64_t)(i + 1));
        std::swap(perm[i], perm[j]);
    }
    // shard filter on the SrcIP slot (16 bytes, IPv4 left-aligned)
    std::vector<uint32_t> keep;
    keep.reserve(F / G + 16);
    std::vector<double> w;
    for (uint32_t r = 0; r < F; r++) {
        const uint32_t f = perm[r];
        bool mine = true;
        if (G > 1) {
            uint8_t slot[16] = {0};
            slot[0] = fsrc[f] >> 24; slot[1] = fsrc[f] >> 16; slot[2] = fsrc[f] >> 8; slot[3] = fsrc[f];
            mine = mm3_host(slot, 16, 0xA5A5A5A5u) % G == shard;
        }
        if (mine) { keep.push_back(f); w.push_back(std::pow((double)(r + 1), -s)); }
    }
    const uint32_t nf = (uint32_t)keep.size();
    if (nf == 0) { set_error("shard has no flows"); return GNS_E_ARG; }
    std::vector<double> cdf(nf);
    double acc = 0;
    for (uint32_t i = 0; i < nf; i++) acc += w[i];
    double run = 0;
    for (uint32_t i = 0; i < nf; i++) { run += w[i]; cdf[i] = run / acc; }
    cdf[nf - 1] = 1.0;
    std::vector<uint32_t> ksrc(nf), kdst(nf), kports(nf);
    std::vector<uint8_t> kproto(nf);
    for (uint32_t i = 0; i < nf; i++) {
        ksrc[i] = fsrc[keep[i]]; kdst[i] = fdst[keep[i]]; kports[i] = fports[keep[i]]; kproto[i] = fproto[keep[i]];
    }
    if (hipSetDevice(p->device) != hipSuccess) { set_error("hipSetDevice failed"); return GNS_E_NODEV; }
    gns_synth *sy = new gns_synth();
    sy->device = p->device;
    int rc = GNS_OK;
    if ((rc = dalloc_t(&sy->src, nf)) || (rc = dalloc_t(&sy->dst, nf)) || (rc = dalloc_t(&sy->ports, nf)) ||
        (rc = dalloc_t(&sy->proto, nf)) || (rc = dalloc_t(&sy->cdf, nf))) {
        gns_synth_destroy(sy);
        return rc;
    }
    if (hipMemcpy(sy->src, ksrc.data(), nf * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(sy->dst, kdst.data(), nf * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(sy->ports, kports.data(), nf * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(sy->proto, kproto.data(), nf, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(sy->cdf, cdf.data(), nf * 8, hipMemcpyHostToDevice) != hipSuccess) {
        set_error("synth upload failed");
        gns_synth_destroy(sy);
        return GNS_E_HIP;
    }
    uint32_t nd = p->fanout;
    if (nd) {
        std::vector<double> dc(nd);
        double dacc = 0;
        for (uint32_t i = 0; i < nd; i++) dacc += std::pow((double)(i + 1), -s);
        double drun = 0;
        for (uint32_t i = 0; i < nd; i++) { drun += std::pow((double)(i + 1), -s); dc[i] = drun / dacc; }
        dc[nd - 1] = 1.0;
        if ((rc = dalloc_t(&sy->dcdf, nd)) != GNS_OK) { gns_synth_destroy(sy); return rc; }
        if (hipMemcpy(sy->dcdf, dc.data(), nd * 8, hipMemcpyHostToDevice) != hipSuccess) {
            set_error("synth upload failed");
            gns_synth_destroy(sy);
            return GNS_E_HIP;
        }
    }
    sy->dev = SynthDev{sy->src, sy->dst, sy->ports, sy->proto, sy->cdf, nf,
                       rseed + (uint64_t)shard * 0xD1B54A32D192ED03ull, lseed + (uint64_t)shard * 0x8CB92BA72F3D8DD7ull,
                       sy->dcdf, nd, rseed ^ 0x7F4A7C159E3779B9ull};
    *out = sy;
    return GNS_OK;
}

int gns_synth_destroy(gns_synth *s) {
    if (!s) return GNS_OK;
    dfree(s->src); dfree(s->dst); dfree(s->ports); dfree(s->proto); dfree(s->cdf); dfree(s->dcdf);
    delete s;
    return GNS_OK;
}

int gns_synth_fill(gns_synth *s, uint8_t *hdr_dev, uint32_t *wirelen_dev, uint64_t first, uint64_t n) {
    if (!s || (n && (!hdr_dev || !wirelen_dev))) { set_error("null argument"); return GNS_E_ARG; }
    (void)hipGetLastError();  // clear a stale error of an earlier runtime call on this thread
    GNS_HIP(hipSetDevice(s->device));
    const uint64_t step = 1ull << 26;
    for (uint64_t off = 0; off < n; off += step) {
        const uint64_t m = std::min(step, n - off);
        hipLaunchKernelGGL(k_synth, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, nullptr, s->dev,
                           reinterpret_cast<uint32_t *>(hdr_dev + off * 64), wirelen_dev + off, first + off, m);
        GNS_HIP(hipGetLastError());
    }
    GNS_HIP(hipDeviceSynchronize());
    return GNS_OK;
}

int gns_synth_flows(gns_synth *s, uint32_t *n_flows) {
    if (!s || !n_flows) return GNS_E_ARG;
    *n_flows = s->dev.nf;
    return GNS_OK;
}

}  // extern "C"
