// gns_common.cpp -- host plumbing (see gns_common.hpp).
#include "gns_common.hpp"

#include <mutex>

namespace gns {

static thread_local std::string g_last_error;

void set_error(const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
}

int dalloc(void **p, size_t bytes) {
    *p = nullptr;
    hipError_t e = hipMalloc(p, bytes ? bytes : 16);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        set_error("hipMalloc(%zu bytes) failed: %s", bytes, hipGetErrorString(e));
        *p = nullptr;
        return GNS_E_OOM;
    }
    return GNS_OK;
}

void dfree(void *p) {
    if (p) (void)hipFree(p);
}

uint32_t layout_bytes(const gns_layout &l) {
    uint32_t k = 0;
    for (uint32_t i = 0; i < l.n_fields && i < 8; i++) {
        switch (l.fields[i]) {
        case GNS_F_SRCIP: case GNS_F_DSTIP: k += 16; break;
        case GNS_F_SRCPORT: case GNS_F_DSTPORT: k += 2; break;
        case GNS_F_PROTO: k += 1; break;
        default: break;  // unknown field names contribute nothing (task.go:335-336)
        }
    }
    return k;
}

int make_plan(const gns_layout &l, uint32_t key_bytes, KeyPlanN *kp) {
    memset(kp, 0, sizeof(*kp));
    if (l.n_fields > 8) { set_error("layout has %u fields (max 8)", l.n_fields); return GNS_E_ARG; }
    const uint32_t K = l.n_fields ? layout_bytes(l) : key_bytes;
    if (K > 37) {  // task.go:74: the pooled key buffer is 37 bytes; Go panics beyond
        set_error("flow key of %u bytes exceeds the reference maximum of 37", K);
        return GNS_E_ARG;
    }
    if (l.n_fields && key_bytes && key_bytes != K) {
        set_error("key_bytes=%u disagrees with the layout's %u bytes", key_bytes, K);
        return GNS_E_ARG;
    }
    kp->K = K;
    // tuple byte index of every key byte
    uint32_t off = 0;
    for (uint32_t i = 0; i < l.n_fields; i++) {
        uint32_t base = 0, len = 0;
        switch (l.fields[i]) {
        case GNS_F_SRCIP: base = 0; len = 16; break;
        case GNS_F_DSTIP: base = 16; len = 16; break;
        case GNS_F_SRCPORT: base = 32; len = 2; break;
        case GNS_F_DSTPORT: base = 34; len = 2; break;
        case GNS_F_PROTO: base = 36; len = 1; break;
        default: break;
        }
        for (uint32_t j = 0; j < len; j++) kp->src[off + j] = (uint8_t)(base + j);
        off += len;
    }
    for (uint32_t j = off; j < 80; j++) kp->src[j] = 255;
    // SLICE fast path: key == tuple bytes [4*woff, 4*woff+K)
    kp->woff = -1;
    for (int woff : {0, 4}) {
        bool ok = K > 0;
        for (uint32_t j = 0; j < K && ok; j++) ok = kp->src[j] == (uint8_t)(4 * woff + j);
        if (ok) { kp->woff = woff; break; }
    }
    return GNS_OK;
}

int make_plan2(const gns_layout &a, const gns_layout &b, KeyPlanN *kp) {
    KeyPlanN pa, pb;
    GNS_TRY(make_plan(a, 0, &pa));
    GNS_TRY(make_plan(b, 0, &pb));
    memset(kp, 0, sizeof(*kp));
    kp->K = pa.K + pb.K;
    for (uint32_t j = 0; j < 80; j++) kp->src[j] = 255;
    for (uint32_t j = 0; j < pa.K; j++) kp->src[j] = pa.src[j];
    for (uint32_t j = 0; j < pb.K; j++) kp->src[pa.K + j] = pb.src[j];
    kp->woff = -1;
    for (int woff : {0, 4}) {
        bool ok = kp->K > 0;
        for (uint32_t j = 0; j < kp->K && ok; j++) ok = kp->src[j] == (uint8_t)(4 * woff + j);
        if (ok) { kp->woff = woff; break; }
    }
    return GNS_OK;
}

hipEvent_t StageTimer::get() {
    if (!pool.empty()) {
        hipEvent_t e = pool.back();
        pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

void StageTimer::begin(int stage, hipEvent_t *a) {
    *a = nullptr;
    if (!on || !((mask >> stage) & 1u)) return;
    *a = get();
    if (*a) (void)hipEventRecord(*a, stream);
}

void StageTimer::end(int stage, hipEvent_t a) {
    if (!on || !a) return;
    hipEvent_t b = get();
    if (!b) return;
    (void)hipEventRecord(b, stream);
    pending.push_back({a, b, stage});
}

int StageTimer::collect() {
    for (auto &p : pending) {
        (void)hipEventSynchronize(p.b);
        float t = 0.f;
        if (hipEventElapsedTime(&t, p.a, p.b) == hipSuccess) {
            ms[p.stage] += t;
            launches[p.stage] += 1;
        }
        pool.push_back(p.a);
        pool.push_back(p.b);
    }
    pending.clear();
    return GNS_OK;
}

void StageTimer::destroy() {
    collect();
    for (auto e : pool) (void)hipEventDestroy(e);
    pool.clear();
}

void default_seeds(uint32_t *out, uint32_t n) {
    uint64_t s = 0x9747B28Cull;
    for (uint32_t i = 0; i < n; i++) {
        s += 0x9E3779B97F4A7C15ull;
        uint64_t z = s;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        out[i] = (uint32_t)(z ^ (z >> 31));
    }
}

}  // namespace gns

extern "C" int gns_device_alloc(uint64_t bytes, int device, void **out) {
    if (!out) { gns::set_error("null argument"); return GNS_E_ARG; }
    *out = nullptr;
    (void)hipGetLastError();
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        (void)hipGetLastError();
        gns::set_error("no HIP device available");
        return GNS_E_NODEV;
    }
    if (device < 0 || device >= ndev) { gns::set_error("device %d out of range", device); return GNS_E_ARG; }
    if (hipSetDevice(device) != hipSuccess) { gns::set_error("hipSetDevice(%d) failed", device); return GNS_E_HIP; }
    return gns::dalloc(out, bytes);
}

extern "C" int gns_device_free(void *p, int device) {
    if (!p) return GNS_OK;
    if (hipSetDevice(device) != hipSuccess) { gns::set_error("hipSetDevice(%d) failed", device); return GNS_E_HIP; }
    return hipFree(p) == hipSuccess ? GNS_OK : GNS_E_HIP;
}

extern "C" const char *gns_last_error(void) { return gns::g_last_error.c_str(); }
extern "C" const char *gns_version(void) { return "gns-sketch 0.1 (gfx950)"; }
