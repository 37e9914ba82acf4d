// gns_common.hpp -- host-side plumbing shared by the Count-Min and SuperSpread
// engines: error reporting, device buffers, per-stage HIP-event timing, and
// staging of host inputs into device memory.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/gns_sketch.h"
#include "gns_device.cuh"
#include "gns_keys.cuh"

namespace gns {

void set_error(const char *fmt, ...);

#define GNS_HIP(call)                                                                  \
    do {                                                                               \
        hipError_t e_ = (call);                                                        \
        if (e_ != hipSuccess) {                                                        \
            ::gns::set_error("%s:%d %s: %s", __FILE__, __LINE__, #call,                \
                             hipGetErrorString(e_));                                   \
            return GNS_E_HIP;                                                          \
        }                                                                              \
    } while (0)

#define GNS_TRY(expr)                  \
    do {                               \
        int r_ = (expr);               \
        if (r_ != GNS_OK) return r_;   \
    } while (0)

// Device allocation that reports OOM as GNS_E_OOM.
int dalloc(void **p, size_t bytes);
template <class T>
int dalloc_t(T **p, size_t count) {
    return dalloc(reinterpret_cast<void **>(p), count * sizeof(T) + 16);
}
void dfree(void *p);

// Flow-key plan from a configured layout (task.go:265-300, :327-338).
int make_plan(const gns_layout &l, uint32_t key_bytes, KeyPlanN *out);
// plan for the concatenation a ‖ b (SuperSpread merged key, super_spread.go:183-190)
int make_plan2(const gns_layout &a, const gns_layout &b, KeyPlanN *out);
uint32_t layout_bytes(const gns_layout &l);

// Per-stage timing with HIP events recorded on the engine stream.
struct StageTimer {
    enum { kStages = 8 };
    bool on = false;
    uint32_t mask = 0xFFFFFFFFu;  // stages timed while on
    double ms[kStages] = {};
    uint64_t launches[kStages] = {};
    std::vector<hipEvent_t> pool;
    struct Pending { hipEvent_t a, b; int stage; };
    std::vector<Pending> pending;
    hipStream_t stream = nullptr;

    hipEvent_t get();
    void begin(int stage, hipEvent_t *a);
    void end(int stage, hipEvent_t a);
    int collect();  // synchronizes pending events and accumulates
    void destroy();
};

// gns_*_set_timing's argument: 0 off, GNS_TIMING_MASK | stage bits = only those stages (fewer
// events inside a batch), any other nonzero value = every stage
inline void set_timing_arg(StageTimer &t, int on) {
    t.on = on != 0;
    t.mask = (on & GNS_TIMING_MASK) ? ((uint32_t)on & 0xFFu) : 0xFFFFFFFFu;
}

struct ScopedStage {
    StageTimer &t; int stage; hipEvent_t a = nullptr;
    ScopedStage(StageTimer &tt, int s) : t(tt), stage(s) { t.begin(stage, &a); }
    ~ScopedStage() { t.end(stage, a); }
};

// splitmix64 row seeds used when the caller passes none.
void default_seeds(uint32_t *out, uint32_t n);

// Dictionary record words {tag, key words}: a power of two (4, 8 or 16 words)
// so that no record straddles a 64-byte line (one line per probe).
inline uint32_t dict_record_words(uint32_t K) {
    const uint32_t w = 1 + (K + 3) / 4;
#ifdef GNS_DICT_PACKED
    return (w + 3) & ~3u;
#else
    return w <= 4 ? 4u : (w <= 8 ? 8u : 16u);
#endif
}

// Count-Min records: 16 words whenever the key leaves words 12..15 free, which
// then cache the flow's bucket indices of rows 0..3 (written by the claimer),
// so a packet of a known flow needs no per-row MurmurHash3; deeper sketches take
// 32-word records (one 128-byte line, as a 64-byte record's probe fetches anyway)
// whose words 12..19 cache rows 0..7.
inline uint32_t dict_record_words_cm(uint32_t K, uint32_t d) {
    const uint32_t w = 1 + (K + 3) / 4;
    return (K > 12 && w <= 12) ? (d > 4 ? 32u : 16u) : dict_record_words(K);
}

// Flow-dictionary rebuild (gns_dict.hip): keep the records whose id some
// array in `mark` names (or whose keep_nz entry is nonzero), reinsert them into
// the cleared table -- or a new one of new_slots slots -- and rewrite the ids of
// every array in `remap_arrays`.  D.rec / D.mask / slots are updated; the
// scratch's remap (old slot -> new slot, ~0 = dropped) stays valid until the
// next rebuild.  D.ctl[0] restarts at the live count.  Synchronizes stream s.
struct DictIds {
    uint32_t *ids;
    uint64_t n;
};
struct DictScratch {
    uint32_t *remap = nullptr, *stage = nullptr, *stage_slot = nullptr, *cnt = nullptr, *h_cnt = nullptr;
    uint64_t remap_n = 0, stage_n = 0;
    void free_all();
};
// grow_max != 0: the table also doubles (up to grow_max slots) while the live
// flows exceed a quarter of it.
int dict_rebuild(DictDev &D, uint64_t &slots, const DictIds *mark, int nmark, const unsigned long long *keep_nz,
                 DictIds *remap_arrays, int nremap, uint64_t new_slots, hipStream_t s, DictScratch &sc,
                 uint64_t *live_out, uint32_t **old_rec_out, uint64_t grow_max = 0);
// Largest dictionary: flow ids are u32 slots below kDictMarked (0xFFFFFFFE /
// GNS_ID_NONE are reserved); 2^30 slots keep a 64-byte-record table at 64 GB.
constexpr uint64_t kDictMaxSlots = 1ull << 30;

// gns_frame.cpp: one captured frame -> one 64-byte record for the device
// parser.  Returns 0 = copied verbatim (device fast-path shape), 1 = decoded
// into a pre-parsed 0x88B5 record, 2 = no IP layer (a record the device drops).
int frame_record(const uint8_t *frame, uint32_t caplen, uint32_t wirelen, uint8_t *rec);
// frame_record's record (and its return code) -> compact 16-byte record; returns
// the class (kRecSide: the caller stores the side index in word 0)
int compact_record(int code, const uint8_t *rec, uint8_t *out16);
// the 16-byte form: the wire length in word 3 bits 16..31 (-1: above 65535); a tuple
// record is IPv4 both ways, any other tuple escapes to the side array
int compact_record16(int code, const uint8_t *rec, uint32_t orig, uint8_t *out16);

inline uint32_t ceil_log2(uint64_t x) {
    uint32_t b = 0;
    while ((1ull << b) < x) b++;
    return b;
}

}  // namespace gns
