// gns_dict.hip -- flow-dictionary rebuild: reclaim dead flows, grow the table.
//
// The reference sketches are fixed-size: a bucket holds its fingerprint's key
// bytes (count_min.go:66-81, super_spread.go:163-176), so Go keeps inserting
// however many distinct flows a period (configs/config.yaml:83, 720h) brings.
// Here a fingerprint is a flow id = the slot of the key in the device
// dictionary, and a flow's slot stays claimed after its last bucket is taken
// over.  Between device batches the engines rebuild the dictionary:
//   mark     the ids some bucket (or a live snapshot view) still names -- or,
//            for the exact aggregator, every flow with packets -- are live
//   gather   live records -> a compact stage (tag, key words, bucket cache)
//   reinsert into the cleared table (or a larger one), CAS on empty slots
//            from each key's home slot; remap[old slot] = new slot
//   remap    every id array in place (buckets, view snapshots, SuperSpread cell
//            keys); the exact engine permutes its per-flow state with remap.
// A flow that no bucket names can be dropped without changing any result: no
// fingerprint compares equal to its id, so when it reappears it gets a fresh id
// and every comparison "FP == flow" answers as before.  Live ids are bounded by
// the sketch (at most 2*d*w for Count-Min, d*w for SuperSpread), so the
// dictionary stays bounded under any number of distinct flows.
#include <algorithm>

#include "gns_common.hpp"

namespace gns {

// remap[] during a rebuild: GNS_ID_NONE = not named, kDictMarked = named (live if its
// record is occupied), else the record's new slot.  A named id whose record is
// empty (it cannot be, short of a caller bug) is never reinserted and remaps to
// GNS_ID_NONE -- no fingerprint -- instead of aliasing a real slot.
__global__ __launch_bounds__(256) void k_dict_mark(const uint32_t *ids, uint64_t n, uint64_t slots, uint32_t *remap) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint32_t id = ids[i];
        if (id < slots) remap[id] = kDictMarked;
    }
}

__global__ __launch_bounds__(256) void k_dict_mark_nz(const unsigned long long *keep, uint64_t slots, uint32_t *remap) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < slots; i += (uint64_t)gridDim.x * 256)
        if (keep[i] != 0ull) remap[i] = kDictMarked;
}

// live = occupied and marked; stage them (record words, old slot) compactly
template <bool GATHER>
__global__ __launch_bounds__(256) void k_dict_gather(DictDev D, uint64_t slots, const uint32_t *remap, uint32_t *stage,
                                                     uint32_t *stage_slot, uint32_t *count) {
    for (uint64_t s0 = (uint64_t)blockIdx.x * 256; s0 < slots; s0 += (uint64_t)gridDim.x * 256) {  // wave-uniform
        const uint64_t s = s0 + threadIdx.x;
        const bool live = s < slots && remap[s] == kDictMarked && D.rec[s * D.RW] != 0u;
        const uint64_t m = __ballot(live);
        if (m == 0) continue;
        const uint32_t lane = __lane_id();
        const int leader = __ffsll((unsigned long long)m) - 1;
        uint32_t base = 0;
        if ((int)lane == leader) base = atomicAdd(count, (uint32_t)__popcll(m));
        base = __shfl(base, leader);
        if (GATHER && live) {
            const uint32_t j = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
            const uint32_t *r = D.rec + s * D.RW;
            for (uint32_t w = 0; w < D.RW; w++) stage[(uint64_t)j * D.RW + w] = r[w];
            stage_slot[j] = (uint32_t)s;
        }
    }
}

// reinsert the staged records into the (cleared) table of D; keys are distinct,
// so the first empty slot from the home slot is the record's new place
__global__ __launch_bounds__(256) void k_dict_reinsert(DictDev D, const uint32_t *stage, const uint32_t *stage_slot,
                                                       uint64_t n, uint32_t *remap, uint32_t *fail) {
    const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= n) return;
    const uint32_t *r = stage + j * D.RW;
    uint32_t kw[GNS_KWMAX];
    const uint32_t nkw = (D.K + 3) >> 2;
#pragma unroll
    for (int i = 0; i < GNS_KWMAX; i++) kw[i] = (uint32_t)i < nkw ? r[1 + i] : 0u;
    uint32_t slot = mm3_n<GNS_KWMAX>(kw, D.K, D.seed) & D.mask;
    for (uint32_t probe = 0; probe <= D.mask; probe++) {
        uint32_t *tp = D.rec + (size_t)slot * D.RW;
        if (atomicCAS(tp, 0u, r[0]) == 0u) {
            for (uint32_t w = 1; w < D.RW; w++) tp[w] = r[w];
            remap[stage_slot[j]] = slot;
            return;
        }
        slot = (slot + 1u) & D.mask;
    }
    atomicAdd(fail, 1u);
}

__global__ __launch_bounds__(256) void k_dict_remap(uint32_t *ids, uint64_t n, uint64_t slots, const uint32_t *remap) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint32_t id = ids[i];
        if (id < slots) {
            const uint32_t r = remap[id];
            ids[i] = r < kDictMarked ? r : GNS_ID_NONE;
        }
    }
}

static unsigned grid_for(uint64_t n) { return (unsigned)std::min<uint64_t>(8192, (n + 255) / 256 + 1); }

void DictScratch::free_all() {
    dfree(remap); dfree(stage); dfree(stage_slot); dfree(cnt);
    if (h_cnt) (void)hipHostFree(h_cnt);
    remap = stage = stage_slot = cnt = h_cnt = nullptr;
    remap_n = stage_n = 0;
}

int dict_rebuild(DictDev &D, uint64_t &slots, const DictIds *mark, int nmark, const unsigned long long *keep_nz,
                 DictIds *remap_arrays, int nremap, uint64_t new_slots, hipStream_t s, DictScratch &sc,
                 uint64_t *live_out, uint32_t **old_rec_out, uint64_t grow_max) {
    if (new_slots < slots) new_slots = slots;
    if (!sc.cnt) GNS_TRY(dalloc_t(&sc.cnt, 4));
    if (!sc.h_cnt && hipHostMalloc(reinterpret_cast<void **>(&sc.h_cnt), 16, 0) != hipSuccess) {
        sc.h_cnt = nullptr;
        set_error("hipHostMalloc failed");
        return GNS_E_OOM;
    }
    if (sc.remap_n < std::max(slots, new_slots)) {
        dfree(sc.remap);
        sc.remap = nullptr;
        sc.remap_n = 0;
        GNS_TRY(dalloc_t(&sc.remap, std::max(slots, new_slots)));
        sc.remap_n = std::max(slots, new_slots);
    }
    // mark
    GNS_HIP(hipMemsetAsync(sc.remap, 0xFF, slots * 4, s));
    for (int i = 0; i < nmark; i++)
        if (mark[i].n) hipLaunchKernelGGL(k_dict_mark, dim3(grid_for(mark[i].n)), dim3(256), 0, s, mark[i].ids, mark[i].n, slots, sc.remap);
    if (keep_nz) hipLaunchKernelGGL(k_dict_mark_nz, dim3(grid_for(slots)), dim3(256), 0, s, keep_nz, slots, sc.remap);
    // count, stage
    GNS_HIP(hipMemsetAsync(sc.cnt, 0, 8, s));
    hipLaunchKernelGGL(k_dict_gather<false>, dim3(grid_for(slots)), dim3(256), 0, s, D, slots, sc.remap, nullptr, nullptr, sc.cnt);
    GNS_HIP(hipGetLastError());
    GNS_HIP(hipMemcpyAsync(sc.h_cnt, sc.cnt, 4, hipMemcpyDeviceToHost, s));
    GNS_HIP(hipStreamSynchronize(s));
    const uint64_t live = sc.h_cnt[0];
    // growth: the live set alone past a quarter of the table doubles it (the
    // reclaim that follows a batch then leaves at least half the slots free)
    while (grow_max && live > new_slots / 4 && new_slots < grow_max) new_slots *= 2;
    if (live > new_slots - new_slots / 8) {
        set_error("flow dictionary: %llu live flows do not fit %llu slots", (unsigned long long)live,
                  (unsigned long long)new_slots);
        return GNS_E_FULL;
    }
    if (sc.stage_n < std::max<uint64_t>(live, 1)) {
        dfree(sc.stage); dfree(sc.stage_slot);
        sc.stage = sc.stage_slot = nullptr;
        sc.stage_n = 0;
        const uint64_t want = std::max<uint64_t>(live + live / 4, 1024);
        GNS_TRY(dalloc_t(&sc.stage, want * D.RW));
        GNS_TRY(dalloc_t(&sc.stage_slot, want));
        sc.stage_n = want;
    }
    GNS_HIP(hipMemsetAsync(sc.cnt, 0, 8, s));
    hipLaunchKernelGGL(k_dict_gather<true>, dim3(grid_for(slots)), dim3(256), 0, s, D, slots, sc.remap, sc.stage, sc.stage_slot, sc.cnt);
    GNS_HIP(hipGetLastError());
    // the new table: the same one cleared, or a larger one
    DictDev N = D;
    uint32_t *old_rec = nullptr;
    if (new_slots != slots) {
        GNS_TRY(dalloc_t(&N.rec, new_slots * D.RW));
        N.mask = (uint32_t)(new_slots - 1);
        old_rec = D.rec;
    }
    GNS_HIP(hipMemsetAsync(N.rec, 0, new_slots * D.RW * 4, s));
    if (live) hipLaunchKernelGGL(k_dict_reinsert, dim3((unsigned)((live + 255) / 256)), dim3(256), 0, s, N, sc.stage,
                                 sc.stage_slot, live, sc.remap, sc.cnt + 1);
    for (int i = 0; i < nremap; i++)
        if (remap_arrays[i].n)
            hipLaunchKernelGGL(k_dict_remap, dim3(grid_for(remap_arrays[i].n)), dim3(256), 0, s, remap_arrays[i].ids,
                               remap_arrays[i].n, slots, sc.remap);
    GNS_HIP(hipGetLastError());
    // claims since the rebuild start from the live count; the abort flag is clear
    sc.h_cnt[2] = (uint32_t)live;
    sc.h_cnt[3] = 0;
    GNS_HIP(hipMemcpyAsync(D.ctl, sc.h_cnt + 2, 8, hipMemcpyHostToDevice, s));
    GNS_HIP(hipMemcpyAsync(sc.h_cnt + 1, sc.cnt + 1, 4, hipMemcpyDeviceToHost, s));
    GNS_HIP(hipStreamSynchronize(s));
    if (sc.h_cnt[1]) {  // cannot happen: live <= 7/8 of the slots
        set_error("flow dictionary rebuild lost %u records", sc.h_cnt[1]);
        return GNS_E_HIP;
    }
    if (old_rec_out) *old_rec_out = old_rec;
    else dfree(old_rec);
    D.rec = N.rec;
    D.mask = N.mask;
    slots = new_slots;
    if (live_out) *live_out = live;
    return GNS_OK;
}

}  // namespace gns
