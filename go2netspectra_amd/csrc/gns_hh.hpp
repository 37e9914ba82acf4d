// gns_hh.hpp -- the device heavy-hitter list (gns_cm.hip) shared with SuperSpread.
//
// One (value, fingerprint id) cell array whose ids are slots of a flow dictionary
// -> the list of flows whose max over their cells reaches `thr`, in canonical order
// (value desc, flow bytes asc): candidate compaction, per-flow max + one emit per
// flow, the hand-written LSD radix order, one D2H.  count_min.go:178-247 and
// super_spread.go:254-294 are both this computation (a flow's estimate is the max
// over the cells that hold it, so it reaches thr iff one of those cells does).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "gns_keys.cuh"

struct CmScratch;  // grow-only device / pinned buffers of the list (gns_cm.hip)

namespace gns {
CmScratch *hh_scratch_new();
void hh_scratch_free(CmScratch *sc);
// flows: n*K bytes, vals: n values; *n_io = capacity in, full list length out.
// Runs on stream st and returns after the list is in host memory.
int hh_heavy_list(CmScratch *sc, hipStream_t st, const DictDev &D, uint64_t dict_slots, uint32_t K, uint64_t cells,
                  const uint32_t *val, const uint32_t *fp, uint32_t thr, uint8_t *flows, uint32_t *vals,
                  uint64_t *n_io);
}  // namespace gns
