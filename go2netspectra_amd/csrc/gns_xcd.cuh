// XCD-contiguous workgroup order for the run-writing partition kernels.
//
// Workgroups are dealt round-robin over the MI355X's 8 XCDs (observed, not promised by HIP;
// /opt/skills/guides/MI355X_MICROARCH.md "Workgroup dispatch"), so in a partition whose
// region b and region b + 1 write adjacent runs of every bin, the partial lines at each run
// boundary would be written through two different L2s.  xcd_block gives XCD x (workgroups
// x, x + 8, ...) the contiguous range of regions starting at x*floor(G/8) + min(x, G mod 8):
// a bijection of [0, G), so only the speed depends on the placement.  Build with
// -DGNS_NO_XCD_MAP for the round-robin order (A/B).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace gns {

__device__ __forceinline__ uint32_t xcd_block(uint32_t bid, uint32_t G) {
#ifdef GNS_NO_XCD_MAP
    (void)G;
    return bid;
#else
    const uint32_t x = bid & 7u, q = G >> 3, r = G & 7u;
    return x * q + min(x, r) + (bid >> 3);
#endif
}

}  // namespace gns
