// gns_gomath.cuh -- the float64 steps SuperSpread needs, restated so the device
// rounds exactly like Go (super_spread.go:105-109,200,206,222):
//   math.Pow (integer exponent path: Frexp, square-and-multiply, Ldexp),
//   math.Ldexp / math.Frexp (bit level), the declared counter-based RNG that
//   replaces rand.Float64, and the per-HLL seed derivation.
// Compiled with FP contraction off: no fused multiply-add may change a rounding.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gns {

#pragma clang fp contract(off)

__host__ __device__ __forceinline__ uint64_t gm_mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// declared generator (oracle: or_ss_uniform)
__host__ __device__ __forceinline__ double ss_uniform(uint64_t rng_seed, uint64_t pkt, uint32_t row,
                                                      uint32_t draw) {
    uint64_t x = gm_mix64(rng_seed + pkt * 0x9E3779B97F4A7C15ull);
    x = gm_mix64(x ^ ((uint64_t)row << 32 | draw) ^ 0xD1B54A32D192ED03ull);
    return (double)(x >> 11) * 0x1.0p-53;
}

// GeneralHLL.seeds[0..1] of one cell (oracle: or_ss_hll_seeds)
__host__ __device__ __forceinline__ void ss_hll_seeds(uint64_t master, uint64_t cell, uint32_t &s0,
                                                      uint32_t &s1) {
    const uint64_t x = gm_mix64(master + cell * 0x9E3779B97F4A7C15ull);
    s0 = (uint32_t)x;
    s1 = (uint32_t)(x >> 32);
}

__host__ __device__ __forceinline__ uint64_t gm_bits(double x) {
    union { double d; uint64_t u; } v;
    v.d = x;
    return v.u;
}
__host__ __device__ __forceinline__ double gm_from(uint64_t u) {
    union { double d; uint64_t u; } v;
    v.u = u;
    return v.d;
}

// Go math.Ldexp (src/math/ldexp.go)
__host__ __device__ inline double go_ldexp(double frac, int e) {
    if (frac == 0 || frac != frac || (gm_bits(frac) & 0x7FFFFFFFFFFFFFFFull) == 0x7FF0000000000000ull) return frac;
    int ne = 0;
    if ((gm_bits(frac) & 0x7FF0000000000000ull) == 0) {  // subnormal: normalize
        frac *= 4503599627370496.0;                        // 2^52
        ne = -52;
    }
    e += ne;
    uint64_t x = gm_bits(frac);
    e += (int)((x >> 52) & 0x7FF) - 1023;
    if (e < -1075) return gm_from(x & 0x8000000000000000ull);  // copysign(0, frac)
    if (e > 1023) return gm_from((x & 0x8000000000000000ull) | 0x7FF0000000000000ull);
    double m = 1.0;
    if (e < -1022) { e += 53; m = 1.0 / 9007199254740992.0; }  // 2^-53
    x &= ~(0x7FFull << 52);
    x |= (uint64_t)(e + 1023) << 52;
    return m * gm_from(x);
}

// Go math.Frexp for finite nonzero x
__host__ __device__ inline double go_frexp(double x, int *e) {
    if (x == 0 || x != x || (gm_bits(x) & 0x7FFFFFFFFFFFFFFFull) == 0x7FF0000000000000ull) { *e = 0; return x; }
    int ne = 0;
    if ((gm_bits(x) & 0x7FF0000000000000ull) == 0) { x *= 4503599627370496.0; ne = -52; }
    uint64_t u = gm_bits(x);
    *e = ne + (int)((u >> 52) & 0x7FF) - 1022;
    u &= ~(0x7FFull << 52);
    u |= (uint64_t)1022 << 52;
    return gm_from(u);
}

// Go math.Pow for x > 0 finite and integer y (|y| < 2^63), src/math/pow.go
__host__ __device__ inline double go_pow_int(double x, double y) {
    if (y == 0 || x == 1) return 1.0;
    if (y == 1) return x;
    const double ay = y < 0 ? -y : y;
    double a1 = 1.0;
    int ae = 0;
    int xe;
    double x1 = go_frexp(x, &xe);
    for (int64_t i = (int64_t)ay; i != 0; i >>= 1) {
        if (xe < -(1 << 12) || (1 << 12) < xe) { ae += xe; break; }
        if (i & 1) { a1 *= x1; ae += xe; }
        x1 *= x1;
        xe <<= 1;
        if (x1 < .5) { x1 += x1; xe--; }
    }
    if (y < 0) { a1 = 1 / a1; ae = -ae; }
    return go_ldexp(a1, ae);
}

#pragma clang fp contract(on)

}  // namespace gns
