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

// deterministic log on (0, 1] (oracle: or_det_log)
__host__ __device__ inline double gm_log(double x) {
    const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10;
    const double L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01;
    const double L3 = 2.857142874366239149e-01, L4 = 2.222219843214978396e-01;
    const double L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01;
    const double L7 = 1.479819860511658591e-01;
    int ki;
    double f1 = go_frexp(x, &ki);
    if (f1 < 0.70710678118654752440) { f1 *= 2; ki--; }
    const double f = f1 - 1;
    const double k = (double)ki;
    const double s = f / (2 + f);
    const double s2 = s * s;
    const double s4 = s2 * s2;
    const double t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)));
    const double t2 = s4 * (L2 + s4 * (L4 + s4 * L6));
    const double R = t1 + t2;
    const double hfsq = 0.5 * f * f;
    return k * Ln2Hi - ((hfsq - (s * (hfsq + R) + k * Ln2Lo)) - f);
}

// log(1 - p), 0 < p < 1 (oracle: or_det_log1m)
__host__ __device__ inline double gm_log1m(double p) {
    if (p < 1e-4) {
        const double t = p * p;
        double r = p + t * 0.5;
        r = r + t * p * (1.0 / 3.0);
        return -r;
    }
    return gm_log(1.0 - p);
}

#pragma clang fp contract(on)

}  // namespace gns
