// pt_math.h -- binary32 arithmetic of the hot path, shared by host-side precompute and the
// gfx950 kernels.  Every function here is pinned so that the HIP kernels,
// the host precompute and the CPU oracle round every operation identically:
//   * IEEE binary32, round to nearest even, no contraction (build with -ffp-contract=off),
//     correctly rounded division and square root;
//   * dot(a,b) = (a.x*b.x + a.y*b.y) + a.z*b.z ; cross per the GLSL spec;
//   * normalize(v) = v * (1 / sqrt(dot(v,v))) ; mix(x,y,a) = x*(1-a) + y*a ;
//   * log / cos: the build's pinned polynomials (logf_pinned, cosf_pinned below).
// computeShader.c leaves transcendental precision to the GL driver (implementation-defined);
// these are the build's pinned choices.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define PT_HD __host__ __device__ __forceinline__
#else
#include <math.h>
#include <string.h>
#define PT_HD inline
#endif

namespace pt {

PT_HD uint32_t fbits(float f) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __float_as_uint(f);
#else
    uint32_t u; __builtin_memcpy(&u, &f, 4); return u;
#endif
}
PT_HD float bitsf(uint32_t u) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __uint_as_float(u);
#else
    float f; __builtin_memcpy(&f, &u, 4); return f;
#endif
}
PT_HD float fsqrt(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_sqrtf(x);      // correctly rounded (-fhip-fp32-correctly-rounded-divide-sqrt)
#else
    return sqrtf(x);
#endif
}

// Guarded fast forms of the correctly rounded reciprocal and square root, for arguments the
// caller has bounded to [2^-100, 2^100] in magnitude (no scaling, no special cases): one
// v_rcp_f32 / v_sqrt_f32 plus fma corrections.  Bit-identical to 1.0f/x and sqrtf(x) over
// EVERY binary32 in that range on gfx950 -- checked exhaustively by tools/verify_fastmath.hip
// (tests/test_gpu_fastmath.py).  Host builds use the IEEE operations themselves.
PT_HD float rcp_fast(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    float y = __builtin_amdgcn_rcpf(x);
    float e = __builtin_fmaf(-x, y, 1.0f);
    return __builtin_fmaf(e, y, y);
#else
    return 1.0f / x;
#endif
}
PT_HD float sqrt_fast(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    // v_rsq_f32, s0 = x * y, and one fma correction s0 + (x - s0^2) * y/2: 5 VALU (the
    // former v_sqrt_f32 + neighbour-residual selects took 9); correctly rounded for every x
    // in the guard on gfx950 (tools/verify_fastmath.hip, exhaustive)
    const float y = __builtin_amdgcn_rsqf(x);
    const float s0 = x * y, h = 0.5f * y;
    const float r = __builtin_fmaf(-s0, s0, x);
    return __builtin_fmaf(r, h, s0);
#else
    return sqrtf(x);
#endif
}

// a / b for |a| in [2^-20, 2^60] and b with RN(1/b) = rb exactly (Markstein: the remainder
// a - q0*b is exact and fma(r, rb, q0) is the correctly rounded quotient).
PT_HD float div_mk(float a, float b, float rb) {
    float q = a * rb;
    float r = __builtin_fmaf(-q, b, a);
    return __builtin_fmaf(r, rb, q);
}

// log and cos of the Box-Muller draw (computeShader.c:115-120).  GLSL leaves their precision
// to the driver (GLSL 4.30 §4.7.1: log within 3 ulp, cos within 2^-11 absolute), and the
// reference's image depends on the driver's choice; these are the build's pinned choices,
// restated independently by the oracle (oracle/pt_oracle.cpp) and its numpy twin.  Both are
// branch-free polynomials in fma (exactly rounded on the CPU's FMA and on v_fma_f32, so host
// and device agree bit for bit: tools/verify_fastmath.hip, tests/test_exact_div.py).
// Measured over every binary32 of the hot-path domains (tests/test_oracle_pinning.py):
//   logf_pinned: at most 1.2 ulp;  cosf_pinned: at most 1.06e-7 absolute.
// (Rounds 1-2 pinned fdlibm e_logf and Cephes cosf: 58 and 41 VALU against 22 and 18 here,
// +5.7% on C2.)
//
// log(x), x in {0} U [2^-32, 1]: x = 2^k z with z in [0.699, 1.398) (the exponent split at
// 0x3f330000), f = z - 1, log(1 + f) = f + f^2 P(f) with P a degree-7 fit (relative error
// 3e-8 on the interval), then + k ln2 in two parts (k * ln2_hi exact).  log(0) = -inf.
PT_HD float logf_pinned(float x) {
    const uint32_t ix = fbits(x);
    const uint32_t tmp = ix - 0x3f330000u;
    const int k = (int32_t)tmp >> 23;
    const float z = bitsf(ix - (tmp & 0xff800000u));
    const float f = z - 1.0f, f2 = f * f;
    float P = __builtin_fmaf(f, 0x1.87c9c0p-4f, -0x1.2bf636p-3f);
    P = __builtin_fmaf(f, P, 0x1.2f3194p-3f);
    P = __builtin_fmaf(f, P, -0x1.52694ep-3f);
    P = __builtin_fmaf(f, P, 0x1.98eb62p-3f);
    P = __builtin_fmaf(f, P, -0x1.000924p-2f);
    P = __builtin_fmaf(f, P, 0x1.5556ccp-2f);
    P = __builtin_fmaf(f, P, -0x1.fffff0p-2f);
    const float kf = (float)k;
    const float r = __builtin_fmaf(kf, 0x1.62e300p-1f, __builtin_fmaf(kf, 0x1.2fefa2p-17f, __builtin_fmaf(f2, P, f)));
    // log 0 = -inf by a select on the bits (x = +0 has no other encoding here): a compare on
    // the float made the compiler branch around the whole polynomial
    return ix == 0u ? bitsf(0xff800000u) : r;
}
// cos(t), t in [0, 2 pi] (the draw's angle): q = rint(t 2/pi), r = t - q pi/2 (two-part
// pi/2 by fma, |r| <= pi/4), then cos r or sin r by degree-6 / degree-7 fits (absolute error
// 3e-8 / 2e-9) for quadrant q mod 4, negated in quadrants 1 and 2.
PT_HD float cosf_pinned(float t) {
    const float qf = __builtin_rintf(t * 0x1.45f306p-1f);
    float r = __builtin_fmaf(-qf, 0x1.921fb6p+0f, t);
    r = __builtin_fmaf(-qf, -0x1.777a5cp-25f, r);
    const float r2 = r * r;
    const float c = __builtin_fmaf(r2, __builtin_fmaf(r2, __builtin_fmaf(r2, -0x1.64756cp-10f, 0x1.553f94p-5f), -0x1.ffffbap-2f), 1.0f);
    const float u = __builtin_fmaf(r2, __builtin_fmaf(r2, -0x1.98da64p-13f, 0x1.1105b4p-7f), -0x1.555540p-3f);
    const float sn = __builtin_fmaf(r * r2, u, r);
    const int q = (int)qf;
    const float v = (q & 1) ? sn : c;
    return bitsf(fbits(v) ^ ((uint32_t)((q + 1) & 2) << 30));
}

struct f3 { float x, y, z; };
PT_HD f3 mk(float x, float y, float z) { f3 r; r.x = x; r.y = y; r.z = z; return r; }
PT_HD f3 operator+(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
PT_HD f3 operator-(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
PT_HD f3 operator*(f3 a, f3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
PT_HD f3 operator*(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
PT_HD f3 operator/(f3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
PT_HD float dot(f3 a, f3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
PT_HD f3 cross(f3 a, f3 b) { return mk(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y); }
// The guard of rcp_fast / sqrt_fast; NaN fails it.
// Range predicates of the guards and hit windows, in two forms that agree on every input:
// float compares (_f) and one unsigned compare of the bit patterns (_u; positive floats order
// as their bits, and zeros, negatives, inf and NaN fall outside each window as they fail the
// float compares).  tests/test_int_windows.py checks the agreement on special values and
// random bit patterns; the guards use the _u forms, PT_INT_WINDOWS the windows too.
PT_HD bool range_abs_f(float v, float lo, float hi) {      // |v| in [lo, hi], 0 < lo <= hi
    const float a = __builtin_fabsf(v);
    return (a >= lo) & (a <= hi);
}
PT_HD bool range_abs_u(float v, float lo, float hi) {
    return (fbits(v) & 0x7fffffffu) - fbits(lo) <= fbits(hi) - fbits(lo);
}
PT_HD bool guard_f(float v, float lo, float hi) { return (v == 0.0f) | range_abs_f(v, lo, hi); }
PT_HD bool guard_u(float v, float lo, float hi) { return ((fbits(v) & 0x7fffffffu) == 0u) | range_abs_u(v, lo, hi); }
// 1e-4 < x < t and 1e-4 <= x < t, for t > 1e-4 (t starts at +inf and only takes accepted
// distances, which exceed 1e-4)
PT_HD bool win_open_f(float x, float t) { return (x > 0.0001f) & (x < t); }
PT_HD bool win_open_u(float x, float t) {
    const uint32_t lo = fbits(0.0001f) + 1u;
    return fbits(x) - lo < fbits(t) - lo;
}
PT_HD bool win_closed_f(float x, float t) { return (x >= 0.0001f) & (x < t); }
PT_HD bool win_closed_u(float x, float t) {
    const uint32_t lo = fbits(0.0001f);
    return fbits(x) - lo < fbits(t) - lo;
}
PT_HD bool fast_range_f(float q) { return q >= 0x1p-100f && q <= 0x1p100f; }
PT_HD bool fast_range_u(float q) { return fbits(q) - fbits(0x1p-100f) <= fbits(0x1p100f) - fbits(0x1p-100f); }
// the guards use the unsigned forms (measured, same-process A/B: +0.49% on C2, +0.23% / +0.26%
// on the C3 / C4 stand-ins); the hit windows keep the float compares by default (the unsigned
// ones measured +0.32% / +0.25% / +0.37%, within the guards' gain)
PT_HD bool in_range_abs(float v, float lo, float hi) { return range_abs_u(v, lo, hi); }
PT_HD bool in_guard(float v, float lo, float hi) { return guard_u(v, lo, hi); }
#if defined(PT_INT_WINDOWS)
PT_HD bool win_open(float x, float t) { return win_open_u(x, t); }
PT_HD bool win_closed(float x, float t) { return win_closed_u(x, t); }
#else
PT_HD bool win_open(float x, float t) { return win_open_f(x, t); }
PT_HD bool win_closed(float x, float t) { return win_closed_f(x, t); }
#endif
PT_HD bool fast_range(float q) {
    return fast_range_u(q);
}
PT_HD float sqrt_g(float q) {
    if (fast_range(q)) return sqrt_fast(q);
    return fsqrt(q);
}
PT_HD float length(f3 a) { return sqrt_g(dot(a, a)); }
// length(a) > 0.01f without the root: RN(sqrt(q)) is non-decreasing in q, and the least
// binary32 q with RN(sqrt(q)) > 0.01f is 0x38d1b719 (tests/test_exact_div.py checks every
// binary32 against the IEEE root); NaN fails both forms.
PT_HD bool length_gt_001(f3 a) { return dot(a, a) >= bitsf(0x38d1b719u); }
// num / den, correctly rounded: by the exact reciprocal and a Markstein correction when
// both magnitudes lie in [2^-60, 2^60] (quotient in [2^-120, 2^120], remainder granularity
// >= 2^-106: no overflow, no underflow), else the IEEE division.
PT_HD float div_g(float num, float den) {
    const float an = num < 0.0f ? -num : num, ad = den < 0.0f ? -den : den;
    if (an >= 0x1p-60f && an <= 0x1p60f && ad >= 0x1p-60f && ad <= 0x1p60f) return div_mk(num, den, rcp_fast(den));
    return num / den;
}
// v * (1/sqrt(dot(v,v))): the two correctly rounded steps, each by its guarded fast form
// (dot in [2^-100, 2^100] puts the root in [2^-50, 2^50]).
PT_HD f3 normalize(f3 a) {
    float q = dot(a, a), r;
    if (fast_range(q)) r = rcp_fast(sqrt_fast(q));
    else r = 1.0f / fsqrt(q);
    return a * r;
}
PT_HD f3 mix(f3 x, f3 y, float a) {
    float oma = 1.0f - a;
    return mk(x.x * oma + y.x * a, x.y * oma + y.y * a, x.z * oma + y.z * a);
}

// PCG-style hash RNG (computeShader.c:87-98): uint32 wraparound; value/2^32 in [0,1].
PT_HD uint32_t next_random(uint32_t& s) {
    s = s * 747796405u + 2891336453u;
    uint32_t r = ((s >> ((s >> 28) + 4)) ^ s) * 277803737u;
    return (r >> 22) ^ r;
}
PT_HD float random01(uint32_t& s) { return (float)next_random(s) * (1.0f / 4294967296.0f); }
PT_HD float random_normal(uint32_t& s) {            // :115-120 (theta first, then rho)
#if defined(PT_EXP_HW_NORMAL) && defined(__HIP_DEVICE_COMPILE__)
    // timing experiment only (NOT the pinned arithmetic): hardware log2 / cos
    float u1 = random01(s);
    float u2 = random01(s);
    return __builtin_sqrtf(-1.3862944f * __builtin_amdgcn_logf(u2)) * __builtin_amdgcn_cosf(u1);
#endif
    // (2 * 3.1415926f) * (float(r) * 2^-32) as ONE rounding: float(r) * 2^-32 is exact (r >= 1
    // or 0: no subnormal) and so is the constant's 2^-32 scaling, so both forms round the same
    // real product
    float theta = (float)next_random(s) * ((2.0f * 3.1415926f) * (1.0f / 4294967296.0f));
    // -2 log(u) is 0 (u = 1), +inf (u = 0) or in [2^-24, 45]: inside sqrt_fast's guard except
    // the two ends, which are their own roots -- a select instead of sqrt_g's branch
    const float q = -2.0f * logf_pinned(random01(s));
    const float rho = ((q == 0.0f) | (q == __builtin_huge_valf())) ? q : sqrt_fast(q);
    return rho * cosf_pinned(theta);
}
PT_HD f3 random_unit_vector(uint32_t& s) {          // :122-129, x, y, z order
    float x = random_normal(s);
    float y = random_normal(s);
    float z = random_normal(s);
    return normalize(mk(x, y, z));
}
PT_HD uint32_t seed(int x, int y, int frame) {      // :514-515, mod 2^32
    return ((uint32_t)y * 831266u + (uint32_t)x * 923766u) + (uint32_t)frame * 719393u;
}

}  // namespace pt
