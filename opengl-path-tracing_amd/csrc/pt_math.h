// pt_math.h -- binary32 arithmetic of the hot path, shared by host-side precompute and the
// gfx950 kernels.  Every function here is pinned so that the HIP kernels,
// the host precompute and the CPU oracle round every operation identically:
//   * IEEE binary32, round to nearest even, no contraction (build with -ffp-contract=off),
//     correctly rounded division and square root;
//   * dot(a,b) = (a.x*b.x + a.y*b.y) + a.z*b.z ; cross per the GLSL spec;
//   * normalize(v) = v * (1 / sqrt(dot(v,v))) ; mix(x,y,a) = x*(1-a) + y*a ;
//   * log: fdlibm e_logf algorithm; cos: Cephes cosf algorithm (octant reduction, 3-part pi/4).
// computeShader.c leaves transcendental precision to the GL driver (implementation-defined);
// these are the build's pinned choices (both < 2 ulp on the ranges the hot path feeds).
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
    uint32_t u; memcpy(&u, &f, 4); return u;
#endif
}
PT_HD float bitsf(uint32_t u) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __uint_as_float(u);
#else
    float f; memcpy(&f, &u, 4); return f;
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

// fdlibm e_logf (FreeBSD constants).  x in {0} U [2^-32, 1] on the hot path.
PT_HD float logf_pinned(float x) {
    const float ln2_hi = 6.9313812256e-01f, ln2_lo = 9.0580006145e-06f, two25 = 3.355443200e+07f;
    const float Lg1 = bitsf(0x3f2aaaaau), Lg2 = bitsf(0x3ecccce1u), Lg3 = bitsf(0x3e91e9eeu),
                Lg4 = bitsf(0x3e789e26u);
    int32_t ix = (int32_t)fbits(x);
    int32_t k = 0;
    if (ix < 0x00800000) {
        if ((ix & 0x7fffffff) == 0) return bitsf(0xff800000u);   // -inf
        if (ix < 0) return bitsf(0x7fc00000u);                    // NaN
        k -= 25; x *= two25; ix = (int32_t)fbits(x);
    }
    if (ix >= 0x7f800000) return x + x;
    k += (ix >> 23) - 127;
    ix &= 0x007fffff;
    int32_t i = (ix + (0x95f64 << 3)) & 0x800000;
    x = bitsf((uint32_t)(ix | (i ^ 0x3f800000)));
    k += (i >> 23);
    float f = x - 1.0f;
    float dk;
    if ((0x007fffff & (0x8000 + ix)) < 0xc000) {
        if (f == 0.0f) {
            if (k == 0) return 0.0f;
            dk = (float)k;
            return dk * ln2_hi + dk * ln2_lo;
        }
        float R = f * f * (0.5f - 0.33333333333333333f * f);
        if (k == 0) return f - R;
        dk = (float)k;
        return dk * ln2_hi - ((R - dk * ln2_lo) - f);
    }
    // |f| >= 2^-20 on this path (the branch above takes smaller f) and 2+f in [1.58, 2.42]:
    // the quotient by an exact reciprocal (rcp_fast) and a Markstein correction
    const float tf = 2.0f + f;
    float s = div_mk(f, tf, rcp_fast(tf));
    dk = (float)k;
    float z = s * s;
    int32_t ii = ix - (0x6147a << 3);
    float w = z * z;
    int32_t j = (0x6b851 << 3) - ix;
    float t1 = w * (Lg2 + w * Lg4);
    float t2 = z * (Lg1 + w * Lg3);
    ii |= j;
    float R = t2 + t1;
    if (ii > 0) {
        float hfsq = 0.5f * f * f;
        if (k == 0) return f - (hfsq - s * (hfsq + R));
        return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
    }
    if (k == 0) return f - s * (f - R);
    return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

// Cephes cosf; valid for finite |x| < 8192 (the hot path feeds [0, 2*pi]).
PT_HD float cosf_pinned(float xx) {
    uint32_t ax = fbits(xx) & 0x7fffffffu;
    if (ax >= 0x7f800000u) return bitsf(0x7fc00000u);
    const float DP1 = 0.78515625f, DP2 = 2.4187564849853515625e-4f, DP3 = 3.77489497744594108e-8f,
                FOPI = 1.27323954473516f;
    float x = bitsf(ax);
    int j = (int)(FOPI * x);
    float y = (float)j;
    if (j & 1) { j += 1; y += 1.0f; }
    j &= 7;
    bool neg = false;
    if (j > 3) { j -= 4; neg = !neg; }
    if (j > 1) neg = !neg;
    x = ((x - y * DP1) - y * DP2) - y * DP3;
    float z = x * x;
    float r;
    if (j == 1 || j == 2) {
        r = ((-1.9515295891E-4f * z + 8.3321608736E-3f) * z - 1.6666654611E-1f) * z * x + x;
    } else {
        r = ((2.443315711809948E-005f * z - 1.388731625493765E-003f) * z + 4.166664568298827E-002f) * z * z;
        r -= 0.5f * z;
        r += 1.0f;
    }
    return neg ? -r : r;
}

// Branch-free forms of logf_pinned / cosf_pinned for the kernels' Box-Muller draw: the same
// operations on the same values, every fdlibm / Cephes branch evaluated and chosen by a
// select (a wave otherwise runs each divergent branch in turn, with exec-mask bookkeeping).
// Bit-identical to the branchy forms over their whole hot-path domains (x in {0} U
// [2^-32, 1] for log, every finite theta in [0, 2*pi] for cos): checked exhaustively on the
// host (tests/test_exact_div.py) and on the GPU (tools/verify_fastmath.hip).
//   log: fdlibm's k == 0 returns are the general k != 0 expressions with dk = +0 (RN(a - b)
//   = -RN(b - a), x - 0 = x, and 0 - (+-0) = +0 = f - f), so only the small-|f| / main and
//   ii > 0 choices remain; f == 0 (x a power of two) is the small-|f| expression at f = 0.
PT_HD float logf_bf(float x) {                     // x in {0} U [2^-32, 1]
    const float ln2_hi = 6.9313812256e-01f, ln2_lo = 9.0580006145e-06f;
    const float Lg1 = bitsf(0x3f2aaaaau), Lg2 = bitsf(0x3ecccce1u), Lg3 = bitsf(0x3e91e9eeu),
                Lg4 = bitsf(0x3e789e26u);
    int32_t ix = (int32_t)fbits(x);
    int32_t k = (ix >> 23) - 127;
    ix &= 0x007fffff;
    const int32_t i = (ix + (0x95f64 << 3)) & 0x800000;
    const float xr = bitsf((uint32_t)(ix | (i ^ 0x3f800000)));
    k += (i >> 23);
    const float f = xr - 1.0f;
    const float dk = (float)k;
    const float hi = dk * ln2_hi, lo = dk * ln2_lo;
    // main branch (2 + f in [1.58, 2.42]: exact reciprocal + Markstein, as logf_pinned)
    const float tf = 2.0f + f;
    const float s = div_mk(f, tf, rcp_fast(tf));
    const float z = s * s;
    const float w = z * z;
    const float t1 = w * (Lg2 + w * Lg4);
    const float t2 = z * (Lg1 + w * Lg3);
    const float R = t2 + t1;
    const int32_t ii = (ix - (0x6147a << 3)) | ((0x6b851 << 3) - ix);
    const float hfsq = 0.5f * f * f;
    const float m1 = hi - ((hfsq - (s * (hfsq + R) + lo)) - f);
    const float m2 = hi - ((s * (f - R) - lo) - f);
    float r = ii > 0 ? m1 : m2;
    // |f| < 2^-20 branch (x within ~2^-20 of a power of two: about 1 draw in 2^19), run
    // only when a lane of the wave needs it
    const bool is_small = (0x007fffff & (0x8000 + ix)) < 0xc000;
#if defined(__HIP_DEVICE_COMPILE__)
    if (__any(is_small))
#endif
    {
        const float Rs = f * f * (0.5f - 0.33333333333333333f * f);
        const float small = hi - ((Rs - lo) - f);
        r = is_small ? small : r;
    }
    return x == 0.0f ? bitsf(0xff800000u) : r;
}
PT_HD float cosf_bf(float xx) {                    // finite xx >= 0 (theta in [0, 2*pi])
    const float DP1 = 0.78515625f, DP2 = 2.4187564849853515625e-4f, DP3 = 3.77489497744594108e-8f,
                FOPI = 1.27323954473516f;
    const float x0 = bitsf(fbits(xx) & 0x7fffffffu);
    int j = (int)(FOPI * x0);
    float y = (float)j;
    const bool odd = (j & 1) != 0;
    j = odd ? j + 1 : j;
    y = odd ? y + 1.0f : y;
    j &= 7;
    bool neg = j > 3;
    j = j > 3 ? j - 4 : j;
    neg = (j > 1) != neg;
    const float x = ((x0 - y * DP1) - y * DP2) - y * DP3;
    const float z = x * x;
    const float rs = ((-1.9515295891E-4f * z + 8.3321608736E-3f) * z - 1.6666654611E-1f) * z * x + x;
    float rc = ((2.443315711809948E-005f * z - 1.388731625493765E-003f) * z + 4.166664568298827E-002f) * z * z;
    rc -= 0.5f * z;
    rc += 1.0f;
    const float r = (j == 1 || j == 2) ? rs : rc;
    return neg ? -r : r;
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
PT_HD bool fast_range(float q) { return q >= 0x1p-100f && q <= 0x1p100f; }
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
#if defined(__HIP_DEVICE_COMPILE__)
    float rho = sqrt_g(-2.0f * logf_bf(random01(s)));
    return rho * cosf_bf(theta);
#else
    float rho = sqrt_g(-2.0f * logf_pinned(random01(s)));
    return rho * cosf_pinned(theta);
#endif
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
