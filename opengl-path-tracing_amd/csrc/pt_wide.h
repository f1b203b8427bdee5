// pt_wide.h -- the 4-wide quantised tree of the global-memory walk, shared
// by the HIP kernel (pt_render.hip), the host builder (pt_wide.cpp) and the CPU walk model
// (tests/wide/wide_sim.cpp).
//
// The reference walks a binary tree threaded in preorder (calculateRayCollision,
// computeShader.c:389-431; links from bvh.h:221-252), testing one box per step.  On a scene
// too large for LDS every step is a scattered global-memory gather of one 32-B node -- the
// texture path's distinct cache lines per lane bound that walk.  This tree
// covers the same binary tree with 4-ary records: a record holds the boxes of up to four
// descendants (a frontier of its binary subtree, left to right), quantised to 8 bits per
// plane inside the record's own box and rounded outward.  A ray tests all four in one step
// and visits them left to right, so the leaves it reaches come in the reference's preorder.
//
// Why the result is the reference's (the argument of the culling walk): on a
// nested tree (pt_bvh_culling_ok) the reference tests exactly the leaves, in preorder, whose
// own box passes the exact slab test at the t of that moment.  The conservative child test
// here accepts every box the exact test accepts (same or larger t: t only decreases), so the
// walk reaches a superset of those leaves in the same order; a leaf reached in vain is
// rejected by the exact test of its own box, which the leaf phase runs before one of its
// triangles may move t.  Only rays inside the exact-reciprocal guard use it.
//
// Record (64 B, 3 quads used; records, leaf triangle pairs and leaf boxes share one index
// space g -- a record's children occupy g = cbase .. cbase + n - 1):
//   q0 = {O.x, O.y, O.z, w}    O = the record's box minimum; w = ex | ey << 8 | ez << 16 (int8
//                              per axis: the quantisation step 2^e) | types << 24
//   q1 = {lo.x, hi.x, lo.y, hi.y}  child j's 8-bit plane codes in byte j of each word
//   q2 = {lo.z, hi.z, cbase, exit}
// child plane j of axis i = O_i + code * 2^e_i, lo codes rounded down, hi codes up.
// types: 2 bits per child slot (bits 2j, 2j+1): 0 none, 1 record, 2 leaf, 3 leaf whose two
// triangles are coplanar (the leaf phase computes one plane distance).
// exit: where the walk resumes once this record's subtree is done, as a position (below),
// or -1 at the root.
//
// Walk state (per lane): cur, a K-entry stack e[0] (top) .. e[K-1] and a resume position R.
//   cur >= 0: visit record cur >> 3; s = cur & 7 = 0 descends into it, s in 1..4 resumes it
//             at child slot s (and sets R = its exit);
//   cur == -1: the walk is done;  cur <= -2: stopped at leaf g, code = -2 - cur = g << 1 | cop.
//   stack entry: cbase << 8 | the types of the children still pending (hit, not yet taken);
//   R: the position after everything on the stack (a record resumed at a slot), or -1.
// A push onto a full stack flushes it: R becomes "this record from the next slot on", whose
// exit chain re-tests the flushed records' remaining children (a superset again, in order).
#pragma once

#include "pt_math.h"

namespace ptw {

constexpr int kRecQuads = 4;          // float4 per record (64 B)
// pending-child stack entries per lane (measured, same-process A/B on the C3 / C4 stand-ins:
// 4 entries +0.4% / +0.2% over 3 with the optimal collapse and best-first numbering; 3 was
// +0.5% / +2.6% over 2 in round 4)
#ifndef PT_WIDE_STACK
#define PT_WIDE_STACK 4
#endif
constexpr int kStack = PT_WIDE_STACK;
constexpr int kMaxRecords = 1 << 24;  // cbase << 8 in a 32-bit stack entry

// Per-ray constants of the conservative child test: rd = RN(1/d) and the addends ord -+ E
// (ord = RN(-o * rd), E_i = 2^-18 M_i |rd_i| + 2^-16 |ord_i|, M_i the scene's largest
// |coordinate| on axis i).  Error bound: for the true child plane b and the
// quantised one b' (b' <= b for a near plane of d_i > 0, mirrored otherwise), every rounding
// of the record test -- rd, ord, ord -+ E, fma(O, rd, .), fma(code, 2^e rd, .) -- and the two
// roundings of the reference's quotient RN(RN(b - o) / d) add up to at most
// 9.2u M_i |rd_i| + 8.2u |ord_i| (u = 2^-24; |b'| <= 1.02 M_i, |code 2^e| <= 4 M_i), against
// E_i = 64u M_i |rd_i| + 256u |ord_i|: near_i <= the reference's near quotient and far_i >=
// its far quotient on every axis, so an exact hit is always a hit here.
struct WRay {
    float rdx, rdy, rdz;      // RN(1/d)
    float olx, oly, olz;      // ord - E
    float ohx, ohy, ohz;      // ord + E
    bool sx, sy, sz;          // direction sign bits (near plane = hi code)
};

PT_HD WRay make_wray(pt::f3 o, pt::f3 rd, const float cw[3], bool sx, bool sy, bool sz) {
    WRay r;
    r.rdx = rd.x; r.rdy = rd.y; r.rdz = rd.z;
    const float ordx = -(o.x * rd.x), ordy = -(o.y * rd.y), ordz = -(o.z * rd.z);
    const float ex = __builtin_fmaf(cw[0], __builtin_fabsf(rd.x), 0x1p-16f * __builtin_fabsf(ordx));
    const float ey = __builtin_fmaf(cw[1], __builtin_fabsf(rd.y), 0x1p-16f * __builtin_fabsf(ordy));
    const float ez = __builtin_fmaf(cw[2], __builtin_fabsf(rd.z), 0x1p-16f * __builtin_fabsf(ordz));
    r.olx = ordx - ex; r.oly = ordy - ey; r.olz = ordz - ez;
    r.ohx = ordx + ex; r.ohy = ordy + ey; r.ohz = ordz + ez;
    r.sx = sx; r.sy = sy; r.sz = sz;
    return r;
}

PT_HD float ubyte(uint32_t w, int j) {   // v_cvt_f32_ubyte{j}
    return (float)((w >> (8 * j)) & 0xffu);
}
PT_HD float ldexp2(float x, int e) {     // v_ldexp_f32 (exact here: no under / overflow)
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_ldexpf(x, e);
#else
    return ldexpf(x, e);
#endif
}
PT_HD float max3(float a, float b, float c) { return fmaxf(fmaxf(a, b), c); }
PT_HD float min3(float a, float b, float c) { return fminf(fminf(a, b), c); }
PT_HD float min_t(float tf, float t) {
#if defined(__HIP_DEVICE_COMPILE__)
    // min(tf, t) for non-NaN operands as one v_med3 (no canonicalising v_max on the
    // loop-carried t; both are finite or +inf inside the guard)
    return __builtin_amdgcn_fmed3f(tf, t, -__builtin_huge_valf());
#else
    return fminf(tf, t);
#endif
}

// The conservative test of a record's children at the current t: pending types (2 bits per
// slot, types of the hit children at slots >= s).  (ox, oy, oz, w) = q0, (a0..a3) = q1,
// (b0, b1) = q2.xy.
PT_HD uint32_t wide_hits(float ox, float oy, float oz, uint32_t w, uint32_t a0, uint32_t a1, uint32_t a2,
                         uint32_t a3, uint32_t b0, uint32_t b1, const WRay& r, float t, int s) {
    const int ex = (int)(int8_t)(w & 0xffu), ey = (int)(int8_t)((w >> 8) & 0xffu), ez = (int)(int8_t)((w >> 16) & 0xffu);
    const float Bx = ldexp2(r.rdx, ex), By = ldexp2(r.rdy, ey), Bz = ldexp2(r.rdz, ez);
    // near codes: lo for a positive direction, hi for a negative one
    const uint32_t nxw = r.sx ? a1 : a0, fxw = r.sx ? a0 : a1;
    const uint32_t nyw = r.sy ? a3 : a2, fyw = r.sy ? a2 : a3;
    const uint32_t nzw = r.sz ? b1 : b0, fzw = r.sz ? b0 : b1;
    uint32_t hit = 0;
    // (the near and far fmas of an axis paired into v_pk_fma_f32 -- bit for bit the same --
    // measured -10.4% / -10.9% on the C3 / C4 stand-ins: on gfx950 a packed f32 op takes the
    // VALU cycles of two, and the pairing costs moves and spills)
    const float Anx = __builtin_fmaf(ox, r.rdx, r.olx), Afx = __builtin_fmaf(ox, r.rdx, r.ohx);
    const float Any = __builtin_fmaf(oy, r.rdy, r.oly), Afy = __builtin_fmaf(oy, r.rdy, r.ohy);
    const float Anz = __builtin_fmaf(oz, r.rdz, r.olz), Afz = __builtin_fmaf(oz, r.rdz, r.ohz);
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
    for (int j = 0; j < 4; j++) {
        const float nx = __builtin_fmaf(ubyte(nxw, j), Bx, Anx), fx = __builtin_fmaf(ubyte(fxw, j), Bx, Afx);
        const float ny = __builtin_fmaf(ubyte(nyw, j), By, Any), fy = __builtin_fmaf(ubyte(fyw, j), By, Afy);
        const float nz = __builtin_fmaf(ubyte(nzw, j), Bz, Anz), fz = __builtin_fmaf(ubyte(fzw, j), Bz, Afz);
        const float tn = max3(nx, ny, nz), tf = min3(fx, fy, fz);
        hit |= (tn <= min_t(tf, t)) ? (3u << (2 * j)) : 0u;
    }
    return (w >> 24) & hit & ((0xffu << (2 * s)) & 0xffu);
}

// The leaf re-test certificate.  A leaf reached on the conservative test
// must pass the reference's exact slab test of its own box at the current t before one of
// its triangles may move t (computeShader.c:406-428 tests the leaf only then).  When the
// leaf's box contains the hit triangle's vertices (pt_upload_scene checks every leaf; the
// reference builder expands leaf boxes over them, bvh.h:29-52), each axis i is certified by
// one of:
//   margin: for the triangle's vertex interval [m_i, M_i] and the hit point p = o + d*t_h
//   (componentwise RN(o_i + RN(d_i t_h)), as the kernel forms it), if RN(p_i - m_i) and
//   RN(M_i - p_i) both clear g = 2^-20 (max_j |p_j| + max_j |o_j|) + 2^-100, then through |p - (o + s)| <=
//   2^-23 |p|, |s - d t_h| <= 2^-23 |s| (s = RN(d_i t_h)), |RN(m - o) - (m - o)| <= 2^-24 |m - o|
//   and |m_i| <= |p_i| + (p_i - m_i), RN(m_i - o_i) <= d_i t_h <= RN(M_i - o_i); the leaf box
//   contains the triangle (lo_i <= m_i, M_i <= hi_i), so RN(lo_i - o_i) <= d_i t_h <=
//   RN(hi_i - o_i), and for either sign of d_i RN's monotonicity puts the reference's near
//   quotient RN(RN(b - o)/d) of axis i at or below t_h and the far one at or above it (t_h is
//   a float).  The margin needed is below 2^-21.9 (|p_i| + |o|); g is about four times that.
//   exact axis plane: the triangle is flat on axis i (v0_i = v1_i = v2_i = c) and its stored
//   normal is exactly +-1 there (its other components are then exact zeros): the plane
//   distance -(dot(n, o) + d0) / dot(n, d) (computeShader.c:285-297) is bit for bit
//   RN(RN(c - o_i) / d_i), the reference's slab quotient of the plane c, and lo_i <= c <= hi_i
//   gives near_i <= t_h <= far_i for either sign of d_i.
// All three axes certified: max near <= t_h <= min far and t_h < t, so the exact test passes.
PT_HD float abs_max3(pt::f3 v) { return fmaxf(fmaxf(__builtin_fabsf(v.x), __builtin_fabsf(v.y)), __builtin_fabsf(v.z)); }
// Axis i: m, M = the triangle's vertex interval; RN(p - m) and RN(M - p) against g (the margin
// form), or m == M with |n_i| == 1 (the exact axis plane form).
PT_HD bool cert_axis(float p, float a, float b, float c, float n, float g) {
    const float m = fminf(fminf(a, b), c), M = fmaxf(fmaxf(a, b), c);
    return ((p - m >= g) & (M - p >= g)) | ((m == M) & (__builtin_fabsf(n) == 1.0f));
}
PT_HD bool leaf_certificate(pt::f3 p, pt::f3 n, pt::f3 v0, pt::f3 v1, pt::f3 v2, float omax) {
    const float g = 0x1p-20f * (abs_max3(p) + omax) + 0x1p-100f;
    return cert_axis(p.x, v0.x, v1.x, v2.x, n.x, g) & cert_axis(p.y, v0.y, v1.y, v2.y, n.y, g) &
           cert_axis(p.z, v0.z, v1.z, v2.z, n.z, g);
}

// One transition of the walk state, as selects: the next position from a record's hits `pend`
// (children cbase + slot; `cur` = that record's position) or, with pend == 0, from the stack
// (K entries, e[0] the top) or from R once it is empty.  One child extraction from the hits or
// the stack top, then one of push / flush / keep the top / shift up: the lanes of a wave take
// all of them at once, and the branchy form ran every path for every lane (measured: +4.3% /
// +4.6% on the C3 / C4 stand-ins over that form, the same walk).
template <int K>
PT_HD int wide_next(int cur, uint32_t pend, int cbase, uint32_t (&e)[K], int& R) {
    const bool fresh = pend != 0u;
    const uint32_t src = fresh ? (((uint32_t)cbase << 8) | pend) : e[0];
    const uint32_t p = src & 0xffu;
    const int j2 = __builtin_ctz(p | 0x100u) & ~1;
    const uint32_t ty = (p >> j2) & 3u;
    const int child = (int)(src >> 8) + (j2 >> 1);
    const uint32_t rest = src & ~(3u << j2);
    const bool more = (rest & 0xffu) != 0u;
    // a push onto a full stack flushes it: the walk resumes this record at the next slot
    const bool flush = fresh & more & (e[K - 1] != 0u);
    const bool down = fresh & more;                     // push: the others move down
    const bool up = !fresh & !more & (p != 0u);         // popped the top's last child
    uint32_t n[K];
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
    for (int k = 0; k < K; k++) {
        const uint32_t below = k + 1 < K ? e[k + 1 < K ? k + 1 : k] : 0u;
        const uint32_t v = up ? below : e[k];
        n[k] = k == 0 ? (more ? rest : v)                // rest becomes the top
                      : (down ? e[k > 0 ? k - 1 : 0] : v);
    }
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
    for (int k = 0; k < K; k++) e[k] = n[k];
    const int pos = ty == 1u ? child << 3 : -2 - ((child << 1) | (int)(ty == 3u));
    const int r = R;
    R = p ? R : -1;
    // the flush, rare, off the common path: a wave-uniform branch around its four selects
    // (+0.45% / +0.49% on the C3 / C4 stand-ins over selecting every step)
#if defined(__HIP_DEVICE_COMPILE__)
    if (__any(flush)) {
#else
    {
#endif
        if (flush) {
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
            for (int k = 0; k < K; k++) e[k] = 0u;
            R = (cur & ~7) | ((j2 >> 1) + 1);
        }
    }
    return p ? pos : r;
}

// The next position from the stack, or from R once it is empty (after a leaf).
template <int K>
PT_HD int wide_pop(uint32_t (&e)[K], int& R) {
    return wide_next<K>(0, 0u, 0, e, R);
}

// One record visit: pend = wide_hits(...) of record N = cur >> 3 at slot s = cur & 7, with
// its cbase and exit; returns the next position.
template <int K>
PT_HD int wide_visit(int cur, uint32_t pend, int cbase, int exit_, uint32_t (&e)[K], int& R) {
    R = (cur & 7) ? exit_ : R;      // a resumed record: afterwards, its exit
    return wide_next<K>(cur, pend, cbase, e, R);
}

}  // namespace ptw

// Host builder (pt_wide.cpp).  Input: the reference's std140 node records (12 floats each)
// of a nested tree (pt_bvh_culling_ok) and, per binary node, whether a leaf's two triangles
// are coplanar.  Output: n_index records / leaf slots; records as 16 floats each (q0..q3),
// leaf boxes as 8 floats each (axis-paired {min.x, max.x, min.y, max.y}, {min.z, max.z, 0,
// 0}), and per binary node its index g (leaves: the leaf's slot pair; records: the record;
// nodes inside a record: -1).  cw = 2^-18 M_i rounded up (WRay).
#include <vector>
namespace ptw {
struct WideTree {
    int n_index = 0, n_records = 0, n_leaves = 0, depth = 0;
    std::vector<float> rec;     // 16 floats per index (leaf indices unused)
    std::vector<float> lbox;    // 8 floats per index (record indices unused)
    std::vector<int> g_of;      // per binary node
    std::vector<int> bn_of;     // per index: its binary node (record or leaf)
    float cw[3] = {0, 0, 0};
};
// 0 on success; -1 when the tree does not qualify (not nested, too many records).
int wide_build(const float* bvh, int n_nodes, const unsigned char* leaf_cop, WideTree& out);
}  // namespace ptw
