// pt_render.hip -- the path-tracing hot path on MI355X (gfx950) behind the pt_api.h C ABI.
//
// Replaces LearnOpenGL/computeShader.c (main :505-554, Trace :434-501,
// calculateRayCollision :367-432, bvh_intersect :309-365, hit_triangle :274-307,
// hit_sphere :209-226, RNG :87-129) and the GL plumbing that drives it
// (ogl_path_trace.h:160-204, 367-530).  Results are bit-identical to the CPU oracle's
// restatement of those semantics; every float op is pinned via pt_math.h
// and -ffp-contract=off.
//
// Device layouts, built once at pt_upload_scene from the std140 records:
//   node  32 B : {min.x, max.x, min.y, max.y}, {min.z, max.z, a, b}   (axis-paired so a
//                slab axis is one packed-f32 register pair)
//                internal: a = hit link (left child), b = miss
//                leaf:     a = ~(slot<<1 | single), b = next
//   tri   64 B : {n.xyz, d0}, {v0.xyz, cont}, {v1.xyz, matIdx}, {v2.xyz, 0}
//                n = normalize(cross(v1-v0, v2-v0)) and d0 = -dot(n, v0) are the exact values
//                hit_triangle recomputes per call; a leaf's triangles sit in slots 2k, 2k+1;
//                the plane test reads one quad, shading two (quads 0 and 2).  cont: the LDS
//                walk's continuation of the leaf (first slot only).
//   leaf code  : k << 2 | coplanar << 1 | single (k = leaf pair index, slots 2k and 2k+1)
//   mat   48 B : {color.rgb, smoothness}, {emission*strength, specProb}, {specular.rgb, 0}
//   sphere 32 B: {c.xyz, r*r}, {matIdx, 0, 0, 0}
#include "pt_math.h"
#include "pt_wide.h"
#include "../../include/pt_api.h"
#include "../../include/pt_scene.h"

#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

using pt::f3;
using pt::mk;

namespace {

struct DevScene {
    const float4* nodes;
    // the state-machine kernel's LDS image of the same tree (pt_upload_scene): node planes
    // with WalkLinks (byte offsets, 16 * index)
    const float4* walk_lds;
    const float4* walk_sk;   // the culling walk's images: walk_lds with a ninth image of sinks
    const float4* tris;
    const float4* mats;
    const float4* spheres;
    // the 4-wide quantised tree of the global-memory walk (pt_wide.h): records (4 float4 per
    // index) and the exact leaf boxes (2 float4 per index, axis-paired like the node records)
    const float4* wrec;
    const float4* wlbox;
    int n_nodes, n_spheres;
};

struct KParams {
    DevScene sc;
    float4* accum;                 // rows_local x W
    float cam[12];                 // pos, fwd, right, up (per-dispatch constants)
    int W, H, row0, row_stride, rows_local;
    int x_limit, y_limit;          // PT_FLAG_REF_DISPATCH footprint
    int frame_first, n_frames, acc_first;
    int max_bounce, mode, flags, rpp;
    unsigned long long* counters;  // [5] when counting
    unsigned int* work_counter;    // persistent kernel pixel queue
    int n_slots, n_mats;           // triangle slots / materials (LDS staging sizes)
    int n_top;                     // global-memory scene: nodes [0, n_top) staged in LDS
    int walk_np;                   // LDS walk image: nodes per image plane (n_nodes, or kPadNodes)
    int scene_fast;                // every box coordinate inside the exact-reciprocal guard
    int leaf_thresh, shade_thresh; // wave scheduling thresholds of the state-machine kernel
    int trav_floor;                // ... and the walk floor: fewer walking lanes end a walk phase
    int compact_max;               // leaf phase: compact the edge tests of at most this many pairs (<= 63)
    int pull_batch;                // frame-split mode: queue ids a wave reserves per queue atomic (>= 32)
    unsigned* reset_work;          // k_accum_frames zeroes these queue heads (an overlap slot's) for its next use
    const int* frame_dev;          // progressive graph: device frame counter (null = use frame_first)
    int frame_offset;              // this launch's frame offset from *frame_dev
    const unsigned* tile_perm;     // queue order of the tiles, entries (ty << 16) | tx (null = raster order)
    int tile_shift;                // tiles of 64 pixels: (8 << tile_shift) columns x (8 >> tile_shift) local rows
    unsigned* tile_cost;           // per-tile segment counts of this launch (null = off)
    // frame-split work items (state-machine kernel): a queue item is (pixel, `group`
    // consecutive frames); with rgb != null the lane stores each frame's pixel colour (12 B)
    // to rgb[3 * (k * pixels + pixel)] (frame planes: the accumulate pass reads coalesced)
    // and k_accum_frames applies the running mean in frame order.
    // group = n_frames and rgb = null: the lane owns all frames and accumulates in registers.
    int group;
    float* rgb;                    // 3 floats per (frame, pixel)
    uchar4* aces_out;              // k_accum_frames: also the ACES view of the new image (or null)
    float rW, rH;                  // RN(1/W), RN(1/H) (host IEEE division) for the camera ray
    float fW, fH;                  // W, H as binary32 (kernel arguments: uniform, no VGPR)
    unsigned grp_magic;            // ceil(2^32 / n_groups) when item * n_groups < 2^32 for every item, else 0
    // root box (min.x, max.x, min.y, max.y, min.z, max.z) and its first child (-1: the root is
    // a leaf): a ray starting inside the root box hits it, so the walk may start at the child
    float root_box[6];
    int root_child;
    int shade_lds;                 // global-memory scene: materials + spheres staged in LDS too
    int cons_walk;                 // LDS scene: the culling walk (slab_oct_cons, exact leaf re-test)
    float cons_m[3];               // ... 2^-19 * the scene's largest |coordinate| per axis, rounded up
    int wide_top;                  // wide walk (WIDE instantiations): records [0, wide_top) staged in LDS
    float wide_cw[3];              // ... 2^-18 * the scene's largest |coordinate| per axis, rounded up (WRay)
    int leaf_cert;                 // culling / wide walk: skip the exact leaf re-test where the hit certifies it
};

// Progressive mode (hipGraph replay): the frame range comes from a device counter, and
// accumulate = 0 only on frame 1 -- the reference's run loop after a reset
// (ogl_path_trace.h:164,199-203).
__device__ __forceinline__ void resolve_frames(KParams& p) {
    if (p.frame_dev) {
        p.frame_first = *p.frame_dev + p.frame_offset;
        p.acc_first = p.frame_first != 1;
    }
}

__global__ void k_advance_frames(int* frame_dev, int n) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *frame_dev += n;
}

struct Cnt {
    uint32_t seg, nodes, tri, sph, hits;
    // counting-build diagnostics: per phase, wave iterations (counted once per wave by the
    // first active lane) and active lanes summed over those iterations
    uint32_t tw, tl, lw, ll, sw, sl;
    uint32_t slow;   // segments outside the exact-reciprocal guard (IEEE-division walk)
    uint32_t nan;    // segments whose ray has a NaN component (can never hit)
};
constexpr int kNumCounters = 13;

// Records one wave iteration of a phase: the first active lane adds 1 and popcount(exec).
__device__ __forceinline__ void diag_tick(uint32_t& waves, uint32_t& lanes) {
    unsigned long long e = __builtin_amdgcn_read_exec();
    if ((int)(threadIdx.x & 63) == __ffsll((long long)e) - 1) {
        waves++;
        lanes += (uint32_t)__popcll(e);
    }
}

// ------------------------------------------------------------------ intersection
// bvh_intersect (computeShader.c:309-365): the exact division/compare chain; NaN compares
// are false, which decides axis-parallel rays and zero-thickness boxes.
// (A, B) is the axis-paired node record: A = {min.x, max.x, min.y, max.y}, B = {min.z, max.z, ..}.
__device__ __forceinline__ bool slab(float4 A, float4 B, f3 o, f3 d, float cur_t) {
    float tmin = (A.x - o.x) / d.x;
    float tmax = (A.y - o.x) / d.x;
    if (tmin > tmax) { float q = tmin; tmin = tmax; tmax = q; }
    float tymin = (A.z - o.y) / d.y;
    float tymax = (A.w - o.y) / d.y;
    if (tymin > tymax) { float q = tymin; tymin = tymax; tymax = q; }
    if ((tmin > tymax) || (tymin > tmax)) return false;
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    float tzmin = (B.x - o.z) / d.z;
    float tzmax = (B.y - o.z) / d.z;
    if (tzmin > tzmax) { float q = tzmin; tzmin = tzmax; tzmax = q; }
    if ((tmin > tzmax) || (tzmin > tmax)) return false;
    if (tzmin > tmin) tmin = tzmin;
    return !(tmin > cur_t);
}

// A ray with a NaN component in o or d can never hit: every triangle distance
// -(dot(n,o)+d0)/dot(n,d) and every sphere root is NaN, and NaN fails the `t < tbest` /
// `ht > 0.0001` acceptance tests (:297, :378, :411-428).  Its walk still visits up to every
// node -- a single lane crawling the whole tree (60-70 ms on the 69k-triangle stand-in,
// the tail of its launch) -- so the render kernels skip the walk; its result (no hit, t =
// +inf) is the reference's.  Counting builds still walk, to count the node visits.
__device__ __forceinline__ bool ray_has_nan(f3 o, f3 d) {
    return (o.x != o.x) | (o.y != o.y) | (o.z != o.z) | (d.x != d.x) | (d.y != d.y) | (d.z != d.z);
}

// RayIntersectsTriangle (computeShader.c:228-272), Moller-Trumbore with EPSILON 1e-7: the
// opt-in PT_FLAG_MOLLER_TRUMBORE mode (dead code in the reference, which runs hit_triangle).
// The same operations as the oracle's mt_triangle, evaluated branch-free (the early returns
// become a select); 1/a by the guarded exact reciprocal.  -1 for a miss.  The normal it
// would return, normalize(cross(v1-v0, v2-v0)), is the stored per-triangle n.
__device__ __forceinline__ float tri_mt(float4 q0, float4 q1, float4 q2, f3 o, f3 d) {
    const float EPS = 0.0000001f;
    const f3 v0 = mk(q0.x, q0.y, q0.z), v1 = mk(q1.x, q1.y, q1.z), v2 = mk(q2.x, q2.y, q2.z);
    const f3 e1 = v1 - v0, e2 = v2 - v0;
    const f3 h = pt::cross(d, e2);
    const float a = pt::dot(e1, h);
    bool ok = !(a > -EPS && a < EPS);
    const float f = pt::fast_range(__builtin_fabsf(a)) ? pt::rcp_fast(a) : 1.0f / a;
    const f3 s = o - v0;
    const float u = f * pt::dot(s, h);
    ok = ok && !(u < 0.0f || u > 1.0f);
    const f3 q = pt::cross(s, e1);
    const float v = f * pt::dot(d, q);
    ok = ok && !(v < 0.0f || u + v > 1.0f);
    const float t = f * pt::dot(e2, q);
    ok = ok && t > EPS;
    return ok ? t : -1.0f;
}
// :548-551 running mean, per component, no contraction.
__device__ __forceinline__ float4 accumulate(float4 prev, f3 rgb, int frame, bool acc) {
    if (!acc) return make_float4(rgb.x, rgb.y, rgb.z, 1.0f);
    float ff = (float)frame;
    float w = (ff - 1.0f) / ff;
    return make_float4(prev.x * w + rgb.x / ff, prev.y * w + rgb.y / ff, prev.z * w + rgb.z / ff,
                       prev.w * w + 1.0f / ff);
}

// Non-temporal 16-B accesses (streamed data that must not evict the scene from L2/MALL).
__device__ __forceinline__ void nt_store3(float* dst, f3 v) {
    __builtin_nontemporal_store(v.x, dst);
    __builtin_nontemporal_store(v.y, dst + 1);
    __builtin_nontemporal_store(v.z, dst + 2);
}
__device__ __forceinline__ f3 nt_load3(const float* src) {
    return mk(__builtin_nontemporal_load(src), __builtin_nontemporal_load(src + 1), __builtin_nontemporal_load(src + 2));
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

template <bool COUNT>
__device__ __forceinline__ void flush_counters(const KParams& p, const Cnt& c) {
    if (!COUNT) return;
    unsigned long long v[kNumCounters] = {c.seg, c.nodes, c.tri, c.sph, c.hits, c.tw, c.tl, c.lw, c.ll, c.sw, c.sl,
                                          c.slow, c.nan};
    for (int i = 0; i < kNumCounters; i++) {
        unsigned long long s = wave_sum(v[i]);
        if ((threadIdx.x & 63) == 0) atomicAdd(&p.counters[i], s);
    }
}

// =====================================================================================
// The render kernel: a persistent state-machine kernel with path regeneration.
//
// * Work items are (pixel, group of consecutive frames); lanes pull them from a device queue
//   with wave-aggregated atomics, 8x8-pixel tiles in queue order so a wave starts on a
//   coherent tile.  A lane whose path ended regenerates the next camera ray instead of
//   idling until the wave's longest path ends.  A pixel's frames stay in order, so the
//   running mean is bit-identical.
// * Slab test in exact-reciprocal form: q = RN((b-o)/d) computed as q0 = (b-o)*rd,
//   q = fma(fma(-q0, d, b-o), rd, q0) with rd = RN(1/d) per ray (Markstein's theorem:
//   correctly rounded when no under/overflow).  The guard that makes that hold is checked
//   per ray (|d_i| in [2^-20, 2], origin components 0 or in [2^-40, 2^60]) and per scene
//   (box coordinates likewise, at upload); lanes outside it use the IEEE division chain.
//   With all quotients finite the swap/compare chain of :309-365 equals min/max form.
// * Small scenes are staged in LDS once per workgroup (ds_read instead of vector-memory
//   gathers on the dependent node->node chain).
// =====================================================================================
struct SceneView {
    const float4* nodes;
    const float4* tris;
    const float4* mats;
    const float4* spheres;
    int np, tp;    // plane strides (float4) of the state-machine kernel's LDS copy
    float cm[3];   // culling walk: 2^-19 * the scene's largest |coordinate| per axis (slab_oct_cons)
    const float4* wrec;    // wide walk: records (global), their first `wtop` staged in LDS planes
    const float4* wlbox;   // ... exact leaf boxes
    int wtop;
    float cw[3];
};

// Node / triangle-record access of the state-machine kernel.  Global memory holds AoS
// records (node = 2 float4, triangle slot = 4 float4).  Its LDS copy is split into
// planes -- node half h of node i at [h*np + i], triangle quad k of slot s at [k*tp + s] --
// so random per-lane gathers of one half/quad hit 16-B bank groups spread over all 64
// banks instead of every 2nd (nodes, 32-B stride) or 4th (triangles, 64-B stride) group.
//
// WalkLinks: in the LDS image a node's (hi.z, hi.w) are the walk's next position after a
// box hit and after a miss, as byte offsets of the node (16 * index, its lo-plane entry) or
// -1 (chain ends):
//   internal node: (first child, next-right)
//   leaf node:     (-2 - code, next-right), code = k << 2 | coplanar << 1 | single: a hit
//                  stops the walk
// so one select is the whole link step.  The leaf's continuation (its next-right) rides in
// the spare .w of its first triangle's quad 1 (beside v0).
// The LDS walk holds 8 such images, one per octant of ray directions (image k at byte
// 32 * N * k, links absolute inside their image): image k stores the bounds of each axis
// whose direction sign bit is set in k swapped, near bound first (slab_oct); image 0 is the
// reference order.  A leaf's continuation is stored as its image-0 offset.
// The global-memory walk keeps the reference links (node indices, a = ~code at a leaf):
// there the loads, not the selects, set the pace, and the reference form measured faster.
extern __shared__ float4 g_lds[];   // the state-machine kernel's scene copy (nodes first)
// Scenes of at most kPadNodes nodes get walk images padded to kPadNodes nodes per plane, so
// the hi half of a node sits at the compile-time offset 16 * kPadNodes from its lo half (an
// immediate ds_read_b128 offset instead of an address add per walk step).  67: consecutive
// images start 134 16-B granules apart, 6 mod 16, spreading them over the LDS bank groups.
#ifndef PT_PAD_NODES
#define PT_PAD_NODES 67
#endif
constexpr int kPadNodes = PT_PAD_NODES;
typedef float v4f __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const v4f lds_v4f;
template <bool LDS, bool PADN = false>
__device__ __forceinline__ void node_at(const SceneView& S, int i, float4& lo, float4& hi) {
    if (LDS) {      // i = byte offset from the LDS base, which is 0 (checked at kernel entry)
        const v4f x = *(lds_v4f*)(size_t)(unsigned)i;
        const v4f y = PADN ? *(lds_v4f*)(size_t)((unsigned)i + 16u * kPadNodes)
                           : *(lds_v4f*)(size_t)(unsigned)(i + (S.np << 4));
        lo = make_float4(x.x, x.y, x.z, x.w);
        hi = make_float4(y.x, y.y, y.z, y.w);
    } else if (i < S.np) {   // global-memory scene: a top node, staged in LDS
        const v4f x = *(lds_v4f*)(size_t)(unsigned)(i << 4);
        const v4f y = *(lds_v4f*)(size_t)(unsigned)((i + S.np) << 4);
        lo = make_float4(x.x, x.y, x.z, x.w);
        hi = make_float4(y.x, y.y, y.z, y.w);
    } else {
        lo = S.nodes[2 * i];
        hi = S.nodes[2 * i + 1];
    }
}

template <bool LDS>
__device__ __forceinline__ float4 tri_quad(const SceneView& S, int slot, int k) {
#ifdef PT_DIAG_TRIS_GLOBAL   // diagnostic build (LDS bank-conflict attribution): triangles from HBM
    return S.tris[4 * slot + k];
#else
    return LDS ? S.tris[slot + k * S.tp] : S.tris[4 * slot + k];
#endif
}

__device__ __forceinline__ float qdiv(float a, float b, float rb) {
    float q = a * rb;
    float r = __builtin_fmaf(-q, b, a);
    return __builtin_fmaf(r, rb, q);
}

// in_guard / in_range_abs: pt_math.h (one unsigned window on the bit patterns)
using pt::in_guard;
using pt::in_range_abs;

using pt::win_open;     // the hit windows 1e-4 < x < t and 1e-4 <= x < t (pt_math.h)
using pt::win_closed;

// The box tests' "tn <= tf && tn <= t" is evaluated as tn <= min(tf, t):
// one compare instead of two plus a scalar AND of their lane masks, which sat on the walk
// step's dependency chain (vector compare -> scalar AND -> vector select -> next LDS read):
// +1.5..2% on C2.  v_med3(tf, t, -inf) is min(tf, t) for non-NaN operands; inside the
// exact-reciprocal guard every quotient is finite, and t is finite or +inf.
// Scalar on purpose: packed f32 (v_pk_fma_f32) takes two passes on gfx950's SIMD-32, so
// it saves issue slots but no VALU cycles, and its broadcast operand pairs cost registers
// (measured: no gain, spills).  t is compared, not folded into the min3: fminf on a
// loop-carried value costs a canonicalizing v_max.
__device__ __forceinline__ bool slab_fast(float4 A, float4 B, f3 o, f3 d, f3 rd, float cur_t) {
    float x0 = qdiv(A.x - o.x, d.x, rd.x), x1 = qdiv(A.y - o.x, d.x, rd.x);
    float y0 = qdiv(A.z - o.y, d.y, rd.y), y1 = qdiv(A.w - o.y, d.y, rd.y);
    float z0 = qdiv(B.x - o.z, d.z, rd.z), z1 = qdiv(B.y - o.z, d.z, rd.z);
    float tn = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fminf(z0, z1));
    float tf = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fmaxf(z0, z1));
    return tn <= __builtin_amdgcn_fmed3f(tf, cur_t, -__builtin_huge_valf());   // as slab_oct_cons
}

// Slab test on an octant image of the LDS walk (WalkLinks): the node's bounds are stored
// near-first for the ray's direction signs, so the per-axis min/max of slab_fast is known
// in advance.  Equal to slab_fast for boxes with min <= max on every axis (checked at upload
// as part of the scene half of the guard): for d_i > 0 RN((min-o)/d) <= RN((max-o)/d) and for
// d_i < 0 the reverse (RN and the subtraction are monotone), so the near quotient IS the
// minimum; values only enter comparisons, where -0 == +0.
__device__ __forceinline__ bool slab_oct(float4 A, float4 B, f3 o, f3 d, f3 rd, float cur_t) {
    float xn = qdiv(A.x - o.x, d.x, rd.x), xf = qdiv(A.y - o.x, d.x, rd.x);
    float yn = qdiv(A.z - o.y, d.y, rd.y), yf = qdiv(A.w - o.y, d.y, rd.y);
    float zn = qdiv(B.x - o.z, d.z, rd.z), zf = qdiv(B.y - o.z, d.z, rd.z);
    float tn = fmaxf(fmaxf(xn, yn), zn);
    float tf = fminf(fminf(xf, yf), zf);
    return tn <= __builtin_amdgcn_fmed3f(tf, cur_t, -__builtin_huge_valf());   // as slab_oct_cons
}

// Conservative slab_oct of the culling walk.  Inside the exact-reciprocal
// guard every quotient is finite and normal or zero.  With u = 2^-24, q = RN(RN(b - o) / d)
// the exact quotient and rd = RN(1/d), the margin is folded into per-axis addends:
// near = fma(b, rd, ord - E_i), far = fma(b, rd, ord + E_i) with ord = RN(-o * rd) and
// E_i = 2^-19 M_i |rd_i| + 2^-17 |ord_i| (M_i: the largest |coordinate| of the scene on axis i,
// so |b - o| <= M_i + |o_i| and |q| <= M_i |rd_i| + 1.01 |ord_i|): the error of every fma
// quotient, 4.2u |q| + 2.1u |ord| + 2.1u E_i including the rounding of ord -+ E_i, is below
// E_i, so near <= q_near and far >= q_far on every axis, and an exact hit (tn <= tf and
// tn <= t) is always a hit here.  Only culling may use it: a node it accepts and the exact
// test rejects is walked in vain, and a leaf reached that way is rejected by the exact test
// of its own box, which the leaf phase runs before a triangle moves t.  (Measured forms:
// RN(b - o) * rd with a relative margin per node +2.2%, fma with a per-node margin +4.7%,
// this one +7.1% on C2 over the exact test.)
// ol / oh: the per-ray addends ord - E_i, ord + E_i
__device__ __forceinline__ bool slab_oct_cons(float4 A, float4 B, f3 rd, f3 ol, f3 oh, float cur_t) {
    float xn = __builtin_fmaf(A.x, rd.x, ol.x), xf = __builtin_fmaf(A.y, rd.x, oh.x);
    float yn = __builtin_fmaf(A.z, rd.y, ol.y), yf = __builtin_fmaf(A.w, rd.y, oh.y);
    float zn = __builtin_fmaf(B.x, rd.z, ol.z), zf = __builtin_fmaf(B.y, rd.z, oh.z);
    float tn = fmaxf(fmaxf(xn, yn), zn);
    float tf = fminf(fminf(xf, yf), zf);
    // one compare; fminf would add a canonicalizing v_max on the loop-carried t
    return tn <= __builtin_amdgcn_fmed3f(tf, cur_t, -__builtin_huge_valf());
}

// Byte offset of the ray's octant image in the LDS walk: image k = sx | sy << 1 | sz << 2
// holds the nodes with the bounds of each axis whose direction is negative swapped.  Only
// for rays inside the exact-reciprocal guard (d_i != 0, finite); other rays walk image 0
// (the reference order) with the reference slab.
__device__ __forceinline__ int oct_base(f3 d, int img_bytes) {
    const unsigned o = (__float_as_uint(d.x) >> 31) | ((__float_as_uint(d.y) >> 30) & 2u) |
                       ((__float_as_uint(d.z) >> 29) & 4u);
    return (int)o * img_bytes;
}

// hit_triangle split in two for the leaf phase's edge-test compaction: the plane distance
// (:285-297) and the three edge tests at that distance (:299-306), the same operations as
// tri_hit_bf in the same order, so the same bits.
template <bool LDS>
__device__ __forceinline__ float tri_plane(float4 nd, f3 o, f3 d) {    // nd: quad 0 {n, d0}
    const f3 n = mk(nd.x, nd.y, nd.z);
    return -(pt::dot(n, o) + nd.w) / pt::dot(n, d);
}
// The three edge tests (:299-306) of triangle `slot` at p with normal n: the caller has n
// from the plane test (quad 0), so only the vertices (quads 1-3) are read.
// With `cert_on` (wave-uniform) it also evaluates the leaf re-test certificate of this
// triangle at p (ptw::leaf_certificate, pt_wide.h): its vertices are at hand here.
template <bool LDS, bool CERT>
__device__ __forceinline__ bool tri_edges_at(const SceneView& S, int slot, f3 n, f3 p, bool cert_on, float omax,
                                             bool& cert) {
    const float4 q1 = tri_quad<LDS>(S, slot, 1), q2 = tri_quad<LDS>(S, slot, 2), q3 = tri_quad<LDS>(S, slot, 3);
    const f3 v0 = mk(q1.x, q1.y, q1.z), v1 = mk(q2.x, q2.y, q2.z), v2 = mk(q3.x, q3.y, q3.z);
    const float e0 = pt::dot(n, pt::cross(v1 - v0, p - v0));
    const float e1 = pt::dot(n, pt::cross(v2 - v1, p - v1));
    const float e2 = pt::dot(n, pt::cross(v0 - v2, p - v2));
    if (CERT && cert_on) cert = ptw::leaf_certificate(p, n, v0, v1, v2, omax);
    return (e0 > 0.0f) & (e1 > 0.0f) & (e2 > 0.0f);
}
// The lane's index in its wave, recomputed where it is used (two VALU): a value held across
// the state-machine loop is spilled to scratch at 7 waves per SIMD, and its reload sat in
// the leaf and queue paths.  Volatile, so the compiler neither hoists nor merges it.
__device__ __forceinline__ int lane_id() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}
// Number of set bits of m below this lane.
__device__ __forceinline__ int rank_in(unsigned long long m) {
    return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}
__device__ __forceinline__ float fperm_f(int dst_bytes, float v) {
    return __int_as_float(__builtin_amdgcn_ds_permute(dst_bytes, __float_as_int(v)));
}

// The leaf phase of calculateRayCollision (:406-429) for the lanes at a leaf (`at`), with the
// edge tests compacted over the wave.  A leaf's 2-way choice
//   c1 = h1 > 1e-4 && h1 < t && (h1 < h2 || h2 < 1e-4),  c2 = !c1 && h2 > 1e-4 && h2 < t
// only depends on a triangle's edge verdict when its plane distance lies in (1e-4, t) for the
// first triangle and in [1e-4, t) for the second (outside those ranges both verdicts give the
// same c1 / c2: h1 <= 1e-4 fails c1 either way; h2 < 1e-4 or a miss (-1) both satisfy
// `h2 < 1e-4` and fail c2).  About 47% of the triangle tests of a Cornell frame need them
// (81% with the plain t >= 0 cull: a bounce ray starts ON the surface it left, at a plane
// distance near 0).  The wave's needed (lane, triangle) pairs are packed onto its first lanes
// -- forward permutes hand each worker lane its pair's hit point o + d*t and slot -- so one
// pass of edge tests serves both triangles of every lane; a ballot returns the verdicts.  More than 63 pairs: each lane tests its own.  Every edge
// test runs the same operations on the same values as at its source lane: the same bits.
// Returns (through h1 / h2) the hit_triangle results up to that equivalence.
// nda: quad 0 {n, d0} of slot s0; cop: the leaf code's coplanar bit.
// cert_on (wave-uniform): also return each triangle's leaf re-test certificate (ca / cb, for
// a triangle whose edge tests pass; omax = max_i |o_i|), computed by the lane that tests it.
template <bool LDS, bool CERT>
__device__ __forceinline__ void leaf_pair_tests(const SceneView& S, bool at, int s0, float4 nda, bool cop,
                                                f3 o, f3 d, float t, int max_pairs, float& h1, float& h2,
                                                bool cert_on, bool& cta, bool& ctb) {
    float ta = 0.0f, tb = 0.0f;
    if (at) ta = tri_plane<LDS>(nda, o, d);
    // a coplanar pair (n and d0 equal up to the sign of zero components, flagged at upload)
    // has the same plane distance wherever it can pass the acceptance tests, so the second
    // one is only computed when some lane's leaf is not such a pair.  Its edge tests may use
    // the first triangle's n: a zero factor of either sign cannot change a `> 0` verdict.
    float4 ndb = nda;
    if (__any(at & !cop)) {
        if (at & !cop) {
            ndb = tri_quad<LDS>(S, s0 + 1, 0);
            tb = tri_plane<LDS>(ndb, o, d);
        }
    }
    tb = cop ? ta : tb;
    const f3 na3 = mk(nda.x, nda.y, nda.z), nb3 = mk(ndb.x, ndb.y, ndb.z);
    const bool na = at & win_open(ta, t);
    const bool nb = at & win_closed(tb, t);
    const unsigned long long ma = __ballot(na), mb = __ballot(nb);
    const int ca = __popcll(ma), n = ca + __popcll(mb);
    bool oka = false, okb = false;
    const float omax = ptw::abs_max3(o);
    if (n <= max_pairs) {      // max_pairs <= 63 (tuning key 7; 0 = every lane tests its own)
        const int lane = lane_id();
        const int ja = rank_in(ma), jb = ca + rank_in(mb);
        // forward permutes hand worker j its pair's hit point o + d*t and slot; lanes
        // without a pair send to lane 63, never a worker (n <= 63)
        const int da = (na ? ja : 63) << 2, db = (nb ? jb : 63) << 2;
        const f3 pa = o + d * ta, pb = o + d * tb;
        const bool first = lane < ca;
        // (all eight permutes run on the full wave: a permute only moves data between
        // active lanes, so none of them may sit under the `first` select)
        const float ax = fperm_f(da, pa.x), ay = fperm_f(da, pa.y), az = fperm_f(da, pa.z);
        const float bx = fperm_f(db, pb.x), by = fperm_f(db, pb.y), bz = fperm_f(db, pb.z);
        const int as = __builtin_amdgcn_ds_permute(da, s0), bs = __builtin_amdgcn_ds_permute(db, s0 + 1);
        const f3 wp = first ? mk(ax, ay, az) : mk(bx, by, bz);
        const int ws = first ? as : bs;
        // the worker's normal: re-read from LDS, or for a global-memory scene (where the
        // loads, not the permutes, set the pace) handed over with the hit point
        f3 wn;
        if (LDS) {
            const float4 q0 = tri_quad<LDS>(S, ws, 0);
            wn = mk(q0.x, q0.y, q0.z);
        } else {
            const float nax = fperm_f(da, na3.x), nay = fperm_f(da, na3.y), naz = fperm_f(da, na3.z);
            const float nbx = fperm_f(db, nb3.x), nby = fperm_f(db, nb3.y), nbz = fperm_f(db, nb3.z);
            wn = first ? mk(nax, nay, naz) : mk(nbx, nby, nbz);
        }
        bool pass = false, cert = false;
        float wom = 0.0f;
        if (CERT && cert_on) {
            const float oa = fperm_f(da, omax), ob = fperm_f(db, omax);
            wom = first ? oa : ob;
        }
        if (lane < n) pass = tri_edges_at<LDS, CERT>(S, ws, wn, wp, cert_on, wom, cert);
        const unsigned long long r = __ballot(pass);
        oka = na & (((r >> ja) & 1ull) != 0ull);
        okb = nb & (((r >> jb) & 1ull) != 0ull);
        if (CERT && cert_on) {
            const unsigned long long rc = __ballot(pass & cert);
            cta = oka & (((rc >> ja) & 1ull) != 0ull);
            ctb = okb & (((rc >> jb) & 1ull) != 0ull);
        }
    } else {
        if (na) oka = tri_edges_at<LDS, CERT>(S, s0, na3, o + d * ta, cert_on, omax, cta);
        if (nb) okb = tri_edges_at<LDS, CERT>(S, s0 + 1, nb3, o + d * tb, cert_on, omax, ctb);
        cta = cta & oka;
        ctb = ctb & okb;
    }
    h1 = oka ? ta : -1.0f;
    h2 = okb ? tb : -1.0f;
}

// =====================================================================================
// The state machine (variants 0 and 3).  Every lane carries one path through three
// states -- TRAV (walking the link chain), LEAF (stopped at a leaf whose box it hit), SHADE
// (segment finished: shade / regenerate / set up the next segment) -- and each wave
// iteration runs ONE phase for the lanes in that state, picked by ballot counts:
//   SHADE when >= shade_thresh lanes wait to shade (or nothing else is runnable),
//   LEAF  when >= leaf_thresh lanes wait at leaves (or no lane is walking),
//   TRAV  otherwise (an inner walk loop that yields when either threshold is reached).
// A lane's own operation sequence is exactly the reference's (node, leaf tests before the
// next node, same t), so results are bit-identical; only lane interleaving changes.
// =====================================================================================
enum : int { ST_DONE = 0, ST_TRAV = 1, ST_LEAF = 2, ST_SHADE = 3 };
constexpr unsigned kPullBatch = 32;
// work-queue head stride (unsigned): each context stream / overlap slot has its own head on
// its own 128-B line
constexpr int kQueueStride = 32;
#ifndef PT_WALK_UNROLL
#define PT_WALK_UNROLL 4
#endif
#ifndef PT_SINK_UNROLL
#define PT_SINK_UNROLL 6    // its node steps per yield check (measured: 4 -2.2%, 8 -1.4% against 6)
#endif
constexpr int kWalkUnroll = PT_WALK_UNROLL;   // node steps per yield check of the walk (measured: 1 -> 2 +3.6%, 4 +5.7%, 6/8 slower)

// The TRAV phase: each TRAV lane advances one node per iteration (bvh_intersect + the link
// choice of calculateRayCollision :389-431) until it stops at a leaf whose box it hit
// (-> LEAF) or its walk ends (-> SHADE).  The wave yields once leaf_thresh lanes wait at
// leaves or shade_thresh lanes wait to shade; lanes only ever leave TRAV here, so the two
// separate counts are needed only once the waiting total reaches the smaller threshold.
// ALL_FAST: every walking lane is inside the exact-reciprocal guard (wave-uniform).
// No step counter: the reference's `steps < numNodes` bound (:393) can never bind on an
// accepted scene -- pt_upload_scene rejects link graphs with a cycle, and a walk in an
// acyclic graph visits each node at most once.  The transition is select-only; `leaf`
// keeps the raw link (~code), decoded in LEAF.
// CONS (LDS scenes, never counting): the culling walk -- lanes inside the guard test every
// node with slab_oct_cons; a leaf they stop at is re-tested exactly in the leaf phase.
template <bool ALL_FAST, bool COUNT, bool LDS, bool PADN, bool CONS = false>
__device__ __forceinline__ void trav_walk(const SceneView& S, f3 o, f3 d, f3 rd, bool fast, float t,
                                          unsigned long long live, unsigned long long m_trav,
                                          unsigned long long m_leaf, unsigned long long m_shade,
                                          int leaf_thresh, int shade_thresh,
                                          int trav_floor, int& st, int& bi, int& leaf, Cnt& c,
                                          bool eligible = true) {
    const int min_thresh = leaf_thresh < shade_thresh ? leaf_thresh : shade_thresh;
    f3 ol = mk(0, 0, 0), oh = mk(0, 0, 0);
    if (CONS) {   // S.cm[i] = 2^-19 M_i (slab_oct_cons)
        const f3 ord = mk(-(o.x * rd.x), -(o.y * rd.y), -(o.z * rd.z));
        const f3 e = mk(__builtin_fmaf(S.cm[0], __builtin_fabsf(rd.x), 0x1p-17f * __builtin_fabsf(ord.x)),
                        __builtin_fmaf(S.cm[1], __builtin_fabsf(rd.y), 0x1p-17f * __builtin_fabsf(ord.y)),
                        __builtin_fmaf(S.cm[2], __builtin_fabsf(rd.z), 0x1p-17f * __builtin_fabsf(ord.z)));
        ol = ord - e;
        oh = ord + e;
    }
    // Inside the walk one register carries the lane's state (WalkLinks): w >= 0 the next
    // node, w == -1 the chain ended (-> SHADE), w <= -2 stopped at the hit leaf with code
    // -2 - w (-> LEAF, bi = w).  st / bi are written back once at the end.
    // The culling walk's images end in sinks instead (pt_upload_scene): w < sink0 walks,
    // w == sink0 ended, w == sink0 + 16 (1 + k) stopped at leaf pair k; a stopped lane steps
    // in place, so the step runs unmasked.
    const int sink0 = (PADN ? kPadNodes : S.np) << 8;
    // LDS walks take the lane masks of the three states from the phase choice (uniform values:
    // no per-lane booleans copied into the walk loop, +1.2..1.5% on C2); the global-memory walk
    // measured 0.8-1% slower that way and keeps its own ballots
    // (eligible: the wide walk's scenes send only the lanes outside the exact-reciprocal guard
    // here, and the walking lanes inside it wait)
    const bool walking = (st == ST_TRAV) & eligible;
    const unsigned long long mw = LDS ? m_trav : __ballot(walking);
    const unsigned long long pre_leaf = LDS ? m_leaf : __ballot(st == ST_LEAF);
    const unsigned long long pre_shade = LDS ? m_shade : __ballot(st == ST_SHADE);
    int w = walking ? bi : (CONS ? sink0 : -1);
    // the yield test in counts: the walkers (ballot of w < sink0, or w >= 0) are live lanes, so
    // the lanes waiting elsewhere number popc(live) - walkers, and "waiting >= min_thresh" is
    // walkers <= popc(live) - min_thresh; floor1 >= 1 also covers "no walker left" (fewer
    // scalar instructions per yield check than the mask form)
    const int floor1 = trav_floor > 1 ? trav_floor : 1;
    const int wait_lim = __popcll(live) - min_thresh;
    if (CONS) {
        auto sstep = [&]() {
            float4 lo, hi;
            node_at<LDS, PADN>(S, w, lo, hi);
            const int a = __float_as_int(hi.z), b = __float_as_int(hi.w);
            const bool hb = (ALL_FAST || fast) ? slab_oct_cons(lo, hi, rd, ol, oh, t) : slab(lo, hi, o, d, t);
#ifdef PT_PHASE_CLOCK
            if (w < sink0) diag_tick(c.tw, c.tl);
#endif
            w = hb ? a : b;
        };
        for (;;) {
#pragma unroll
            for (int u = 0; u < PT_SINK_UNROLL; u++) sstep();
            const int nw = __popcll(__ballot(w < sink0));
            if (nw < floor1) break;
            if (nw <= wait_lim) {
                if (__popcll(pre_leaf | __ballot(w > sink0)) >= leaf_thresh) break;
                if (__popcll(pre_shade | (__ballot(w == sink0) & mw)) >= shade_thresh) break;
            }
        }
        if (walking) {
            st = w < sink0 ? ST_TRAV : (w == sink0 ? ST_SHADE : ST_LEAF);
            bi = w;
            leaf = ((w - sink0) >> 4) - 1;   // the leaf pair
        }
        return;
    }
    auto step = [&]() {
        if (!LDS && !COUNT && ALL_FAST) {
            // global-memory walk without the per-step exec-mask branch: a lane whose walk has
            // stopped (w < 0) steps on the root, an LDS top node (S.np >= 1 for any tree), and
            // keeps its w and leaf
            const bool on = w >= 0;
            float4 lo, hi;
            node_at<LDS, PADN>(S, on ? w : 0, lo, hi);
            const int a = __float_as_int(hi.z), b = __float_as_int(hi.w);
            const bool hb = slab_fast(lo, hi, o, d, rd, t);
            leaf = on ? a : leaf;
            w = on ? (hb ? (a >= 0 ? a : -3 - b) : b) : w;
            return;
        }
        if (w >= 0) {
            float4 lo, hi;
            node_at<LDS, PADN>(S, w, lo, hi);
            int a = __float_as_int(hi.z), b = __float_as_int(hi.w);
            bool hb = (ALL_FAST || fast) ? (LDS ? (CONS ? slab_oct_cons(lo, hi, rd, ol, oh, t)
                                                        : slab_oct(lo, hi, o, d, rd, t))
                                                 : slab_fast(lo, hi, o, d, rd, t))
                                         : slab(lo, hi, o, d, t);
            if (COUNT) { c.nodes++; diag_tick(c.tw, c.tl); }
#ifdef PT_PHASE_CLOCK
            if (!COUNT) diag_tick(c.tw, c.tl);
#endif
            if (LDS) {
                w = hb ? a : b;                       // WalkLinks: one select
            } else {                                  // reference links: a = ~code at a leaf
                leaf = a;
                w = hb ? (a >= 0 ? a : -3 - b) : b;
            }
        }
    };
    for (;;) {
#pragma unroll
        for (int u = 0; u < kWalkUnroll; u++) step();
        const int nw = __popcll(__ballot(w >= 0));
        if (nw < floor1) break;                   // too few walkers (or none): run a waiting phase
        if (nw <= wait_lim) {
            if (__popcll(pre_leaf | __ballot(w <= -2)) >= leaf_thresh) break;
            if (__popcll(pre_shade | (__ballot(w == -1) & mw)) >= shade_thresh) break;
        }
    }
    if (walking) {
        st = w >= 0 ? ST_TRAV : (w == -1 ? ST_SHADE : ST_LEAF);
        if (LDS) {
            bi = w;
            leaf = -2 - w;                // the leaf's code
        } else {
            bi = w >= -1 ? w : -3 - w;    // the leaf's continuation; leaf = ~code
        }
    }
}

// ------------------------------------------------------------------ the wide walk
// Global-memory scenes whose tree is nested (pt_bvh_culling_ok) walk the 4-wide quantised tree
// of pt_wide.h: one 48-B record per step tests up to four descendants
// conservatively, and the lane keeps a two-entry stack of pending children plus a resume
// position.  Lanes inside the exact-reciprocal guard only; their leaf boxes are re-tested
// exactly in the leaf phase before a triangle may move t.  The first `wtop` records sit in
// LDS as three planes (q0 at [i], q1 at [wtop + i], q2 at [2 wtop + i]).
// (measured, same-process A/B on the C3 / C4 stand-ins: stack depth 3 and three record visits
// per yield check with packed 48-B records +3.5% / +3.9% over depth 2, two visits, 64-B
// stride; each alone +0.5 / +2.6% (depth), +1.3 / -0.2% (unroll), +0.5 / +0.3% (stride))
constexpr int kWideStack = ptw::kStack;   // pt_wide.h (PT_WIDE_STACK)
// float4 per device record: the three quads of pt_wide.h packed (48 B) or on a 64-B stride
#ifndef PT_WIDE_STRIDE
#define PT_WIDE_STRIDE 3
#endif
constexpr int kWideStride = PT_WIDE_STRIDE;
#ifndef PT_WIDE_UNROLL
#define PT_WIDE_UNROLL 3
#endif
__device__ __forceinline__ void wrec_at(const SceneView& S, int n, float4& q0, float4& q1, float4& q2) {
    if (n < S.wtop) {
        const unsigned b = (unsigned)n << 4, k = (unsigned)S.wtop << 4;
        const v4f x = *(lds_v4f*)(size_t)b;
        const v4f y = *(lds_v4f*)(size_t)(b + k);
        const v4f z = *(lds_v4f*)(size_t)(b + 2u * k);
        q0 = make_float4(x.x, x.y, x.z, x.w);
        q1 = make_float4(y.x, y.y, y.z, y.w);
        q2 = make_float4(z.x, z.y, z.z, z.w);
    } else {
        const float4* r = S.wrec + kWideStride * n;
        q0 = r[0];
        q1 = r[1];
        q2 = r[2];
    }
}

// The TRAV phase of the wide walk (every walking lane inside the guard): each lane visits one
// record per step (ptw::wide_hits + wide_visit, the functions the CPU model in
// tests/wide/wide_sim.cpp checks against the reference walk) until it stops at a leaf (-> LEAF)
// or its walk ends (-> SHADE).  Stopped lanes step on record 0 (in LDS) without changing their
// state.  The yield rule is trav_walk's.
__device__ __forceinline__ void trav_wide(const SceneView& S, f3 o, f3 rd, float t, unsigned long long live,
                                          int leaf_thresh, int shade_thresh, int trav_floor, int& st, int& bi,
                                          uint32_t (&e)[kWideStack], int& R) {
    const int min_thresh = leaf_thresh < shade_thresh ? leaf_thresh : shade_thresh;
    const ptw::WRay wr = ptw::make_wray(o, rd, S.cw, rd.x < 0.0f, rd.y < 0.0f, rd.z < 0.0f);
    const bool walking = st == ST_TRAV;
    const unsigned long long mw = __ballot(walking);
    const unsigned long long pre_leaf = __ballot(st == ST_LEAF), pre_shade = __ballot(st == ST_SHADE);
    int cur = walking ? bi : -1;
    const int floor1 = trav_floor > 1 ? trav_floor : 1;
    const int wait_lim = __popcll(live) - min_thresh;
    for (;;) {
#pragma unroll
        for (int u = 0; u < PT_WIDE_UNROLL; u++) {
            const bool on = cur >= 0;
            float4 q0, q1, q2;
            wrec_at(S, on ? cur >> 3 : 0, q0, q1, q2);
            const uint32_t pend = ptw::wide_hits(q0.x, q0.y, q0.z, __float_as_uint(q0.w), __float_as_uint(q1.x),
                                                 __float_as_uint(q1.y), __float_as_uint(q1.z), __float_as_uint(q1.w),
                                                 __float_as_uint(q2.x), __float_as_uint(q2.y), wr, t, cur & 7);
            if (on) cur = ptw::wide_visit<kWideStack>(cur, pend, __float_as_int(q2.z), __float_as_int(q2.w), e, R);
        }
        const int nw = __popcll(__ballot(cur >= 0));
        if (nw < floor1) break;
        if (nw <= wait_lim) {
            if (__popcll(pre_leaf | __ballot(cur <= -2)) >= leaf_thresh) break;
            if (__popcll(pre_shade | (__ballot(cur == -1) & mw)) >= shade_thresh) break;
        }
    }
    if (walking) {
        st = cur >= 0 ? ST_TRAV : (cur == -1 ? ST_SHADE : ST_LEAF);
        bi = cur;
    }
}

#ifdef PT_PHASE_CLOCK
// experiment builds only (tools/ab_build.sh with PT_EXTRA=-DPT_PHASE_CLOCK): per-phase
// wave-clock accounting of the state machine, read back by pt_debug_phase_clock
__device__ unsigned long long g_phase_clk[8];
#endif

#ifdef PT_WAVE_TRACE
// experiment builds only (-DPT_WAVE_TRACE): per wave of the last render launch, the wall clock
// (s_memrealtime, 100 MHz) at kernel entry, after the LDS staging and at exit, and the work
// items it took; read back by pt_debug_wave_trace
constexpr int kWaveTraceMax = 16384;
__device__ unsigned long long g_wave_trace[kWaveTraceMax * 4];
#endif

template <bool COUNT, bool LDS, int MINW, bool MULTI, bool SPLIT, bool PADN = false, int NT = 256, bool WIDE = false>
__global__ __launch_bounds__(NT, MINW) void k_render_sm(KParams p) {
    static_assert(!WIDE || (!LDS && !COUNT), "the wide walk is the global-memory walk of a render build");
#ifdef PT_WAVE_TRACE
    const unsigned long long wt_entry = __builtin_amdgcn_s_memrealtime();
    unsigned wt_items = 0;
#endif
    resolve_frames(p);
    extern __shared__ float4 lds[];
    SceneView S;
    if (LDS) {      // planes (see node_at / tri_quad)
        // node_at addresses LDS by raw offset: the dynamic LDS block must start at offset 0
        if ((unsigned)(size_t)(__attribute__((address_space(3))) const char*)g_lds != 0u) __builtin_trap();
        // 8 octant images (the culling walk: + its sink image)
        const int N = PADN ? kPadNodes : p.walk_np, T = p.n_slots, nt = 4 * T;
        const bool sk = !COUNT && p.cons_walk;
        const int nn = sk ? 18 * N : 16 * N;
        const float4* wsrc = sk ? p.sc.walk_sk : p.sc.walk_lds;
        const int nm = 3 * p.n_mats, ns = 2 * p.sc.n_spheres;
        for (int i = threadIdx.x; i < nn; i += blockDim.x) lds[i] = wsrc[i];   // ready-made image
        for (int i = threadIdx.x; i < nt; i += blockDim.x) lds[nn + (i & 3) * T + (i >> 2)] = p.sc.tris[i];
        for (int i = threadIdx.x; i < nm; i += blockDim.x) lds[nn + nt + i] = p.sc.mats[i];
        for (int i = threadIdx.x; i < ns; i += blockDim.x) lds[nn + nt + nm + i] = p.sc.spheres[i];
        __syncthreads();
        S.nodes = lds;
        S.tris = lds + nn;
        S.mats = lds + nn + nt;
        S.spheres = lds + nn + nt + nm;
        S.np = N;
        S.tp = T;
#ifdef PT_DIAG_TRIS_GLOBAL
        S.tris = p.sc.tris;
#endif
#ifdef PT_DIAG_SHADE_GLOBAL  // diagnostic build: materials and spheres from HBM
        S.mats = p.sc.mats;
        S.spheres = p.sc.spheres;
#endif
        S.cm[0] = p.cons_m[0];
        S.cm[1] = p.cons_m[1];
        S.cm[2] = p.cons_m[2];
    } else {
        S.nodes = p.sc.nodes;     // reference layout; the walk image is for LDS only
        S.tris = p.sc.tris;
        S.mats = p.sc.mats;
        S.spheres = p.sc.spheres;
        S.wrec = p.sc.wrec;
        S.wlbox = p.sc.wlbox;
        S.cw[0] = p.wide_cw[0];
        S.cw[1] = p.wide_cw[1];
        S.cw[2] = p.wide_cw[2];
        if ((unsigned)(size_t)(__attribute__((address_space(3))) const char*)g_lds != 0u) __builtin_trap();
        // the top nodes (breadth-first numbering) in LDS planes: lo at [i], hi at [n_top + i];
        // the wide walk stages its top records instead (wrec_at), and the binary walk of its
        // lanes outside the guard reads every node from global memory
        const int K = WIDE ? p.wide_top : p.n_top;
        if (WIDE) {
            for (int i = threadIdx.x; i < 3 * K; i += blockDim.x) lds[(i % 3) * K + i / 3] = p.sc.wrec[kWideStride * (i / 3) + i % 3];
        } else {
            for (int i = threadIdx.x; i < 2 * K; i += blockDim.x) lds[(i & 1) * K + (i >> 1)] = p.sc.nodes[i];
        }
        const int KQ = WIDE ? 3 * K : 2 * K;   // float4 before the shading records
        // materials and spheres after them when small (p.shade_lds): every segment's sphere
        // test and every hit's material then read LDS, not scattered global lines (the global
        // walk is bound by its vector-memory lane-loads)
        if (p.shade_lds) {
            const int nm = 3 * p.n_mats, ns = 2 * p.sc.n_spheres;
            for (int i = threadIdx.x; i < nm; i += blockDim.x) lds[KQ + i] = p.sc.mats[i];
            for (int i = threadIdx.x; i < ns; i += blockDim.x) lds[KQ + nm + i] = p.sc.spheres[i];
            S.mats = lds + KQ;
            S.spheres = lds + KQ + nm;
        }
        __syncthreads();
        S.np = WIDE ? 0 : K;
        S.wtop = WIDE ? K : 0;
        S.tp = 0;
    }
#ifdef PT_PHASE_CLOCK
    const int lane = threadIdx.x & 63;
#endif
    const f3 cpos = mk(p.cam[0], p.cam[1], p.cam[2]), cfwd = mk(p.cam[3], p.cam[4], p.cam[5]);
    const f3 cright = mk(p.cam[6], p.cam[7], p.cam[8]), cup = mk(p.cam[9], p.cam[10], p.cam[11]);
    const int tsh = p.tile_shift, tw = 8 << tsh, th = 8 >> tsh;   // tile: tw columns x th local rows
    const int tiles_x = (p.W + tw - 1) >> (3 + tsh);
    const unsigned n_groups = SPLIT ? (unsigned)((p.n_frames + p.group - 1) / p.group) : 1u;
    const unsigned total_ids = (unsigned)tiles_x * (unsigned)((p.rows_local + th - 1) >> (3 - tsh)) * n_groups * 64u;
    const int n_nodes = p.sc.n_nodes;
    const bool use_tris = !(p.flags & PT_FLAG_NO_TRIANGLES) && n_nodes > 0;
    // walk start for a ray inside the root box: its first child (the counting build walks
    // from the root, so the counts stay the reference's)
    const int root_skip = (COUNT || p.root_child < 0) ? -1 : p.root_child << (LDS ? 4 : 0);
#ifdef PT_WAVE_TRACE
    const unsigned long long wt_staged = __builtin_amdgcn_s_memrealtime();
#endif

    Cnt c = {0, 0, 0, 0, 0};
    int st = ST_SHADE;
    // "fresh" (SHADE without a segment to finish: start / after shading) is t < 0, and "a new
    // camera ray is due" is bounce < 0: no lane-mask booleans carried around the loop (their
    // merges cost scalar instructions on every iteration)
    int lx = -1, y = 0;
    int aidx = 0;             // rows_local * W < 2^31 (checked at pt_create)
    int k = 0, kend = 0, r = 0, bounce = -1;   // frames k..kend-1 of this work item
    unsigned qnext = 0, qend = 0;             // wave's reserved queue ids (frame-split mode)
    unsigned tile_id = 0, pcost = 0;    // adaptive queue order: this pixel's tile + segments
    float4 acc = make_float4(0, 0, 0, 0);
    f3 psum = mk(0, 0, 0), o = mk(0, 0, 0), d = mk(0, 0, 1), inc = mk(0, 0, 0), col = mk(1, 1, 1);
    uint32_t state = 0;
    // segment state.  Only the closest primitive and its t are carried; the hit point, the
    // normal and the material are rebuilt at shading time from them with the operations
    // the reference performs when it accepts the hit (o + d*t; the stored/recomputed
    // normal and its flip against d; matIdx), on the same final t -- the same bits.
    //   hprim >= 0: triangle slot, -1: no hit, <= -2: sphere (-2 - index)
    f3 rd = mk(0, 0, 0);
    float t = -1.0f;
    int hprim = -1, bi = -1, leaf = 0;   // bi: walk position (WalkLinks); leaf: code of a hit leaf
    // wide walk (lanes inside the guard): bi is its position (pt_wide.h), plus the stack and R
    uint32_t we[kWideStack] = {};
    int wR = -1;

#ifdef PT_PHASE_CLOCK
    unsigned long long clk[6] = {0, 0, 0, 0, 0, 0};   // cycles + wave iterations per phase
#endif
    for (;;) {
        // inside the exact-reciprocal guard (the segment's "fast" walk) <=> rd was set: |d_i| is
        // in [2^-20, 2] there, so RN(1/d_x) is nonzero; outside it rd stays 0
        const bool fast = rd.x != 0.0f;
        const unsigned long long mS = __ballot(st == ST_SHADE), mL = __ballot(st == ST_LEAF), mT = __ballot(st == ST_TRAV);
        int nS = __popcll(mS);
        int nL = __popcll(mL);
        int nT = __popcll(mT);
        if (nS + nL + nT == 0) break;
#ifdef PT_PHASE_CLOCK
        const unsigned long long clk_t0 = clock64();
        int clk_ph = 2;
        if (nS > 0 && (nS >= p.shade_thresh || (nT < p.trav_floor && nL == 0))) clk_ph = 0;
        else if (nL > 0 && (nL >= p.leaf_thresh || nT < p.trav_floor)) clk_ph = 1;
#endif
        // phase choice: SHADE / LEAF once their thresholds are reached, otherwise TRAV while
        // at least trav_floor lanes walk; below the floor the leaf phase runs if any lane
        // waits at a leaf, else shading (trav_floor 1 = walk until no lane walks)
        const bool low = nT < p.trav_floor;
        if (nS > 0 && (nS >= p.shade_thresh || (low && nL == 0))) {
            // ---------------- SHADE: finish segment, regenerate, set up next segment
            if (st == ST_SHADE && !(t < 0.0f)) {   // a finished segment (t < 0: fresh)
                const bool hit = hprim != -1;
                if (COUNT) { c.seg++; if (hit) c.hits++; diag_tick(c.sw, c.sl); }
                pcost++;
                bool finished = false;
                f3 rgb = inc;
                if (hit && pt::length_gt_001(col)) {
                    const f3 hitp = o + d * t;
                    f3 normal;
                    int mat;
                    if (hprim >= 0) {             // triangle: stored n, flipped (:421-428)
                        const float4 nq = tri_quad<LDS>(S, hprim, 0);
                        normal = mk(nq.x, nq.y, nq.z);
                        mat = __float_as_int(tri_quad<LDS>(S, hprim, 2).w);
                    } else {                      // sphere: normalize(hit - center) (:380)
                        const int si = -2 - hprim;
                        float4 s0 = S.spheres[2 * si];
                        normal = pt::normalize(hitp - mk(s0.x, s0.y, s0.z));
                        mat = __float_as_int(S.spheres[2 * si + 1].x);
                    }
                    if (pt::dot(normal, d) > 0.0f) normal = normal * -1.0f;
                    if (p.mode == 2) {
                        rgb = (normal + mk(1, 1, 1)) * 0.5f;
                        finished = true;
                    } else if (p.mode == 4) {
                        float s = pt::length(hitp - o);
                        float dist = 1.0f - pt::fsqrt(s + 1.0f) / (s + 1.0f);
                        float q = dist * dist;
                        rgb = mk(q, q, q);
                        finished = true;
                    } else {
                        o = hitp;
                        f3 diffuse = pt::normalize(normal + pt::random_unit_vector(state));
                        float kk = 2.0f * pt::dot(normal, d);
                        f3 specular = pt::normalize(d - normal * kk);
                        float4 m0 = S.mats[3 * mat], m1 = S.mats[3 * mat + 1], m2 = S.mats[3 * mat + 2];
                        if (p.mode == 3) {
                            rgb = mk(m0.x, m0.y, m0.z);
                            finished = true;
                        } else {
                            float is_spec = (m1.w > pt::random01(state)) ? 1.0f : 0.0f;
                            d = pt::mix(diffuse, specular, m0.w * is_spec);
                            inc = inc + mk(m1.x, m1.y, m1.z) * col;
                            col = col * pt::mix(mk(m0.x, m0.y, m0.z), mk(m2.x, m2.y, m2.z), is_spec);
                            bounce++;
                            if (bounce > p.max_bounce) {
                                rgb = inc;
                                finished = true;
                            }
                        }
                    }
                } else {
                    f3 env = mk(0, 0, 0);
                    if (!(p.flags & PT_FLAG_NO_SKY)) {
                        f3 dir = pt::normalize(d);
                        float tt = 0.5f * (dir.z + 1.0f);
                        float omt = 1.0f - tt;
                        env = mk(omt * 1.0f + tt * 0.5f, omt * 1.0f + tt * 0.7f, omt * 1.0f + tt * 1.0f);
                    }
                    rgb = inc + env * col;
                    finished = true;
                }
                if (finished) bounce = -1;
                if (finished) {
                    bool frame_done = true;
                    f3 px;
                    if (MULTI) {          // raysPerPixel > 1: pixel = 0 + sum of rays, / rpp
                        psum = psum + rgb;
                        r++;
                        frame_done = r >= p.rpp;
                        px = psum / (float)p.rpp;
                    } else {              // raysPerPixel == 1: pixel = (0 + rgb) / 1
                        px = (mk(0, 0, 0) + rgb) / 1.0f;
                    }
                    if (frame_done) {
                        if (SPLIT) {
                            // streamed once, read once by k_accum_frames: non-temporal, so the
                            // colour stream does not evict the scene from L2/MALL
                            nt_store3(p.rgb + 3 * ((size_t)k * (size_t)(p.rows_local * p.W) + (size_t)aidx), px);
                        } else {
                            int f = p.frame_first + k;
                            acc = accumulate(acc, px, f, k > 0 || p.acc_first == 1);
                        }
                        if (MULTI) {
                            psum = mk(0, 0, 0);
                            r = 0;
                        }
                        k++;
                    }
                }
                t = -1.0f;
            }
            if ((st == ST_SHADE) & (bounce < 0) & (lx >= 0) & (k >= (SPLIT ? kend : p.n_frames))) {
                if (!SPLIT) p.accum[aidx] = acc;
                if (p.tile_cost && tile_id != ~0u) atomicAdd(&p.tile_cost[tile_id], pcost);
                lx = -1;
            }
            // wave-aggregated pull from the work queue.  Frame-split items are short, so
            // there a wave reserves ids in batches of pull_batch (one queue atomic per batch
            // instead of per pull; the counter is one address for the whole chip).  (A queue
            // sharded over 8 heads, one per XCD, measured slower on one-frame launches with
            // and without overlap, and cost 5% on C2 in the same kernel.)
            bool want = st == ST_SHADE && lx < 0;
            unsigned long long m = __ballot(want);
            if (m) {
                const unsigned need = (unsigned)__popcll(m);
                const unsigned rank = (unsigned)rank_in(m);
                const int leader = __ffsll((long long)m) - 1;
                unsigned id;
                if (SPLIT && qend - qnext >= need) {
                    id = qnext + rank;
                    qnext += need;
                } else {
                    const unsigned avail = SPLIT ? qend - qnext : 0u;
                    const unsigned take = SPLIT ? max(need - avail, (unsigned)p.pull_batch) : need;
                    unsigned base = 0;
                    if (want && rank == 0u) base = atomicAdd(p.work_counter, take);   // the leader
                    base = (unsigned)__builtin_amdgcn_readlane((int)base, leader);
                    id = rank < avail ? qnext + rank : base + (rank - avail);
                    if (SPLIT) {
                        qnext = base + (need - avail);
                        qend = base + take;
                    }
                }
                if (want) {
                    if (id >= total_ids) {
                        st = ST_DONE;
                    } else {
                        const unsigned item = id >> 6, w = id & 63u;
                        // item -> (tile, frame group): by the host's exact magic reciprocal
                        // (kernel argument) when it is valid for every item
                        unsigned tile = item;
                        if (SPLIT) tile = p.grp_magic ? __umulhi(item, p.grp_magic) : item / n_groups;
                        const int g = SPLIT ? (int)(item - tile * n_groups) : 0;
                        int tx, ty;
                        if (p.tile_perm) {          // packed (ty << 16) | tx: no division
                            const unsigned pk = p.tile_perm[tile];
                            tx = (int)(pk & 0xffffu);
                            ty = (int)(pk >> 16);
                        } else {
                            tx = (int)(tile % (unsigned)tiles_x);
                            ty = (int)(tile / (unsigned)tiles_x);
                        }
                        tile = (unsigned)(ty * tiles_x + tx);
                        int cx = tx * tw + (int)(w & (unsigned)(tw - 1));
                        int crow = ty * th + (int)(w >> (3 + tsh));
                        int cy = p.row0 + crow * p.row_stride;
                        if ((cx < p.W) & (crow < p.rows_local) & (cx < p.x_limit) & (cy < p.y_limit)) {
                            lx = cx;
#ifdef PT_WAVE_TRACE
                            wt_items++;
#endif
                            y = cy;
                            aidx = crow * p.W + cx;
                            // cost sample: 4 pixels per 8x8 tile report (one 64-B memory-side
                            // atomic each), the rest keep tile_id = ~0u
                            tile_id = ((w & 0x1bu) == 0u) ? tile : ~0u;
                            pcost = 0;
                            k = g * p.group;
                            if (SPLIT) kend = min(k + p.group, p.n_frames);
                            r = 0;
                            psum = mk(0, 0, 0);
                            if (!SPLIT) acc = p.acc_first ? p.accum[aidx] : make_float4(0, 0, 0, 0);
                            bounce = -1;
                        }
                    }
                }
            }
            if (st == ST_SHADE && lx >= 0) {
                if (bounce < 0) {    // camera ray due (:514-542)
                    if (r == 0) state = pt::seed(lx, y, p.frame_first + k);
                    float ax = 0.0f, ay = 0.0f;
                    if (!(p.flags & PT_FLAG_NO_AA)) {
                        ax = pt::random01(state);
                        ay = pt::random01(state);
                    }
                    // (x + jitter) / W by the exact reciprocal RN(1/W) and a Markstein
                    // correction: the numerator is 0 or in [2^-32, 2^17), W <= 2^16, so the
                    // remainder is exact and the quotient correctly rounded (test_exact_div)
                    float u = pt::div_mk((float)lx + ax, p.fW, p.rW) - 0.5f;
                    float v = pt::div_mk((float)y + ay, p.fH, p.rH) - 0.5f;
                    d = pt::normalize((cfwd + cright * u) + cup * v);
                    o = cpos;
                    inc = mk(0, 0, 0);
                    col = mk(1, 1, 1);
                    bounce = 0;
                }
                // segment set-up: exact-reciprocal guard, spheres (:372-385), walk start
                // the ray half of the guard, evaluated without short-circuit branches (each
                // && of the old form was an exec-mask branch): every origin component 0 or
                // in [2^-40, 2^60], every direction component in [2^-20, 2] (NaN fails)
                const bool fast_seg =
                       (p.scene_fast != 0) & in_guard(o.x, 0x1p-40f, 0x1p60f) & in_guard(o.y, 0x1p-40f, 0x1p60f) &
                       in_guard(o.z, 0x1p-40f, 0x1p60f) & in_range_abs(d.x, 0x1p-20f, 2.0f) &
                       in_range_abs(d.y, 0x1p-20f, 2.0f) & in_range_abs(d.z, 0x1p-20f, 2.0f);
                // under the guard |d_i| is in [2^-20, 2]: rcp_fast is the exact RN(1/d_i); rd = 0
                // marks a segment outside it
                rd = fast_seg ? mk(pt::rcp_fast(d.x), pt::rcp_fast(d.y), pt::rcp_fast(d.z)) : mk(0, 0, 0);
                if (COUNT && !fast_seg) c.slow++;
                if (COUNT && ray_has_nan(o, d)) c.nan++;
                t = __builtin_huge_valf();
                hprim = -1;
                if (!(p.flags & PT_FLAG_NO_SPHERES)) {
                    for (int si = 0; si < p.sc.n_spheres; si++) {
                        float4 s0 = S.spheres[2 * si];
                        f3 oc = o - mk(s0.x, s0.y, s0.z);
                        float a = pt::dot(d, d);
                        float half_b = pt::dot(oc, d);
                        float cq = pt::dot(oc, oc) - s0.w;
                        float disc = half_b * half_b - a * cq;
                        // the IEEE division sequence, not div_g: its range guard's four compares
                        // cost more than the sequence (same quotient; +0.6% on C2, round 5)
                        float ht = disc < 0.0f ? -1.0f : (-half_b - pt::sqrt_g(disc)) / a;
                        if (COUNT) c.sph++;
                        if (win_open(ht, t)) {
                            t = ht;
                            hprim = -2 - si;
                        }
                    }
                }
                const bool walk = use_tris & (COUNT || !ray_has_nan(o, d));
                // inside the root box (all three axes, inclusive) each axis has near <= 0 <=
                // far, so the exact slab says hit for any t >= 0: skip the root's test
                const bool inside = (root_skip >= 0) & fast_seg & (o.x >= p.root_box[0]) & (o.x <= p.root_box[1]) &
                                    (o.y >= p.root_box[2]) & (o.y <= p.root_box[3]) & (o.z >= p.root_box[4]) &
                                    (o.z <= p.root_box[5]);
                const int img = (LDS && fast_seg) ? oct_base(d, S.np << 5) : 0;   // octant image
                bi = walk ? ((WIDE && fast_seg) ? 0 : (inside ? root_skip : 0) + img) : -1;
                if (WIDE) {   // the wide walk starts at the root record with an empty stack
#pragma unroll
                    for (int k = 0; k < kWideStack; k++) we[k] = 0u;
                    wR = -1;
                }
                st = walk ? ST_TRAV : ST_SHADE;
            }
        } else if (nL > 0 && (nL >= p.leaf_thresh || low)) {
            // ---------------- LEAF: both triangle tests + the 2-way choice (:406-429)
            const bool at = st == ST_LEAF;
            int s0 = 0, cont = -1;
            bool cop = false;
            float4 nd0 = make_float4(0, 0, 0, 0);
            if (at) {
                if (COUNT) { c.tri += 2; diag_tick(c.lw, c.ll); }
                const int code = LDS ? leaf : ~leaf;         // k << 2 | coplanar << 1 | single
                s0 = (code >> 1) & ~1;                       // slots 2k, 2k+1
                cop = (code & 2) != 0;
                if (WIDE && fast) {                          // wide walk: bi = -2 - (g << 1 | cop)
                    const int gc = -2 - bi;
                    s0 = gc & ~1;                            // slots 2g, 2g+1
                    cop = (gc & 1) != 0;
                }
                if (LDS && !COUNT && p.cons_walk) {   // sinks carry the pair k only
                    s0 = 2 * leaf;
                    cop = __float_as_int(tri_quad<LDS>(S, s0 + 1, 1).w) != 0;
                }
                nd0 = tri_quad<LDS>(S, s0, 0);               // {n, d0} of the first triangle
                cont = LDS ? __float_as_int(tri_quad<LDS>(S, s0, 1).w) : bi;   // LDS: next-right, image 0
                if (LDS && (fast & (cont >= 0))) cont += oct_base(d, S.np << 5);
            }
            float h1 = -1.0f, h2 = -1.0f;
            bool ca = false, cb = false;   // the chosen triangle certifies its leaf's box (pt_wide.h)
            if (p.flags & PT_FLAG_MOLLER_TRUMBORE) {   // wave-uniform
                if (at) {
                    h1 = tri_mt(tri_quad<LDS>(S, s0, 1), tri_quad<LDS>(S, s0, 2), tri_quad<LDS>(S, s0, 3), o, d);
                    h2 = tri_mt(tri_quad<LDS>(S, s0 + 1, 1), tri_quad<LDS>(S, s0 + 1, 2),
                                tri_quad<LDS>(S, s0 + 1, 3), o, d);
                }
            } else {
                leaf_pair_tests<LDS, WIDE>(S, at, s0, nd0, cop, o, d, t, p.compact_max, h1, h2, WIDE && p.leaf_cert != 0, ca, cb);
            }
            bool c1 = false, c2 = false;
            if (at) {
                c1 = win_open(h1, t) & ((h1 < h2) | (h2 < 0.0001f));
                c2 = !c1 & win_open(h2, t);
            }
            if (LDS && !COUNT && p.cons_walk) {
                // the culling walk stopped here on the conservative test: the reference tests
                // this leaf's triangles only if its box passes the exact test at this t, and
                // only a triangle that moves t makes the difference (a leaf's hit and miss
                // links are the same next-right).  Its image-0 offset: slot 2k+1 quad 3 .w.
                const bool chk = at & fast & ((c1 & !ca) | (c2 & !cb));
                if (__any(chk)) {
                    if (chk) {
                        float4 lo, hi;
                        node_at<LDS, PADN>(S, __float_as_int(tri_quad<LDS>(S, s0 + 1, 3).w) + oct_base(d, S.np << 5),
                                           lo, hi);
                        if (!slab_oct(lo, hi, o, d, rd, t)) c1 = c2 = false;
                    }
                }
            }
            if (WIDE) {
                // the wide walk reached this leaf on the conservative test: as the culling walk,
                // its own box is tested exactly at this t before a triangle may move t (leaf g's
                // box at wlbox[2g], [2g + 1]) -- unless the chosen triangle certifies that test
                const bool chk = at & fast & ((c1 & !ca) | (c2 & !cb));
                if (__any(chk)) {
                    if (chk) {
                        if (!slab_fast(S.wlbox[s0], S.wlbox[s0 + 1], o, d, rd, t)) c1 = c2 = false;
                    }
                }
            }
            if (at) {
                if (c1 | c2) {
                    t = c1 ? h1 : h2;
                    hprim = s0 + (c1 ? 0 : 1);
                }
                if (WIDE && fast) {   // the next pending child, or the resume position
                    bi = ptw::wide_pop<kWideStack>(we, wR);
                    st = bi >= 0 ? ST_TRAV : (bi == -1 ? ST_SHADE : ST_LEAF);
                } else {
                    bi = cont;
                    st = bi > -1 ? ST_TRAV : ST_SHADE;
                }
            }
        } else {
            // ---------------- TRAV: walk until a leaf is hit / the chain ends; yield to the
            // other phases once enough lanes wait there.  `fast` is fixed for the segment,
            // so a wave whose walking lanes are all inside the guard runs a walk without
            // the per-node IEEE-division branch.
            const unsigned long long live = LDS ? mS | mL | mT : __ballot(st != ST_DONE);
            const bool all_fast = LDS ? (__ballot(fast) & mT) == mT : __all(fast || st != ST_TRAV);
            if (LDS && !COUNT && p.cons_walk) {    // the culling walk (kernel argument: uniform)
                if (all_fast)
                    trav_walk<true, COUNT, LDS, PADN, true>(S, o, d, rd, fast, t, live, mT, mL, mS, p.leaf_thresh, p.shade_thresh, p.trav_floor, st, bi, leaf, c);
                else
                    trav_walk<false, COUNT, LDS, PADN, true>(S, o, d, rd, fast, t, live, mT, mL, mS, p.leaf_thresh, p.shade_thresh, p.trav_floor, st, bi, leaf, c);
            } else if (WIDE) {
                // lanes outside the guard walk the binary tree first (rare), then the wide walk
                if (__ballot((st == ST_TRAV) & !fast))
                    trav_walk<false, COUNT, LDS, PADN>(S, o, d, rd, fast, t, live, mT, mL, mS, p.leaf_thresh, p.shade_thresh, p.trav_floor, st, bi, leaf, c, !fast);
                else
                    trav_wide(S, o, rd, t, live, p.leaf_thresh, p.shade_thresh, p.trav_floor, st, bi, we, wR);
            } else if (all_fast) {
                trav_walk<true, COUNT, LDS, PADN>(S, o, d, rd, fast, t, live, mT, mL, mS, p.leaf_thresh, p.shade_thresh, p.trav_floor, st, bi, leaf, c);
            } else {
                trav_walk<false, COUNT, LDS, PADN>(S, o, d, rd, fast, t, live, mT, mL, mS, p.leaf_thresh, p.shade_thresh, p.trav_floor, st, bi, leaf, c);
            }
        }
#ifdef PT_PHASE_CLOCK
        clk[clk_ph] += clock64() - clk_t0;
        clk[3 + clk_ph] += 1;
#endif
    }
#ifdef PT_PHASE_CLOCK
    if (lane == 0)
        for (int i = 0; i < 6; i++) atomicAdd(&g_phase_clk[i], clk[i]);
    {
        unsigned long long tw = wave_sum(c.tw), tl = wave_sum(c.tl);
        if (lane == 0) { atomicAdd(&g_phase_clk[6], tw); atomicAdd(&g_phase_clk[7], tl); }
    }
#endif
#ifdef PT_WAVE_TRACE
    {
        const unsigned long long wt_end = __builtin_amdgcn_s_memrealtime();
        unsigned items = wt_items;
        for (int off = 32; off > 0; off >>= 1) items += __shfl_xor(items, off, 64);
        const int wid = blockIdx.x * (NT / 64) + (int)(threadIdx.x >> 6);
        if ((threadIdx.x & 63) == 0 && wid < kWaveTraceMax) {
            g_wave_trace[4 * wid] = wt_entry;
            g_wave_trace[4 * wid + 1] = wt_staged;
            g_wave_trace[4 * wid + 2] = wt_end;
            g_wave_trace[4 * wid + 3] = items;
        }
    }
#endif
    flush_counters<COUNT>(p, c);
}

// Adaptive tile order, on the device after every launch that recorded tile
// costs: longest-processing-time-first order of the 8x8 tiles for the next launches -- a
// counting sort of the recorded segment counts into 1024 buckets, most expensive first --
// then the counts are cleared.  Stream-ordered, so the next launch reads the new order with
// no host round trip (the host form cost ~0.2 ms per pt_render: three synchronous copies).
// The order inside a bucket is whatever the LDS atomics give: tile order changes only the
// launch tail, never the image.  One 1024-thread workgroup.
__global__ __launch_bounds__(1024) void k_tile_order(unsigned* __restrict__ cost, unsigned* __restrict__ perm,
                                                     int n_tiles, int tiles_x) {
    constexpr int nb = 1024;
    __shared__ unsigned hist[nb], base[nb], wmax[16];
    const int tid = threadIdx.x;
    unsigned mx = 1u;
    for (int t = tid; t < n_tiles; t += 1024) mx = max(mx, cost[t]);
    for (int o = 32; o > 0; o >>= 1) mx = max(mx, (unsigned)__shfl_xor((int)mx, o));
    if ((tid & 63) == 0) wmax[tid >> 6] = mx;
    hist[tid] = 0u;
    __syncthreads();
    mx = wmax[0];
    for (int w = 1; w < 16; w++) mx = max(mx, wmax[w]);
    auto bucket = [&](unsigned v) { return nb - 1 - (int)((unsigned long long)v * (nb - 1) / mx); };
    for (int t = tid; t < n_tiles; t += 1024) atomicAdd(&hist[bucket(cost[t])], 1u);
    __syncthreads();
    const unsigned own = hist[tid];
    for (int off = 1; off < nb; off <<= 1) {      // inclusive scan of the bucket sizes
        const unsigned add = tid >= off ? hist[tid - off] : 0u;
        __syncthreads();
        hist[tid] += add;
        __syncthreads();
    }
    base[tid] = hist[tid] - own;
    __syncthreads();
    for (int t = tid; t < n_tiles; t += 1024) {
        const unsigned pos = atomicAdd(&base[bucket(cost[t])], 1u);
        perm[pos] = ((unsigned)(t / tiles_x) << 16) | (unsigned)(t % tiles_x);
    }
    __syncthreads();
    for (int t = tid; t < n_tiles; t += 1024) cost[t] = 0u;
}

// ACES film tonemap (screenQuadFrag.c:12-26) of one pixel -> RGBA8, alpha 255.
__device__ __forceinline__ uchar4 aces_px(float4 v) {
    float c[3] = {v.x, v.y, v.z};
    unsigned char o[3];
    for (int k = 0; k < 3; k++) {
        float x = c[k];
        float tm = (x * (2.51f * x + 0.03f)) / (x * (2.43f * x + 0.59f) + 0.14f);
        tm = tm < 0.0f ? 0.0f : (tm > 1.0f ? 1.0f : tm);
        if (!(tm == tm)) tm = 0.0f;
        o[k] = (unsigned char)(int)(tm * 255.0f + 0.5f);
    }
    return make_uchar4(o[0], o[1], o[2], 255);
}
// Running mean of the frame-split mode (:548-551): per local pixel, the launch's frames in
// order from the per-frame colours the render kernel stored -- the same accumulate() the
// lane applies in registers otherwise.  Pixels outside the dispatch footprint are skipped.
// Each thread takes kAccumPix pixels a block-width apart (coalesced), their loads issued
// together: beside a running render this pass gets a few block slots per CU, and with one
// pixel per thread it was latency-bound (about 100 us for a 1080p frame against 15 us alone).
#ifndef PT_ACCUM_PIX
#define PT_ACCUM_PIX 4
#endif
constexpr int kAccumPix = PT_ACCUM_PIX;
// Long launches (more than kShortLaunch frames): 2 pixels per thread and 8 frames per load
// group (same-process A/B, a 1080p/8 share's 1024-frame launch: +1.6% for the whole render
// against one frame per group, +1.1% with 4 x 4; the full 1080p image unchanged).  Short
// launches keep 4 pixels and one frame per group (the pass beside the next one-frame render).
constexpr int kAccumPixLong = 2, kAccumFramesLong = 8;
template <int kAccumPix, int kAccumFrames>
__global__ __launch_bounds__(256) void k_accum_frames(KParams p) {
    resolve_frames(p);
    // the render that used these queue heads has ended (this pass runs after it): ready them
    // for the slot's next render, which waits for this pass (no fill dispatch per launch)
    if (p.reset_work && blockIdx.x == 0 && threadIdx.x == 0) *p.reset_work = 0u;
    // rows_local * W < 2^31 (pt_create), and the grid covers n rounded up to a block's pixels:
    // 32-bit pixel indices
    const unsigned n = (unsigned)p.rows_local * (unsigned)p.W;
    const unsigned base = blockIdx.x * blockDim.x * kAccumPix + threadIdx.x;
    unsigned idx[kAccumPix];
    bool on[kAccumPix];
    float4 acc[kAccumPix];
#pragma unroll
    for (int j = 0; j < kAccumPix; j++) {
        idx[j] = base + (unsigned)j * blockDim.x;
        on[j] = idx[j] < n;
        if (on[j]) {
            const int crow = (int)(idx[j] / (unsigned)p.W), cx = (int)(idx[j] - (unsigned)crow * (unsigned)p.W);
            on[j] = cx < p.x_limit && p.row0 + crow * p.row_stride < p.y_limit;
        }
        acc[j] = (on[j] && p.acc_first) ? p.accum[idx[j]] : make_float4(0, 0, 0, 0);
    }
    // frames in groups of kAccumFrames whose loads are issued together, then applied in frame
    // order: one load group in flight per thread made a long launch's pass latency-bound when
    // few pixels give few threads (a 1080p/8 share's 1024 frames: 0.96 ms for 3.2 GB)
    int k = 0;
    for (; k + kAccumFrames <= p.n_frames; k += kAccumFrames) {
        f3 v[kAccumFrames][kAccumPix];
#pragma unroll
        for (int u = 0; u < kAccumFrames; u++)
#pragma unroll
            for (int j = 0; j < kAccumPix; j++)
                v[u][j] = on[j] ? nt_load3(p.rgb + 3 * ((size_t)(k + u) * (size_t)n + (size_t)idx[j])) : mk(0, 0, 0);
#pragma unroll
        for (int u = 0; u < kAccumFrames; u++)
#pragma unroll
            for (int j = 0; j < kAccumPix; j++)
                acc[j] = accumulate(acc[j], v[u][j], p.frame_first + k + u, k + u > 0 || p.acc_first == 1);
    }
    for (; k < p.n_frames; k++) {
        f3 v[kAccumPix];
#pragma unroll
        for (int j = 0; j < kAccumPix; j++)
            v[j] = on[j] ? nt_load3(p.rgb + 3 * ((size_t)k * (size_t)n + (size_t)idx[j])) : mk(0, 0, 0);
#pragma unroll
        for (int j = 0; j < kAccumPix; j++)
            acc[j] = accumulate(acc[j], v[j], p.frame_first + k, k > 0 || p.acc_first == 1);
    }
#pragma unroll
    for (int j = 0; j < kAccumPix; j++)
        if (on[j]) p.accum[idx[j]] = acc[j];
    // the ACES view of the new image for pt_present_begin (pixels outside the dispatch
    // footprint keep their old value): the same aces_px of the same values as k_aces
    if (p.aces_out) {
#pragma unroll
        for (int j = 0; j < kAccumPix; j++)
            if (idx[j] < n) p.aces_out[idx[j]] = aces_px(on[j] ? acc[j] : p.accum[idx[j]]);
    }
}

// ACES film tonemap epilogue (aces_px) of n pixels.  Each thread
// takes kAcesPix pixels a block-width apart (coalesced), their loads issued together: the pass
// runs beside the next render with few free slots per CU, latency-bound (as k_accum_frames).
#ifndef PT_ACES_PIX
#define PT_ACES_PIX 4
#endif
constexpr int kAcesPix = PT_ACES_PIX;
__global__ __launch_bounds__(256) void k_aces(const float4* __restrict__ src, uchar4* __restrict__ dst,
                                              long long n) {
    const long long base = (long long)blockIdx.x * blockDim.x * kAcesPix + threadIdx.x;
    float4 v[kAcesPix];
#pragma unroll
    for (int j = 0; j < kAcesPix; j++) {
        const long long i = base + (long long)j * blockDim.x;
        v[j] = i < n ? src[i] : make_float4(0, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < kAcesPix; j++) {
        const long long i = base + (long long)j * blockDim.x;
        if (i < n) dst[i] = aces_px(v[j]);
    }
}

}  // namespace

// ===================================================================== host side
// Stage the scene in LDS up to this size.  One workgroup may hold all 160 KiB of a CU's LDS
// on gfx950; a copy too large for the resident waves' worth of 256-thread workgroups is
// shared by wider ones (lds_threads), so mid-size scenes keep the LDS walk at 4+ waves per
// SIMD instead of the global-memory walk.
#ifndef PT_TILE_AUTO
#define PT_TILE_AUTO 0      // 1: 16 x 4 tiles for LDS scenes (measured equal to 8 x 8, ensure_tiles)
#endif
#ifndef PT_LDS_SCENE_MAX_KIB
#define PT_LDS_SCENE_MAX_KIB 152
#endif
#ifndef PT_LDS_WIDE
#define PT_LDS_WIDE 1
#endif
constexpr size_t kLdsSceneMax = (size_t)PT_LDS_SCENE_MAX_KIB * 1024;
constexpr size_t kLdsSceneSmall = 48 * 1024;  // staged by 256-thread workgroups in every configuration
// global-memory scenes: the first kTopNodes device nodes (breadth-first from the root) are
// staged in LDS, 24 KiB per workgroup (6 workgroups per CU stay resident)
constexpr int kTopNodes = 768;
// overlapped short launches: render slots (tuning key 9).  A slot's scratch is reused only
// after the accumulate pass that read it.  Measured on 1080p Cornell one-frame launches (ms per
// frame, round 3): 1 slot (no overlap) 0.80, 2 slots 0.60, 3 slots 0.62, 4 slots 0.66 -- more
// slots put more renders in flight, whose blocks then held the CUs before the accumulate passes
// (and with them the slots) came free.  With the blocks-per-CU cap (key 18) and presentation
// on the context stream (round 4; render only / every frame shown at lag 2): 2 slots at 6
// blocks per CU 0.516 / 0.522-0.547, 3 slots at 6 0.509 / 0.525, 3 at 5 0.505 / 0.527, 3 at 4
// 0.503 / 0.532, 4 at 4-5 0.615 / 0.59.
constexpr int kMaxSlots = 4, kAutoSlots = 3;
// Scratch ring of overlapped launches: each launch takes the next entry (colour scratch, queue
// head, render / accumulate events) of a ring kRingMult times as long as the render streams, so
// a render waits for the accumulate pass of the launch kRingMult * slots back, not of the one
// that last used its stream (which the stream order already puts before it).
#ifndef PT_RING_MULT
#define PT_RING_MULT 2
#endif
constexpr int kRingMult = PT_RING_MULT, kRingMax = kRingMult * kMaxSlots;
constexpr size_t kQueueSet = kQueueStride;   // unsigned per queue head

constexpr int kPresentBufs = 4;   // pt_present_begin buffers

struct pt_ctx {
    pt_config cfg{};
    int rows_local = 0;
    hipStream_t stream = nullptr;
    std::vector<hipEvent_t> ev_free;                               // recycled events
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pending;     // launches not yet synced
    double total_ms = 0.0;
    int n_launches = 0;
    float4* accum = nullptr;
    uchar4* rgba8 = nullptr;
    float4 *d_nodes = nullptr, *d_tris = nullptr, *d_mats = nullptr, *d_spheres = nullptr;
    float4* d_walk_lds = nullptr;   // LDS walk image (DevScene)
    float4* d_walk_sk = nullptr;    // ... the culling walk's copy with its sink image
    size_t lds_bytes_sk = 0;
    // the wide walk of global-memory scenes (pt_wide.h; nested trees inside the scene guard):
    // records, exact leaf boxes, and the node / triangle arrays with leaf slots numbered by the
    // wide tree's index (the binary walk of the lanes outside the guard shares them)
    float4 *d_wrec = nullptr, *d_wlbox = nullptr, *d_nodesw = nullptr, *d_trisw = nullptr;
    bool wide_ok = false;
    int n_wide = 0;                 // wide index space (records + leaves)
    float wide_cw[3] = {0, 0, 0};
    int wide_off = 0;               // tuning key 16: 1 = the binary global walk
    int cert_off = 0;               // tuning key 19: 1 = always run the exact leaf re-test
    bool leaf_cert_ok = false;      // every leaf box contains its triangles' vertices (pt_wide.h certificate)
    int wide_threads = 0;           // tuning key 17: threads per block of the wide walk (0 = automatic)
    int overlap_bpc = 0;            // tuning key 18: render blocks per CU of overlapped short launches (0 = automatic)
    unsigned long long* d_counters = nullptr;
    unsigned int* d_work = nullptr;
    int* d_frame = nullptr;                      // progressive graph frame counter
    // adaptive queue order ("longest first"): per-tile segment counts measured by the
    // previous renders order the next render's 8x8 tiles so cheap tiles form the tail
    unsigned* d_tile_cost = nullptr;
    unsigned* d_tile_perm = nullptr;
    int n_tiles = 0, tiles_x = 1;
    int tile_shift = 0, tile_key = 0;   // tile shape (KParams::tile_shift) and tuning key 20 (0 = automatic)
    bool adaptive = true;
    hipGraph_t graph = nullptr;
    hipGraphExec_t graph_exec = nullptr;
    int graph_frames = 0;
    int n_nodes = 0, n_spheres = 0, n_mats = 0, n_slots = 0, scene_fast = 0, n_top = 0, walk_np = 1;
    float root_box[6] = {0, 0, 0, 0, 0, 0};
    int root_child = -1;
    // the tree is a full binary tree threaded in preorder whose internal boxes contain their
    // children's (pt_bvh_culling_ok): the LDS walk may cull with slab_oct_cons (tuning key 15 = 1: off)
    bool walk_nested = false;
    int cons_off = 0;
    float cons_m[3] = {0, 0, 0};   // KParams::cons_m
    size_t lds_bytes = 0;
    unsigned persist_blocks = 2048;
    int order_skip = 0;             // short launches since the last tile-order sort
    bool order_sorted = false;      // a sort ran since the scene upload
    // 0 = automatic: 52/44 when the scene is staged in LDS (best on C2 since the octant walk),
    // 20/24 when the walk reads global memory (re-swept after the leaf compaction: +2% on
    // the C3 stand-in, +3% on C4 over 16/32; leaf 20 re-swept in round 2: C3 +1.3%, C4 +0.6%
    // over 16); walk floor 5 / 6 (LDS: 8 until the culling walk
    // made a walk step cheaper; re-swept with the sink walk: 5 +0.9% over 3, 2-8 within 1%)
    // (+0.8% on C2, +0.5% on C3 over no floor) -- tools/probe.py sweeps
    int leaf_thresh = 0, shade_thresh = 0, minw = 0, trav_floor = 0, compact_max = 63, pull_batch = 0;
    // frame-split work items (KParams::group): 0 = automatic, n = frames per item
    int group_force = 0;
    int n_cu = 0;
    float* d_rgb = nullptr;        // per-(frame, pixel) colours of the frame-split mode
    size_t rgb_bytes = 0;
    // overlapped short launches (enqueue_render): the render kernels of consecutive short
    // renders rotate over `n_slots` streams with their own colour scratch and queue counter,
    // so frame f+1 renders while frame f's launch drains; k_accum_frames stays on `stream`
    // (created with the highest priority, so its small grid is dispatched as soon as render
    // blocks retire) in frame order
    hipStream_t rstream[kMaxSlots] = {};
    float* slot_rgb[kRingMax] = {};
    size_t slot_rgb_bytes[kRingMax] = {};
    hipEvent_t ev_rdone[kRingMax] = {}, ev_adone[kRingMax] = {};
    // main-stream fence an overlapped render waits for: recorded after every tile-order sort
    // and graph replay (the writers of tile_perm, which the render reads)
    hipEvent_t ev_fence = nullptr;
    bool adone_rec[kRingMax] = {}, fence_rec = false;
    int slot = 0;
    int ring = 0;                   // next scratch-ring entry of an overlapped launch
    int overlap_slots = kAutoSlots;   // tuning key 9 (1 = one stream, no overlap)
    // frame-split scratch budget: a render needing more is issued as back-to-back launches
    // (tuning key 8; default min(32 GiB, a quarter of the device memory))
    size_t scratch_budget = 0;
    // a captured graph bakes in the scratch pointer it was captured with: that buffer stays
    // alive (owned here once ensure_rgb has moved on to a larger one) until drop_graph
    float* graph_rgb = nullptr;
    std::vector<float*> graph_owned;
    bool scene_ok = false, cam_ok = false, counting = false;
    float cam[12] = {0};
    int variant = 0;
    float last_ms = 0.0f;
    unsigned long long last_counts[16] = {0};
    bool count_pending = false;
    // asynchronous presentation (pt_present_begin / _end): per buffer a pinned host image and
    // its copy event; the device view is rgba8 (one, as the copies and the passes that write
    // it are ordered on the context stream)
    unsigned char* present_host[kPresentBufs] = {};
    hipEvent_t ev_copied[kPresentBufs] = {};
    bool present_pending[kPresentBufs] = {};
    // The accumulate pass writes the ACES view into rgba8 beside the running mean when the
    // caller presented after the previous render (aces_fuse, from `presented`); stage_ok: rgba8
    // holds the view of the current image (set by such a pass, cleared by anything that may
    // change the image or rgba8 afterwards).
    bool presented = false, aces_fuse = false, stage_ok = false;
    std::string err;
};

// Queue-order entry of linear tile t (row-major 8x8 tiles): (ty << 16) | tx, so the kernel
// decodes a tile without an integer division.
static unsigned pack_tile(const pt_ctx* c, unsigned t) {
    return ((t / (unsigned)c->tiles_x) << 16) | (t % (unsigned)c->tiles_x);
}


static void drop_graph(pt_ctx* c);   // a captured graph bakes in scene/camera/config
static int ensure_tiles(pt_ctx* c);  // the tile shape this context's next launch uses


static int fail(pt_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}
#define HIPCHK(ctx, call)                                                                   \
    do {                                                                                    \
        hipError_t e_ = (call);                                                             \
        if (e_ != hipSuccess)                                                               \
            return fail(ctx, PT_E_HIP, std::string(#call ": ") + hipGetErrorString(e_));     \
    } while (0)

// Tile shape of the work queue: 64 pixels as (8 << s) columns x (8 >> s) local rows (tuning
// key 20; automatic: ensure_tiles).  Recomputes the tile count and resets the queue order.
static int set_tiles(pt_ctx* c, int s) {
    c->tile_shift = s;
    const int tw = 8 << s, th = 8 >> s;
    c->tiles_x = (c->cfg.width + tw - 1) / tw;
    c->n_tiles = c->tiles_x * ((c->rows_local + th - 1) / th);
    (void)hipFree(c->d_tile_perm);
    (void)hipFree(c->d_tile_cost);
    c->d_tile_perm = c->d_tile_cost = nullptr;
    std::vector<unsigned> ident(std::max(c->n_tiles, 1));
    for (size_t i = 0; i < ident.size(); i++) ident[i] = pack_tile(c, (unsigned)i);
    HIPCHK(c, hipMalloc(&c->d_tile_perm, ident.size() * sizeof(unsigned)));
    HIPCHK(c, hipMalloc(&c->d_tile_cost, ident.size() * sizeof(unsigned)));
    HIPCHK(c, hipMemcpy(c->d_tile_perm, ident.data(), ident.size() * sizeof(unsigned), hipMemcpyHostToDevice));
    HIPCHK(c, hipMemset(c->d_tile_cost, 0, ident.size() * sizeof(unsigned)));
    c->order_sorted = false;
    c->order_skip = 0;
    return PT_OK;
}

static void free_scene(pt_ctx* c) {
    (void)hipFree(c->d_nodes); (void)hipFree(c->d_tris); (void)hipFree(c->d_mats); (void)hipFree(c->d_spheres);
    (void)hipFree(c->d_walk_lds);
    (void)hipFree(c->d_walk_sk);
    (void)hipFree(c->d_wrec); (void)hipFree(c->d_wlbox); (void)hipFree(c->d_nodesw); (void)hipFree(c->d_trisw);
    c->d_nodes = c->d_tris = c->d_mats = c->d_spheres = c->d_walk_lds = c->d_walk_sk = nullptr;
    c->d_wrec = c->d_wlbox = c->d_nodesw = c->d_trisw = nullptr;
    c->wide_ok = false;
    c->n_wide = 0;
    c->scene_ok = false;
}

extern "C" {

int pt_create(const pt_config* cfg, pt_ctx** out) {
    if (!cfg || !out) return PT_E_ARG;
    *out = nullptr;
    pt_ctx* c = new pt_ctx();
    c->cfg = *cfg;
    if (c->cfg.rays_per_pixel <= 0) c->cfg.rays_per_pixel = 1;
    if (c->cfg.world <= 0) c->cfg.world = 1;
    *out = c;
    if (cfg->width <= 0 || cfg->height <= 0 || cfg->width > 65536 || cfg->height > 65536)
        return fail(c, PT_E_ARG, "width/height out of range");
    if (cfg->display_mode < 1 || cfg->display_mode > 4) return fail(c, PT_E_ARG, "display_mode must be 1..4");
    if (cfg->max_bounce < 0) return fail(c, PT_E_ARG, "max_bounce must be >= 0");
    if (cfg->flags & ~PT_FLAG_ALL) return fail(c, PT_E_ARG, "unknown PT_FLAG bits");
    if (c->cfg.rank < 0 || c->cfg.rank >= c->cfg.world) return fail(c, PT_E_ARG, "rank out of range");
    int ndev = 0;
    HIPCHK(c, hipGetDeviceCount(&ndev));
    if (cfg->device < 0 || cfg->device >= ndev) return fail(c, PT_E_HIP, "no such HIP device");
    HIPCHK(c, hipSetDevice(cfg->device));
    int rank = c->cfg.rank, world = c->cfg.world;
    c->rows_local = cfg->height > rank ? (cfg->height - rank + world - 1) / world : 0;
    if ((long long)c->rows_local * cfg->width >= (1LL << 31)) return fail(c, PT_E_ARG, "framebuffer exceeds 2^31 pixels");
    size_t px = (size_t)c->rows_local * cfg->width;
    {
        int lo = 0, hi = 0;   // hi = the greatest priority (numerically least)
        HIPCHK(c, hipDeviceGetStreamPriorityRange(&lo, &hi));
        HIPCHK(c, hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, hi));
    }
    HIPCHK(c, hipEventCreateWithFlags(&c->ev_fence, hipEventDisableTiming));
    HIPCHK(c, hipMalloc(&c->accum, std::max<size_t>(px, 1) * sizeof(float4)));
    HIPCHK(c, hipMemset(c->accum, 0, std::max<size_t>(px, 1) * sizeof(float4)));
    HIPCHK(c, hipMalloc(&c->rgba8, std::max<size_t>(px, 1) * sizeof(uchar4)));
    HIPCHK(c, hipMalloc(&c->d_counters, 16 * sizeof(unsigned long long)));
    // work-queue heads (kQueueStride apart): one for the main stream and
    // one per overlap slot
    HIPCHK(c, hipMalloc(&c->d_work, kQueueSet * sizeof(unsigned) * (1 + kRingMax)));
    int n_cu = 0;
    HIPCHK(c, hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, cfg->device));
    c->persist_blocks = (unsigned)std::max(1, n_cu) * 8u;   // 8 x 256 threads = 32 waves per CU
    c->n_cu = std::max(1, n_cu);
    {
        size_t total_mem = 0;
        HIPCHK(c, hipDeviceTotalMem(&total_mem, cfg->device));
        c->scratch_budget = std::min<size_t>(32ull << 30, total_mem / 4);
    }
    {
        int rc = set_tiles(c, 0);   // 8 x 8 until a scene picks the automatic shape (ensure_tiles)
        if (rc) return rc;
    }
    // default camera (ogl_path_trace.h:53-54)
    const float defcam[12] = {0, -6, 1, 0, 0, 1, 0, 0, 0, 0, 0, 0};
    pt_set_camera(c, defcam);
    return PT_OK;
}

void pt_destroy(pt_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->cfg.device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    drop_graph(c);
    free_scene(c);
    (void)hipFree(c->accum); (void)hipFree(c->rgba8); (void)hipFree(c->d_counters); (void)hipFree(c->d_work);
    (void)hipFree(c->d_frame);
    (void)hipFree(c->d_tile_perm);
    (void)hipFree(c->d_tile_cost);
    (void)hipFree(c->d_rgb);
    for (int i = 0; i < kMaxSlots; i++) {
        if (c->rstream[i]) (void)hipStreamSynchronize(c->rstream[i]);
        if (c->rstream[i]) (void)hipStreamDestroy(c->rstream[i]);
    }
    for (int i = 0; i < kRingMax; i++) {
        (void)hipFree(c->slot_rgb[i]);
        if (c->ev_rdone[i]) (void)hipEventDestroy(c->ev_rdone[i]);
        if (c->ev_adone[i]) (void)hipEventDestroy(c->ev_adone[i]);
    }
    if (c->ev_fence) (void)hipEventDestroy(c->ev_fence);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (int b = 0; b < kPresentBufs; b++) {
        if (c->present_host[b]) (void)hipHostFree(c->present_host[b]);
        if (c->ev_copied[b]) (void)hipEventDestroy(c->ev_copied[b]);
    }
    for (auto& pr : c->ev_pending) { c->ev_free.push_back(pr.first); c->ev_free.push_back(pr.second); }
    for (hipEvent_t e : c->ev_free) (void)hipEventDestroy(e);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

const char* pt_last_error(const pt_ctx* c) { return c ? c->err.c_str() : "null context"; }

int pt_upload_scene(pt_ctx* c, const float* tris, int n_tris, const float* bvh, int n_nodes,
                    const float* mats, int n_mats, const float* spheres, int n_spheres) {
    if (!c) return PT_E_ARG;
    if (n_tris < 0 || n_nodes < 0 || n_mats < 0 || n_spheres < 0) return fail(c, PT_E_ARG, "negative count");
    if ((n_tris && !tris) || (n_nodes && !bvh) || (n_mats && !mats) || (n_spheres && !spheres))
        return fail(c, PT_E_ARG, "null array with nonzero count");
    if (n_nodes > (1 << 24) || n_tris > (1 << 24)) return fail(c, PT_E_SCENE, "scene exceeds 2^24 records");
    if (n_mats == 0 && (n_nodes > 0 || n_spheres > 0)) return fail(c, PT_E_SCENE, "no materials");
    HIPCHK(c, hipSetDevice(c->cfg.device));
    // --- validate the threaded BVH (every walk must terminate; leaves hit == miss)
    std::vector<float4> dn(2 * (size_t)std::max(n_nodes, 1));
    std::vector<int> leaf_slot(n_nodes, -1);
    int n_leaves = 0;
    for (int i = 0; i < n_nodes; i++) {
        const float* nd = bvh + 12 * (size_t)i;
        bool leaf = nd[8] > -1.0f;
        // the shader's int(float) truncates; values outside (-2, n) -- NaN included -- are
        // rejected before any cast (a float-to-int cast out of range is undefined)
        const auto in_open = [](float v, float lo, float hi) { return v > lo && v < hi; };
        if (!in_open(nd[10], -2.0f, (float)n_nodes) || !in_open(nd[11], -2.0f, (float)n_nodes))
            return fail(c, PT_E_SCENE, "BVH link out of range at node " + std::to_string(i));
        int hl = (int)nd[10], ml = (int)nd[11];
        if (leaf) {
            if (!in_open(nd[8], -1.0f, (float)n_tris) || !in_open(nd[9], -1.0f, (float)n_tris))
                return fail(c, PT_E_SCENE, "leaf triangle index out of range at node " + std::to_string(i));
            int t0 = (int)nd[8], t1 = (int)nd[9];
            if (t0 < 0 || t0 >= n_tris || t1 < 0 || t1 >= n_tris)
                return fail(c, PT_E_SCENE, "leaf triangle index out of range at node " + std::to_string(i));
            if (hl != ml) return fail(c, PT_E_SCENE, "leaf with hit link != miss link is unsupported");
            leaf_slot[i] = n_leaves++;
        } else if (hl < 0) {
            return fail(c, PT_E_SCENE, "internal node without a hit link at node " + std::to_string(i));
        }
    }
    // acyclicity of the (hit, miss) link graph reachable from node 0.  The state-machine
    // kernel relies on it: a walk then visits each node at most once, so the reference's
    // steps < numNodes bound (:393) cannot bind and no step counter is kept.
    if (n_nodes > 0) {
        std::vector<unsigned char> color(n_nodes, 0);
        std::vector<std::pair<int, int>> st;
        st.emplace_back(0, 0);
        color[0] = 1;
        while (!st.empty()) {
            auto& top = st.back();
            const float* nd = bvh + 12 * (size_t)top.first;
            if (top.second >= 2) { color[top.first] = 2; st.pop_back(); continue; }
            int nx = (int)nd[10 + top.second];
            top.second++;
            if (nx < 0) continue;
            if (color[nx] == 1) return fail(c, PT_E_SCENE, "BVH links form a cycle");
            if (color[nx] == 0) { color[nx] = 1; st.emplace_back(nx, 0); }
        }
    }
    for (int i = 0; i < n_tris; i++) {
        const float fm = tris[16 * (size_t)i + 12];
        if (!(fm > -1.0f && fm < (float)n_mats)) return fail(c, PT_E_SCENE, "triangle material index out of range");
    }
    for (int i = 0; i < n_spheres; i++) {
        const float fm = spheres[8 * (size_t)i + 4];
        if (!(fm > -1.0f && fm < (float)n_mats)) return fail(c, PT_E_SCENE, "sphere material index out of range");
    }
    // --- device node numbering: the first kTopNodes nodes in breadth-first order of the walk
    // links from the root (the nodes nearly every walk passes: the global-memory walk keeps
    // them in LDS, node_at), the rest in their original order.  Links are renumbered with the
    // nodes, so every walk visits the same node sequence; the root stays node 0.
    std::vector<int> pos(n_nodes, -1);
    {
        int nx = 0;
        std::vector<int> q;
        if (n_nodes > 0) { pos[0] = nx++; q.push_back(0); }
        for (size_t qi = 0; qi < q.size() && nx < kTopNodes; qi++) {
            const float* nd = bvh + 12 * (size_t)q[qi];
            for (int l = 10; l < 12; l++) {
                const int t = (int)nd[l];
                if (t >= 0 && pos[t] < 0 && nx < kTopNodes) { pos[t] = nx++; q.push_back(t); }
            }
        }
        for (int i = 0; i < n_nodes; i++)
            if (pos[i] < 0) pos[i] = nx++;
    }
    std::vector<int> slot_of(n_nodes, -1);   // leaf slot by device node index
    std::vector<int> code_of(n_nodes, 0);    // leaf code by reference node index
    std::vector<unsigned char> cop_of(n_nodes, 0);   // coplanar leaf pair, by reference node index
    // --- transpose to device layouts
    std::vector<float4> dt(8 * (size_t)std::max(n_leaves, 1));
    auto put_tri = [&](float4* q, int ti) {
        const float* t = tris + 16 * (size_t)ti;
        f3 v0 = mk(t[0], t[1], t[2]), v1 = mk(t[4], t[5], t[6]), v2 = mk(t[8], t[9], t[10]);
        f3 n = pt::normalize(pt::cross(v1 - v0, v2 - v0));
        float d0 = -pt::dot(n, v0);
        int m = (int)t[12];
        float mb;
        std::memcpy(&mb, &m, 4);
        q[0] = make_float4(n.x, n.y, n.z, d0);      // the plane test reads this quad alone
        q[1] = make_float4(v0.x, v0.y, v0.z, 0.0f); // .w: the LDS walk's continuation (below)
        q[2] = make_float4(v1.x, v1.y, v1.z, mb);
        q[3] = make_float4(v2.x, v2.y, v2.z, 0.0f);
    };
    for (int i = 0; i < n_nodes; i++) {
        const float* nd = bvh + 12 * (size_t)i;
        int a, b;
        if (leaf_slot[i] >= 0) {
            int s = leaf_slot[i];
            int t0 = (int)nd[8], t1 = (int)nd[9];
            put_tri(&dt[8 * (size_t)s], t0);
            put_tri(&dt[8 * (size_t)s + 4], t1);
            bool cop;
            {   // coplanar pair: both triangles carry the same (n, d0) up to the sign of zero
                // components (the two halves of an OBJ quad, a single-triangle leaf's copy),
                // flagged in the leaf code (bit 1).  hit_triangle's plane distance
                // -(dot(n,o) + d0) / dot(n,d) is then the same for both wherever it can pass
                // the leaf's acceptance tests: a zero factor of either sign only changes the
                // sign of zero intermediate sums, so the two quotients are bitwise equal or
                // both +-0, +-inf or NaN, which fail t > 1e-4 / t >= 1e-4 alike.  NaN (a
                // degenerate triangle) never compares equal: such pairs are not flagged.
                const float4 A = dt[8 * (size_t)s], B = dt[8 * (size_t)s + 4];
                cop = A.x == B.x && A.y == B.y && A.z == B.z && A.w == B.w;
            }
            a = ~((s << 2) | (cop ? 2 : 0) | (t0 == t1 ? 1 : 0));
            code_of[i] = ~a;
            cop_of[i] = cop ? 1 : 0;
            b = (int)nd[11];
            slot_of[pos[i]] = s;
        } else {
            a = pos[(int)nd[10]];
            b = (int)nd[11];
        }
        if (b >= 0) b = pos[b];
        float fa, fb;
        std::memcpy(&fa, &a, 4);
        std::memcpy(&fb, &b, 4);
        // axis-paired: (min, max) of one axis in adjacent registers for packed-f32 slabs
        const size_t j = (size_t)pos[i];
        dn[2 * j] = make_float4(nd[0], nd[4], nd[1], nd[5]);
        dn[2 * j + 1] = make_float4(nd[2], nd[6], fa, fb);
    }
    std::vector<float4> dm(3 * (size_t)std::max(n_mats, 1));
    for (int i = 0; i < n_mats; i++) {
        const float* m = mats + 16 * (size_t)i;
        float s = m[12];
        dm[3 * (size_t)i] = make_float4(m[0], m[1], m[2], m[13]);
        dm[3 * (size_t)i + 1] = make_float4(m[4] * s, m[5] * s, m[6] * s, m[14]);
        dm[3 * (size_t)i + 2] = make_float4(m[8], m[9], m[10], 0.0f);
    }
    std::vector<float4> ds(2 * (size_t)std::max(n_spheres, 1));
    for (int i = 0; i < n_spheres; i++) {
        const float* s = spheres + 8 * (size_t)i;
        int m = (int)s[4];
        float mb;
        std::memcpy(&mb, &m, 4);
        ds[2 * (size_t)i] = make_float4(s[0], s[1], s[2], s[3] * s[3]);
        ds[2 * (size_t)i + 1] = make_float4(mb, 0, 0, 0);
    }
    // LDS walk images of the state-machine kernel (WalkLinks in the kernel source): per ray
    // octant k the node planes (bounds of the axes whose bit is set in k swapped) with links
    // as byte offsets (16 * (2N * k + index)) and a leaf's hit link -2 - code; the leaf's
    // next-right (image-0 offset) goes to its first triangle's quad 1 .w
    const size_t N = (size_t)(n_nodes <= kPadNodes ? kPadNodes : n_nodes);   // nodes per image plane
    std::vector<float4> dwl(16 * N, make_float4(0, 0, 0, 0));
    for (int k = 0; k < 8; k++) {
        const int base = 16 * 2 * (int)N * k;
        for (int i = 0; i < n_nodes; i++) {
            float4 lo = dn[2 * (size_t)i], hi = dn[2 * (size_t)i + 1];
            int a, b;
            std::memcpy(&a, &hi.z, 4);
            std::memcpy(&b, &hi.w, 4);
            const bool leaf = a < 0;
            int ha = leaf ? -2 - ~a : base + 16 * a, hb = b >= 0 ? base + 16 * b : -1;
            std::memcpy(&hi.z, &ha, 4);
            std::memcpy(&hi.w, &hb, 4);
            if (k & 1) std::swap(lo.x, lo.y);
            if (k & 2) std::swap(lo.z, lo.w);
            if (k & 4) std::swap(hi.x, hi.y);
            dwl[2 * N * k + i] = lo;
            dwl[2 * N * k + N + i] = hi;
            if (leaf && k == 0) {
                std::memcpy(&dt[8 * (size_t)slot_of[i] + 1].w, &hb, 4);
                const int self = 16 * i;           // the culling walk's exact leaf re-test
                std::memcpy(&dt[8 * (size_t)slot_of[i] + 7].w, &self, 4);
            }
        }
    }
    // The culling walk's copy of the walk images: the 8 octant images plus a
    // ninth of "sinks" -- node records whose links both point to themselves.  A leaf's hit link
    // leads to its sink (index 1 + k for leaf pair k) and the chain's end (-1) to sink 0, so a
    // lane that stopped keeps stepping in place: the walk step needs no exec mask, and a lane
    // walks while its position lies below the sink image.  A leaf's coplanar flag moves to
    // slot 2k+1 quad 1 .w (the sink index carries only k).
    std::vector<float4> dsk;
    const bool nested = pt_bvh_culling_ok(bvh, n_nodes) == 1;   // pt_scene.cpp
    if (nested) {
        dsk.assign(18 * N, make_float4(0, 0, 0, 0));
        std::copy(dwl.begin(), dwl.end(), dsk.begin());
        const int sink0 = 16 * 2 * (int)N * 8;
        for (int k = 0; k < 8; k++) {
            for (int i = 0; i < n_nodes; i++) {
                float4& hi = dsk[2 * N * k + N + i];
                int a, b;
                std::memcpy(&a, &hi.z, 4);
                std::memcpy(&b, &hi.w, 4);
                if (a <= -2) a = sink0 + 16 * (1 + ((-2 - a) >> 2));
                if (b == -1) b = sink0;
                std::memcpy(&hi.z, &a, 4);
                std::memcpy(&hi.w, &b, 4);
            }
        }
        for (int i = 0; i <= n_leaves; i++) {
            const int self = sink0 + 16 * i;
            float4 hi = make_float4(0, 0, 0, 0);
            std::memcpy(&hi.z, &self, 4);
            std::memcpy(&hi.w, &self, 4);
            dsk[16 * N + N + i] = hi;
        }
        for (int i = 0; i < n_nodes; i++) {
            const float* nd = bvh + 12 * (size_t)i;
            if (!(nd[8] > -1.0f)) continue;
            const int cop = (code_of[i] >> 1) & 1;
            std::memcpy(&dt[8 * (size_t)leaf_slot[i] + 5].w, &cop, 4);
        }
    }
    // The wide tree of the global-memory walk (pt_wide.h): nested trees only
    // (the superset argument), built whatever the scene size -- variant 3 sends any scene to
    // the global walk.  Its index g numbers records and leaves; leaf g's triangles go to slots
    // 2g, 2g + 1 of a second triangle array and its exact box to wlbox[2g], and a second copy
    // of the device nodes carries leaf codes g << 2 | coplanar << 1 | single for the binary
    // walk of the lanes outside the guard.
    ptw::WideTree wt;
    std::vector<float4> dnw, dtw;
    const bool wide = nested && ptw::wide_build(bvh, n_nodes, cop_of.data(), wt) == 0;
    if (wide) {
        dnw = dn;
        dtw.assign(8 * (size_t)wt.n_index, make_float4(0, 0, 0, 0));
        for (int i = 0; i < n_nodes; i++) {
            const float* nd = bvh + 12 * (size_t)i;
            if (!(nd[8] > -1.0f)) continue;
            const int g = wt.g_of[i], t0 = (int)nd[8], t1 = (int)nd[9];
            // a leaf no walk reaches (not in the nested tree from the root, which is all the
            // links of reachable nodes lead to) has no index: nothing to place
            if (g < 0) continue;
            const int a = ~((g << 2) | (cop_of[i] ? 2 : 0) | (t0 == t1 ? 1 : 0));
            std::memcpy(&dnw[2 * (size_t)pos[i] + 1].z, &a, 4);
            put_tri(&dtw[8 * (size_t)g], t0);
            put_tri(&dtw[8 * (size_t)g + 4], t1);

        }
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));   // a render in flight may still read the old scene
    drop_graph(c);
    free_scene(c);
    if (wide) {
        const size_t nr = (size_t)wt.n_index;
        HIPCHK(c, hipMalloc(&c->d_wrec, nr * kWideStride * sizeof(float4)));
        HIPCHK(c, hipMalloc(&c->d_wlbox, nr * 2 * sizeof(float4)));
        HIPCHK(c, hipMalloc(&c->d_nodesw, dnw.size() * sizeof(float4)));
        HIPCHK(c, hipMalloc(&c->d_trisw, dtw.size() * sizeof(float4)));
        if (kWideStride != 4) {   // pack the three used quads of each 64-B host record
            std::vector<float> packed(nr * kWideStride * 4);
            for (size_t i = 0; i < nr; i++)
                std::memcpy(&packed[i * kWideStride * 4], &wt.rec[i * 16], kWideStride * 16);
            wt.rec.swap(packed);
        }
        HIPCHK(c, hipMemcpy(c->d_wrec, wt.rec.data(), nr * kWideStride * sizeof(float4), hipMemcpyHostToDevice));
        HIPCHK(c, hipMemcpy(c->d_wlbox, wt.lbox.data(), nr * 2 * sizeof(float4), hipMemcpyHostToDevice));
        HIPCHK(c, hipMemcpy(c->d_nodesw, dnw.data(), dnw.size() * sizeof(float4), hipMemcpyHostToDevice));
        HIPCHK(c, hipMemcpy(c->d_trisw, dtw.data(), dtw.size() * sizeof(float4), hipMemcpyHostToDevice));
        c->n_wide = wt.n_index;
        std::memcpy(c->wide_cw, wt.cw, sizeof(c->wide_cw));
    }
    if (nested) {
        HIPCHK(c, hipMalloc(&c->d_walk_sk, dsk.size() * sizeof(float4)));
        HIPCHK(c, hipMemcpy(c->d_walk_sk, dsk.data(), dsk.size() * sizeof(float4), hipMemcpyHostToDevice));
    }
    HIPCHK(c, hipMalloc(&c->d_walk_lds, dwl.size() * sizeof(float4)));
    HIPCHK(c, hipMemcpy(c->d_walk_lds, dwl.data(), dwl.size() * sizeof(float4), hipMemcpyHostToDevice));
    HIPCHK(c, hipMalloc(&c->d_nodes, dn.size() * sizeof(float4)));
    HIPCHK(c, hipMalloc(&c->d_tris, dt.size() * sizeof(float4)));
    HIPCHK(c, hipMalloc(&c->d_mats, dm.size() * sizeof(float4)));
    HIPCHK(c, hipMalloc(&c->d_spheres, ds.size() * sizeof(float4)));
    HIPCHK(c, hipMemcpy(c->d_nodes, dn.data(), dn.size() * sizeof(float4), hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->d_tris, dt.data(), dt.size() * sizeof(float4), hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->d_mats, dm.data(), dm.size() * sizeof(float4), hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->d_spheres, ds.data(), ds.size() * sizeof(float4), hipMemcpyHostToDevice));
    c->n_nodes = n_nodes;
    c->n_spheres = n_spheres;
    c->n_mats = n_mats;
    c->n_slots = 2 * n_leaves;
    c->n_top = std::min(n_nodes, kTopNodes);
    // exact-reciprocal slab guard, scene half: every box coordinate is 0
    // or has magnitude in [2^-40, 2^60], and min <= max on every axis (the octant images'
    // near-first order, slab_oct)
    c->scene_fast = 1;
    for (int i = 0; i < n_nodes && c->scene_fast; i++) {
        const float* nd = bvh + 12 * (size_t)i;
        for (int q = 0; q < 7; q++) {
            if (q == 3) continue;
            float a = std::fabs(nd[q]);
            if (!(nd[q] == 0.0f || (a >= 0x1p-40f && a <= 0x1p60f))) { c->scene_fast = 0; break; }
        }
        if (!(nd[0] <= nd[4] && nd[1] <= nd[5] && nd[2] <= nd[6])) c->scene_fast = 0;
    }
    c->walk_nested = nested;
    c->wide_ok = wide;
    // the leaf re-test certificate (ptw::leaf_certificate) needs each leaf box to contain its
    // triangles' vertices -- the reference builder expands leaf boxes over them (bvh.h:29-52);
    // an uploaded tree is checked, not assumed
    c->leaf_cert_ok = true;
    for (int i = 0; i < n_nodes && c->leaf_cert_ok; i++) {
        const float* nd = bvh + 12 * (size_t)i;
        if (!(nd[8] > -1.0f)) continue;
        for (int k = 0; k < 2 && c->leaf_cert_ok; k++) {
            const float* t = tris + 16 * (size_t)(int)nd[8 + k];
            for (int v = 0; v < 3; v++)
                for (int q = 0; q < 3; q++)
                    if (!(nd[q] <= t[4 * v + q] && t[4 * v + q] <= nd[4 + q])) c->leaf_cert_ok = false;
        }
    }
    c->order_sorted = false;      // the next sort pools the new scene's first short launches
    c->order_skip = 0;
    if (n_nodes > 0) {   // every box lies in the root box (nested): M_i bounds each |coordinate|
        for (int q = 0; q < 3; q++) {
            const double m = std::max(std::fabs((double)bvh[q]), std::fabs((double)bvh[4 + q]));
            c->cons_m[q] = (float)std::ldexp(m * (1.0 + 0x1p-20), -19);   // rounded: within 2^-24 relative
        }
    }
    c->walk_np = (int)N;
    c->lds_bytes = (size_t)(16 * N + 4 * c->n_slots + 3 * n_mats + 2 * n_spheres) * sizeof(float4);
    c->lds_bytes_sk = c->lds_bytes + 2 * N * sizeof(float4);
    c->root_child = -1;
    if (n_nodes > 0) {
        const float4 r0 = dn[0], r1 = dn[1];
        const float box[6] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y};
        std::memcpy(c->root_box, box, sizeof(box));
        int a;
        std::memcpy(&a, &r1.z, 4);
        c->root_child = a >= 0 ? a : -1;
    }
    c->scene_ok = true;
    return PT_OK;
}

int pt_set_camera(pt_ctx* c, const float cam[12]) {
    if (!c || !cam) return PT_E_ARG;
    // camera basis (computeShader.c:519-522), evaluated once per dispatch on the host with
    // the same pinned binary32 ops the shader performs per invocation.
    f3 pos = mk(cam[0], cam[1], cam[2]);
    f3 fwd = pt::normalize(mk(cam[4], cam[5], cam[6]));
    f3 right = pt::normalize(pt::cross(fwd, mk(0, 0, 1)));
    f3 up = (pt::normalize(pt::cross(right, fwd)) * (float)c->cfg.height) / (float)c->cfg.width;
    float v[12] = {pos.x, pos.y, pos.z, fwd.x, fwd.y, fwd.z, right.x, right.y, right.z, up.x, up.y, up.z};
    std::memcpy(c->cam, v, sizeof(v));
    c->cam_ok = true;
    drop_graph(c);
    return PT_OK;
}

int pt_set_display_mode(pt_ctx* c, int mode) {
    if (!c) return PT_E_ARG;
    if (mode < 1 || mode > 4) return fail(c, PT_E_ARG, "display_mode must be 1..4");
    if (mode != c->cfg.display_mode) drop_graph(c);   // a captured graph bakes in the mode
    c->cfg.display_mode = mode;
    return PT_OK;
}

int pt_set_counting(pt_ctx* c, int enable) {
    if (!c) return PT_E_ARG;
    // graph replays never count (pt_progressive_setup refuses counting): a graph captured
    // before counting was switched on would silently produce no counts, so it is dropped
    if ((enable != 0) != c->counting) drop_graph(c);
    c->counting = enable != 0;
    return PT_OK;
}

int pt_set_kernel(pt_ctx* c, int variant) {
    if (!c) return PT_E_ARG;
    if (variant != 0 && variant != 3)
        return fail(c, PT_E_ARG, "unknown kernel variant (0 state machine, 3 state machine with the scene kept in "
                                 "global memory)");
    c->variant = variant;
    drop_graph(c);
    return PT_OK;
}

int pt_set_tuning(pt_ctx* c, int key, int value) {
    if (!c) return PT_E_ARG;
    if (key == 8) {
        if (value < 0) return fail(c, PT_E_ARG, "scratch budget (MiB) must be >= 0 (0 = automatic)");
        if (value == 0) {
            size_t total_mem = 0;
            HIPCHK(c, hipDeviceTotalMem(&total_mem, c->cfg.device));
            c->scratch_budget = std::min<size_t>(32ull << 30, total_mem / 4);
        } else {
            c->scratch_budget = (size_t)value << 20;
        }
        drop_graph(c);
        return PT_OK;
    }
    if (key == 9) {
        if (value < 0 || value > kMaxSlots)
            return fail(c, PT_E_ARG, "overlap slots must be 1..4 (1 = off, 0 = automatic)");
        HIPCHK(c, hipSetDevice(c->cfg.device));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        c->overlap_slots = value ? value : kAutoSlots;
        c->slot = 0;
        c->ring = 0;
        return PT_OK;
    }
    if (key == 15) {
        if (value != 0 && value != 1) return fail(c, PT_E_ARG, "culling walk: 0 = automatic, 1 = off");
        c->cons_off = value;
        drop_graph(c);
        return PT_OK;
    }
    if (key == 18) {
        if (value < 0 || value > 8) return fail(c, PT_E_ARG, "overlapped render blocks per CU must be 1..8 (0 = automatic)");
        c->overlap_bpc = value;
        return PT_OK;
    }
    if (key == 17) {
        if (value != 0 && value != 256 && value != 512 && value != 768 && value != 1024)
            return fail(c, PT_E_ARG, "wide walk workgroup: 256, 512, 768 or 1024 threads (0 = automatic)");
        c->wide_threads = value;
        drop_graph(c);
        return PT_OK;
    }
    if (key == 20) {
        if (value < 0 || value > 4) return fail(c, PT_E_ARG, "tile shape: 1..4 = 8x8, 16x4, 32x2, 64x1 (0 = automatic)");
        c->tile_key = value;
        HIPCHK(c, hipSetDevice(c->cfg.device));
        return ensure_tiles(c);
    }
    if (key == 19) {
        if (value != 0 && value != 1) return fail(c, PT_E_ARG, "leaf re-test certificate: 0 = automatic, 1 = off");
        c->cert_off = value;
        drop_graph(c);
        return PT_OK;
    }
    if (key == 16) {
        if (value != 0 && value != 1) return fail(c, PT_E_ARG, "wide global walk: 0 = automatic, 1 = off");
        c->wide_off = value;
        drop_graph(c);
        return PT_OK;
    }
    if (key == 5) {
        if (value < 0) return fail(c, PT_E_ARG, "frames per work item must be >= 1 (0 = automatic)");
        c->group_force = value;
        drop_graph(c);
        return PT_OK;
    }
    if (key == 4) {
        if (value < 0 || value > 1024) return fail(c, PT_E_ARG, "pull batch must be 1..1024 (0 = auto)");
        c->pull_batch = value;
        drop_graph(c);
        return PT_OK;
    }
    if (key == 7) {
        if (value < 0 || value > 63) return fail(c, PT_E_ARG, "compaction limit must be in 0..63");
        c->compact_max = value;
        drop_graph(c);
        return PT_OK;
    }
    if (value < 0 || value > 64) return fail(c, PT_E_ARG, "threshold must be in 1..64 (0 = automatic)");
    if (key == 0) c->leaf_thresh = value;
    else if (key == 1) c->shade_thresh = value;
    else if (key == 6) c->trav_floor = value;
    else if (key == 3) {
        if (value != 0 && (value < 5 || value > 8)) return fail(c, PT_E_ARG, "waves per SIMD must be 5..8 (0 = auto)");
        c->minw = value;
    }
    else if (key == 2) {
        // a learned order stays when the setting does not change (re-applying the default must
        // not send the next long render back through the cold probe launch)
        if ((value != 0) == c->adaptive) return PT_OK;
        c->adaptive = value != 0;
        c->order_sorted = false;
        c->order_skip = 0;
        if (!c->adaptive && c->n_tiles > 0) {       // back to raster order
            std::vector<unsigned> ident(c->n_tiles);
            for (int i = 0; i < c->n_tiles; i++) ident[i] = pack_tile(c, (unsigned)i);
            HIPCHK(c, hipSetDevice(c->cfg.device));
            HIPCHK(c, hipStreamSynchronize(c->stream));
            HIPCHK(c, hipMemcpy(c->d_tile_perm, ident.data(), ident.size() * sizeof(unsigned), hipMemcpyHostToDevice));
        }
    }
    else return fail(c, PT_E_ARG, "unknown tuning key");
    drop_graph(c);
    return PT_OK;
}

// Frames per work item of the state-machine kernel (KParams::group).  Items of a few frames
// keep every resident lane busy to the end of a launch and let the per-GPU share of a
// multi-GPU split (fewer pixels than lanes at 1080p/8) use the whole chip; the per-frame
// colours go to a buffer and k_accum_frames applies the running mean in frame order.
// Measured (C2 scene, 64-frame launches): 8 frames per item +6% over whole-pixel items on
// one GPU, 2-4 frames +85% on a 1080p/8 share; so ~16 items per resident lane, capped at
// 16 frames (4 for global-memory scenes).  group == n_frames is the register mode (a lane owns all frames of a pixel and
// accumulates in registers).  The counting build follows the same plan: with whole-pixel
// items a 1080p/8 share of a 1024-frame launch would run each lane through 1024 frames
// in sequence (minutes).
// Whether the state-machine kernel stages the scene in LDS:
// up to kLdsSceneSmall always; up to kLdsSceneMax when wide workgroups share the copy
// (lds_threads' configuration).  Variant 3 forces the global-memory walk.
static bool lds_staged(const pt_ctx* c) {
    if (c->variant == 3) return false;
    if (c->lds_bytes <= kLdsSceneSmall) return true;
    return PT_LDS_WIDE && !c->counting && !c->minw && c->cfg.rays_per_pixel == 1 && c->lds_bytes <= kLdsSceneMax;
}

// Round 6: the frames per item follow the frames each resident lane renders in the launch,
// F = pixels * frames / resident lanes.  An item costs a fixed pull and set-up o plus g frames
// of c each, and a launch ends in a tail of about half an item, so the time per lane is about
// F c + (F / g) o + g c / 2: least at g = sqrt(2 F o / c).  Fitted to same-process A/Bs of C2's
// 1024-frame launch (profiles/ab/r06f_*): a 1080p/8 share (F = 578) is fastest at 9-12 frames
// per item (+1.4% over 16), a 1080p/4 share (F = 1157) at 12, the whole image (F = 4628) at
// 16 or more; global-memory scenes cost about 5x more per frame (c), so about sqrt(5) fewer.
// The caps: C2 16 +0.5% over 8; C3 stand-in 4 +8% over 8.
// The work queue's tile shape (set_tiles): tuning key 20, else 8 x 8 (with PT_TILE_AUTO, 16 x 4
// for scenes staged in LDS).  Measured with the builds in alternating order (ABBA, profiles/ab/
// r06n_*): 16 x 4 and 8 x 8 equal within 0.1% on C2 and C5; the +0.4..0.6% of the first A/Bs
// (r06k_*, r06l_*, r06m_*) was tools/ab_inproc.py's first-position bias.  A shape change drains
// the context's streams and drops a captured graph (which holds the tile arrays).
static int ensure_tiles(pt_ctx* c) {
    const int want = c->tile_key ? c->tile_key - 1 : ((PT_TILE_AUTO && c->scene_ok && lds_staged(c)) ? 1 : 0);
    if (want == c->tile_shift) return PT_OK;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (int i = 0; i < kMaxSlots; i++)
        if (c->rstream[i]) HIPCHK(c, hipStreamSynchronize(c->rstream[i]));
    drop_graph(c);
    return set_tiles(c, want);
}

static int plan_group(const pt_ctx* c, int n_frames) {
    if (c->group_force > 0) return std::min(c->group_force, n_frames);
    const int waves = c->minw ? c->minw : (lds_staged(c) ? 7 : 6);
    const double lanes = (double)c->n_cu * 4.0 * waves * 64.0;
    const double px = (double)c->rows_local * c->cfg.width;
    const bool lds_scene = lds_staged(c);
    const double F = px * n_frames / lanes;
    int g = (int)(std::sqrt(F) * (lds_scene ? 0.416 : 0.19) + 0.5);
    g = std::max(1, std::min(g, lds_scene ? 16 : 4));
    return std::min(g, n_frames);
}

// Whether a launch of n_frames with frames-per-item `group` runs in frame-split mode
// (colour planes + k_accum_frames).  Register mode (group == n_frames: a lane owns whole
// pixels, the running mean in registers) pulls one queue id per lane without batching, which
// is right for long items.  But a launch of a few frames has items of a few segments, and
// the chip-wide queue counter then throttles the kernel: one 1080p frame per launch (the
// reference's one dispatch per displayed frame) took 3.2 ms of kernel time, against 0.5 ms
// per frame in long launches.  In automatic mode such launches use the split path and its
// batched reservations; pt_set_tuning key 5 >= n_frames still forces register mode.
constexpr int kShortLaunch = 16;
#ifndef PT_ORDER_EVERY
#define PT_ORDER_EVERY 64
#endif
constexpr int kOrderEvery = PT_ORDER_EVERY;   // short launches per tile-order sort (enqueue_render)
constexpr int kOrderFirst = 8;                // ... and before the first sort after an upload
constexpr int kProbeFrames = 2, kProbeMin = 64;  // cold long renders: a sorted order after 2 frames
static bool split_mode(const pt_ctx* c, int n_frames, int group) {
    if (group < n_frames) return true;
    return c->group_force == 0 && n_frames <= kShortLaunch;
}

// Grows the frame-split scratch to n_frames frame planes.  Earlier launches on the stream may
// still read the old buffer, so the stream is drained first; a buffer a captured graph was
// built with is handed to the graph (freed by drop_graph) instead of being freed under it.
static int ensure_rgb(pt_ctx* c, int n_frames) {
    size_t need = (size_t)std::max(c->rows_local, 1) * (size_t)c->cfg.width * (size_t)n_frames * 3 * sizeof(float);
    if (need <= c->rgb_bytes) return PT_OK;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (c->d_rgb && c->graph_exec && c->d_rgb == c->graph_rgb) c->graph_owned.push_back(c->d_rgb);
    else (void)hipFree(c->d_rgb);
    c->d_rgb = nullptr;
    c->rgb_bytes = 0;
    HIPCHK(c, hipMalloc(&c->d_rgb, need));
    c->rgb_bytes = need;
    return PT_OK;
}

// Render stream `sl` and scratch-ring entry `e` of an overlapped launch (enqueue_render),
// created on first use.  The entry's buffer may still be read by the accumulate pass of the
// last launch that used it, on any render stream, so a reallocation first drains the main
// stream (every accumulate pass) and the render streams.
static int ensure_slot(pt_ctx* c, int sl, int e, int n_frames) {
    if (!c->rstream[sl]) HIPCHK(c, hipStreamCreateWithFlags(&c->rstream[sl], hipStreamNonBlocking));
    if (!c->ev_rdone[e]) {
        HIPCHK(c, hipEventCreateWithFlags(&c->ev_rdone[e], hipEventDisableTiming));
        HIPCHK(c, hipEventCreateWithFlags(&c->ev_adone[e], hipEventDisableTiming));
        // the entry's queue heads start at zero; afterwards each accumulate pass re-zeroes them
        HIPCHK(c, hipMemset(c->d_work + kQueueSet * (1 + e), 0, kQueueSet * sizeof(unsigned)));
    }
    const size_t need = (size_t)std::max(c->rows_local, 1) * (size_t)c->cfg.width * (size_t)n_frames * 3 * sizeof(float);
    if (need <= c->slot_rgb_bytes[e]) return PT_OK;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (int i = 0; i < kMaxSlots; i++)
        if (c->rstream[i]) HIPCHK(c, hipStreamSynchronize(c->rstream[i]));
    (void)hipFree(c->slot_rgb[e]);
    c->slot_rgb[e] = nullptr;
    c->slot_rgb_bytes[e] = 0;
    HIPCHK(c, hipMalloc(&c->slot_rgb[e], need));
    c->slot_rgb_bytes[e] = need;
    return PT_OK;
}

// Queue ids are 32-bit: a launch's items * 64 plus what the resident waves can reserve past
// the end stay below 2^32.  A wave reserves max(pull_batch, 64) ids per queue atomic and, once
// the queue has run dry, at most two more reservations (the one that crossed the end and one
// more; its lanes then finish), so the overshoot is at most (resident waves) * 2 *
// max(pull_batch, 64), with at most persist_blocks * 4 resident waves (256-thread blocks) and
// pull_batch at most 1024 (tuning key 4) or 256 (automatic).
static unsigned long long id_limit(const pt_ctx* c) {
    const unsigned long long pb = (unsigned long long)std::max(256, c->pull_batch);
    const unsigned long long slack = (unsigned long long)c->persist_blocks * 4ull * 2ull * pb;
    return (1ull << 32) - slack - (1ull << 20);
}

// Frames of one launch for a render of n_frames: the largest count whose frame-split scratch
// (12 B per pixel-frame) fits the context's budget and whose queue ids stay 32-bit.  A longer
// render is issued as back-to-back launches of at most this many frames; only the first one
// uses the caller's accumulate flag, so the result is that of n_frames dispatches (pt_api.h).
static int launch_frames(const pt_ctx* c, int n_frames) {
    const unsigned long long px = (unsigned long long)std::max(c->rows_local, 1) * (unsigned long long)c->cfg.width;
    const unsigned long long tiles64 = (unsigned long long)std::max(c->n_tiles, 1) * 64ull;
    int n = n_frames;
    for (;;) {
        const int g = plan_group(c, n);
        if (!split_mode(c, n, g)) return n;    // register mode: no scratch, one group
        // one frame per launch always runs, even when its scratch exceeds the budget (so n
        // strictly decreases to at most 1: the loop ends)
        const unsigned long long by_budget = std::max(1ull, c->scratch_budget / (px * 12ull));
        const unsigned long long ng = (unsigned long long)((n + g - 1) / g);
        const unsigned long long lim = id_limit(c);
        const unsigned long long by_ids = (lim / tiles64) * (unsigned long long)g;
        if (((unsigned long long)n <= by_budget && ng * tiles64 < lim) || n == 1) return n;
        const unsigned long long m = std::min<unsigned long long>({(unsigned long long)n - 1, by_budget, by_ids});
        n = (int)std::max<unsigned long long>(m, 1ull);
    }
}

// Whether the state-machine kernel's LDS walk culls: the tree qualifies
// (walk_nested), key 15 leaves it on, nothing is counted, and the sink image (32 B per node
// beside the 16 N octant records) costs no resident block -- a scene whose copy just fits
// mw blocks per CU in 160 KiB would otherwise lose a block per CU, far more than the walk
// gains (+7%).
static bool cons_walk_on(const pt_ctx* c) {
    if (!c->walk_nested || c->cons_off || c->counting) return false;
    const size_t mw = (size_t)(c->minw ? c->minw : 7);
    const auto blocks = [mw](size_t b) { return b ? std::min(mw, (size_t)(160 * 1024) / b) : mw; };
    return blocks(c->lds_bytes_sk) >= blocks(c->lds_bytes);
}

// Whether a global-memory launch walks the wide tree: the scene has one
// (a nested tree), it lies inside the scene half of the exact-reciprocal guard (otherwise no
// lane could use it), tuning key 16 leaves it on, nothing is counted, and the occupancy is
// one the wide instantiations cover (5-7 waves per SIMD; automatic 6).
constexpr int kWideTopMax = 1 << 14;   // wide records staged in LDS: what the block's LDS share holds
#ifndef PT_WIDE_THREADS
#define PT_WIDE_THREADS 256
#endif
constexpr int kWideThreadsAuto = PT_WIDE_THREADS;   // threads per block of the wide walk (tuning key 17)
static bool wide_walk_on(const pt_ctx* c) {
    return c->wide_ok && c->scene_fast && !c->wide_off && !c->counting && c->minw != 8;
}

// Threads per workgroup of the state-machine kernel on an LDS-staged scene of `lds` bytes:
// the k = 1..4 waves per SIMD per workgroup that make the most resident waves, min(floor(160
// KiB / lds), floor(7 / k)) * k (7 waves per SIMD is the kernel's register budget), the
// narrowest on a tie: 256 threads down to a 23 KiB copy, then 512 / 768 / 1024 (6, 6, 4 waves
// per SIMD at 32 / 54 / 160 KiB).  The wide instantiations are the default configuration's (non-counting, one ray
// per pixel, automatic occupancy); other launches keep 256 threads.
static int lds_threads(const pt_ctx* c, size_t lds) {
    if (!PT_LDS_WIDE || c->counting || c->minw || c->cfg.rays_per_pixel > 1 || !lds) return 256;
    const int per_cu = (int)((size_t)(160 * 1024) / lds);     // copies resident per CU
    int best_k = 1, best = 0;
    for (int k = 1; k <= 4; k++) {      // k waves per SIMD per workgroup, at most 7 per SIMD
        const int waves = std::min(per_cu, 7 / k) * k;
        if (waves > best) { best = waves; best_k = k; }
    }
    return 256 * best_k;
}

// Enqueues one render launch (work-queue reset + kernel) on the context stream.  With
// `frame_dev` the frame range is read on the device (progressive graph replay).
static int enqueue_render(pt_ctx* c, int frame_first, int n_frames, int acc_first, const int* frame_dev,
                          int frame_offset, bool force_sort = false) {
    c->stage_ok = false;    // this launch changes the image: rgba8 holds its view only if written below
    KParams p;
    std::memset(&p, 0, sizeof(p));
    p.sc.nodes = c->d_nodes;
    p.sc.walk_lds = c->d_walk_lds;
    p.sc.tris = c->d_tris;
    p.sc.mats = c->d_mats;
    p.sc.spheres = c->d_spheres;
    p.sc.n_nodes = c->n_nodes;
    p.sc.n_spheres = c->n_spheres;
    p.accum = c->accum;
    std::memcpy(p.cam, c->cam, sizeof(p.cam));
    p.W = c->cfg.width;
    p.H = c->cfg.height;
    p.row0 = c->cfg.rank;
    p.row_stride = c->cfg.world;
    p.rows_local = c->rows_local;
    p.x_limit = (c->cfg.flags & PT_FLAG_REF_DISPATCH) ? (p.W / 10) * 10 : p.W;
    p.y_limit = (c->cfg.flags & PT_FLAG_REF_DISPATCH) ? (p.H / 10) * 10 : p.H;
    p.frame_first = frame_first;
    p.n_frames = n_frames;
    p.acc_first = acc_first;
    p.frame_dev = frame_dev;
    p.frame_offset = frame_offset;
    p.max_bounce = c->cfg.max_bounce;
    p.mode = c->cfg.display_mode;
    p.flags = c->cfg.flags;
    p.rpp = c->cfg.rays_per_pixel;
    p.counters = c->d_counters;
    p.work_counter = c->d_work;
    p.n_slots = c->n_slots;
    p.n_top = c->n_top;
    p.walk_np = c->walk_np;
    p.n_mats = c->n_mats;
    p.scene_fast = c->scene_fast;
    p.cons_walk = cons_walk_on(c);
    // the certificate stands on hit_triangle's plane distance: not in Moller-Trumbore mode.
    // The wide walk only: on the LDS culling walk (C2, VALU-bound, the box re-read from LDS)
    // its ~40 VALU per leaf phase cost more than the re-test (-1.9%, same-process A/B r05c)
    p.leaf_cert = c->leaf_cert_ok && !c->cert_off && !(c->cfg.flags & PT_FLAG_MOLLER_TRUMBORE);
    p.sc.walk_sk = c->d_walk_sk;
    std::memcpy(p.cons_m, c->cons_m, sizeof(p.cons_m));
    std::memcpy(p.root_box, c->root_box, sizeof(p.root_box));
    p.root_child = c->root_child;
    {
        bool lds_scene = lds_staged(c);
        p.leaf_thresh = c->leaf_thresh ? c->leaf_thresh : (lds_scene ? 52 : 20);
        p.shade_thresh = c->shade_thresh ? c->shade_thresh : (lds_scene ? 44 : 24);
        // walk floor: 5 for the small LDS scenes (C2), 8 for the wide-workgroup ones (keysweep
        // on the 150 / 380-triangle stand-ins: +0.8% / +1.2% over 5), 6 for global memory
        p.trav_floor = c->trav_floor ? c->trav_floor : (lds_scene ? (c->lds_bytes > kLdsSceneSmall ? 8 : 5) : 6);
        p.compact_max = c->compact_max;
    }
    p.rW = 1.0f / (float)p.W;
    p.fW = (float)p.W;
    p.fH = (float)p.H;
    p.rH = 1.0f / (float)p.H;
    p.group = plan_group(c, n_frames);
    // queue ids reserved per queue atomic: on an LDS-staged scene an item of one or two
    // frames is a few short segments, and the chip-wide counter then limits the launch (one
    // 1080p Cornell frame per launch: 1.14 ms kernel time with 32 ids per reservation, 0.97
    // with 128; 4K 3.44 -> 2.64 ms; 4-frame launches 0.83 -> 0.62 ms per frame).  A wave
    // that reserves more ids than it soon needs lengthens the launch tail instead, so longer
    // items and the global-memory scenes' long segments keep 32 (C3 stand-in, one frame per
    // launch: 3.19 ms with 32, 3.63 with 128).  With overlapped one-frame launches (2 slots)
    // 256 ids beat 128 (0.594 vs 0.603 ms per 1080p frame; 64: 0.689).  Tuning key 4 overrides.
    //
    // Otherwise (round 3 sweep, same process) the best reservation follows the queue ids a
    // resident wave takes over the launch, I, and the frames per item, g: about I / (8 g),
    // between 32 and 256.  Global-memory scenes (C3 stand-in): one-frame launches best at 48
    // (+4% over 32), 4-frame 128 (+3.8%), 8-frame 64 (+1.9%), 16-frame 32, 32-frame 64 (+1%),
    // 64-frame 128 (+1.3%), 256-frame 192-256 (+2.2%; C4 +2.1%); C2's 1024-frame launch 128
    // (+0.9%).  Fewer ids per wave than that make the queue atomic's round trip frequent;
    // more leave the last waves holding a long reservation in the launch tail.
    {
        const bool lds_items = lds_staged(c);
        const double waves = (double)c->n_cu * 4.0 * (lds_items ? 7.0 : 6.0);
        const double ids = (double)c->n_tiles * (double)((n_frames + p.group - 1) / p.group) * 64.0;
        const int fit = 16 * (int)(ids / std::max(waves, 1.0) / (8.0 * p.group) / 16.0 + 0.5);
        const int auto_batch = std::max((int)kPullBatch, std::min(256, fit));
        p.pull_batch = c->pull_batch ? c->pull_batch
                                     : (lds_items && p.group <= 2 ? (p.group == 1 ? 256 : 64) : auto_batch);
    }
    {   // exact item / n_groups by ceil(2^32 / n_groups) when item * n_groups < 2^32 for every
        // item (then floor(item * m / 2^32) = floor(item / n_groups)), else the division
        const unsigned long long ng = (unsigned long long)((n_frames + p.group - 1) / p.group);
        const unsigned long long items = (unsigned long long)c->n_tiles * ng;
        p.grp_magic = (ng > 1 && items * ng < (1ull << 32)) ? (unsigned)(((1ull << 32) + ng - 1) / ng) : 0u;
    }
    // Overlapped short launches: a short frame-split render (the reference's one dispatch per
    // displayed frame, ogl_path_trace.h:160-204) ends in a tail of nearly empty waves.  Its
    // render kernel runs on overlap slot `sl` (own stream, colour scratch and queue counter)
    // so the next render's waves fill the CUs that this one's tail frees; the accumulate pass
    // stays on the main stream, in frame order (the running mean, :548-551).  Dependencies:
    // the slot's scratch is reused only after the accumulate pass that read it (ev_adone), and
    // a render never overlaps a tile-order sort (ev_sort; the sort runs on the main stream,
    // which has waited for every earlier render).  Not for captured graphs or counting.
    const bool overlap = c->overlap_slots > 1 && !frame_dev && !c->counting && n_frames <= kShortLaunch &&
                         split_mode(c, n_frames, p.group);
    const int sl = c->slot;
    const int ring = kRingMult * c->overlap_slots;
    const int re = c->ring % ring;       // this launch's scratch-ring entry
    hipStream_t rs = c->stream;
    unsigned* work = c->d_work;
    if (overlap) {
        int rc = ensure_slot(c, sl, re, n_frames);
        if (rc) return rc;
        rs = c->rstream[sl];
        work = c->d_work + kQueueSet * (1 + re);
        p.rgb = c->slot_rgb[re];
        p.work_counter = work;
        c->slot = (sl + 1) % c->overlap_slots;
        c->ring = (re + 1) % ring;
    } else if (split_mode(c, n_frames, p.group)) {
        int rc = ensure_rgb(c, n_frames);
        if (rc) return rc;
        p.rgb = c->d_rgb;
    }
    p.tile_perm = c->d_tile_perm;
    p.tile_shift = c->tile_shift;
    p.tile_cost = (c->adaptive && !c->counting) ? c->d_tile_cost : nullptr;
    if (c->rows_local == 0) return PT_OK;
    // variants: 0 state machine (default), 3 = 0 with the scene forced to stay in global memory
    const int variant = c->variant;
    const bool use_lds = variant == 0 && lds_staged(c);
    // the global-memory walk of a nested tree takes the wide tree (pt_wide.h) unless tuning
    // key 16 turns it off; counting builds keep the binary walk (their counts are the
    // reference's), and so do occupancy overrides other than 6 waves per SIMD
    const bool use_wide = !use_lds && wide_walk_on(c);
    p.leaf_cert = p.leaf_cert && use_wide;
    if (use_wide) {
        p.sc.nodes = c->d_nodesw;
        p.sc.tris = c->d_trisw;
        p.sc.wrec = c->d_wrec;
        p.sc.wlbox = c->d_wlbox;
        std::memcpy(p.wide_cw, c->wide_cw, sizeof(p.wide_cw));
    }
    if (overlap) {
        if (c->adone_rec[re]) HIPCHK(c, hipStreamWaitEvent(rs, c->ev_adone[re], 0));
        if (c->fence_rec) HIPCHK(c, hipStreamWaitEvent(rs, c->ev_fence, 0));
    }
    // an overlap slot's heads were zeroed by the accumulate pass of its last render (or at
    // the slot's creation)
    if (overlap) p.reset_work = work;
    else HIPCHK(c, hipMemsetAsync(work, 0, kQueueSet * sizeof(unsigned), rs));
    {
        // persistent grid: enough resident waves to fill every SIMD; surplus blocks find the
        // queue empty and exit.  Never more blocks than 8x8 tiles (64 lanes per tile).
        size_t lds = use_lds ? (p.cons_walk ? c->lds_bytes_sk : c->lds_bytes) : 0;
        unsigned tiles = (unsigned)c->n_tiles;
        unsigned items = tiles * (unsigned)((n_frames + p.group - 1) / p.group);   // 64-lane items
        // the wide walk's workgroup: wider ones share one LDS copy of more top records
        // (tuning key 17); raysPerPixel > 1 keeps 256 threads
        const int wide_nt = (use_wide && p.rpp == 1) ? (c->wide_threads ? c->wide_threads : kWideThreadsAuto) : 256;
        const int nt = (variant == 0 && use_lds) ? lds_threads(c, lds) : (use_wide ? wide_nt : 256);
        const unsigned wpb = (unsigned)nt / 64u;                                    // waves per block
        unsigned blocks = std::min<unsigned>(c->persist_blocks * 256u / (unsigned)nt,
                                             std::max(1u, (items + wpb - 1) / wpb));
        dim3 grid(blocks);
        // occupancy: 7 waves/SIMD for LDS scenes (72 VGPRs, a few spilled: +0.8% on C2 over
        // 6, which was +5% over 5; 8 spills 20+ and loses 7%), 6 for global-memory scenes (7
        // leaves fewer top nodes per block in LDS: -6% on the C3 stand-in)
        const int mw = c->minw ? c->minw : (use_lds ? 7 : 6);
        // Overlapped short renders (tuning key 18): at most this many 256-thread blocks per CU
        // (automatic: one fewer than resident, two fewer with 3+ render slots), so the accumulate pass and the ACES view of the
        // previous render find free slots beside the next render instead of waiting for its
        // blocks to retire.  1080p Cornell, one frame per dispatch (tools/interactive_fps.py):
        // 0.534 -> 0.514 ms per frame, and 0.68 -> 0.55-0.58 with every frame shown
        // (pt_present, lag 2); accumulate pass 243 -> 103 us.  Round 5, 3 slots, 600-800 frames
        // (profiles/ab/r05i_interactive_sweep.json, r05j_*): render only, 2 / 3 / 4 / 5 blocks
        // per CU 0.513 / 0.473 / 0.537 / 0.493 ms per frame; every frame presented at lag 2, 3
        // blocks 0.55-0.62 against 0.530 at 5.  So 3 slots take 3 blocks per CU, or 5 when the
        // caller presented after the previous render (aces_fuse).
        if (overlap && nt == 256) {
            const int bpc = c->overlap_bpc ? c->overlap_bpc
                          : c->overlap_slots >= 3 ? (c->aces_fuse ? std::max(1, mw - 2) : 3)
                                                  : std::max(1, mw - 1);
            grid.x = std::min<unsigned>(grid.x, (unsigned)(bpc * c->n_cu));
        }
        // global scene: the top nodes staged per block, at most what mw blocks per CU fit in
        // its 160 KiB of LDS (the first K of the breadth-first numbering, any K <= n_top)
        if (mw > 6) p.n_top = std::min(c->n_top, 160 * 1024 / mw / 32 - 8);
        // materials + spheres beside the top nodes when they are small (<= 4 KiB)
        const size_t shade_bytes = (size_t)(3 * c->n_mats + 2 * c->n_spheres) * sizeof(float4);
        p.shade_lds = shade_bytes <= 4096;
        if (use_wide) {   // top records: 48 B each, within the block's share of the CU's LDS
            // (256-thread blocks: one per resident wave per SIMD, the instantiation's 5-7; the
            // raysPerPixel > 1 one is built for 6)
            const size_t blocks_cu = wide_nt == 1024 ? 1
                                   : (wide_nt == 256 ? (size_t)(p.rpp > 1 ? 6 : std::min(std::max(mw, 5), 7))
                                                     : (size_t)(6 * 256 / wide_nt));
            // (1 KiB below the even share: the allocation granule must not cost a block per CU)
            p.wide_top = (int)std::min<size_t>({(size_t)c->n_wide, (size_t)kWideTopMax,
                                                ((size_t)160 * 1024 / blocks_cu - (p.shade_lds ? shade_bytes : 0) - 1024) / 48});
        }
        const size_t top_lds = use_wide ? (size_t)p.wide_top * 3 * sizeof(float4) + (p.shade_lds ? shade_bytes : 0)
                                        : (size_t)p.n_top * 2 * sizeof(float4) + (p.shade_lds ? shade_bytes : 0);
#define PT_LAUNCH_SM(L, M)                                                                                \
    if (c->counting && p.rgb) hipLaunchKernelGGL((k_render_sm<true, L, 5, M, true>), grid, dim3(256), L ? lds : top_lds, rs, p); \
    else if (c->counting) hipLaunchKernelGGL((k_render_sm<true, L, 5, M, false>), grid, dim3(256), L ? lds : top_lds, rs, p); \
    else if (p.rgb && mw == 8 && !M) hipLaunchKernelGGL((k_render_sm<false, L, 8, false, true>), grid, dim3(256), L ? lds : top_lds, rs, p); \
    else if (p.rgb && mw == 7 && !M && L && c->walk_np == kPadNodes) hipLaunchKernelGGL((k_render_sm<false, true, 7, false, true, true>), grid, dim3(256), lds, rs, p); \
    else if (p.rgb && mw == 7 && !M) hipLaunchKernelGGL((k_render_sm<false, L, 7, false, true>), grid, dim3(256), L ? lds : top_lds, rs, p); \
    else if (p.rgb && mw >= 6) hipLaunchKernelGGL((k_render_sm<false, L, 6, M, true>), grid, dim3(256), L ? lds : top_lds, rs, p); \
    else if (p.rgb) hipLaunchKernelGGL((k_render_sm<false, L, 5, M, true>), grid, dim3(256), L ? lds : top_lds, rs, p); \
    else if (mw >= 6) hipLaunchKernelGGL((k_render_sm<false, L, 6, M, false>), grid, dim3(256), L ? lds : top_lds, rs, p); \
    else hipLaunchKernelGGL((k_render_sm<false, L, 5, M, false>), grid, dim3(256), L ? lds : top_lds, rs, p);
#define PT_LAUNCH_WIDE(NT, MW)                                                                                \
    if (p.rgb) hipLaunchKernelGGL((k_render_sm<false, true, MW, false, true, false, NT>), grid, dim3(NT), lds, rs, p); \
    else hipLaunchKernelGGL((k_render_sm<false, true, MW, false, false, false, NT>), grid, dim3(NT), lds, rs, p);
        // lds_threads: LDS scene, variant 0, one ray per pixel; the register budget of the
        // waves that are resident (6, 6, 4 per SIMD), not of 7
        if (use_wide) {
#define PT_LAUNCH_WIDE_G(NT, MW)                                                                              \
    if (p.rgb) hipLaunchKernelGGL((k_render_sm<false, false, MW, false, true, false, NT, true>), grid, dim3(NT), top_lds, rs, p); \
    else hipLaunchKernelGGL((k_render_sm<false, false, MW, false, false, false, NT, true>), grid, dim3(NT), top_lds, rs, p);
            if (p.rgb && p.rpp > 1) hipLaunchKernelGGL((k_render_sm<false, false, 6, true, true, false, 256, true>), grid, dim3(256), top_lds, rs, p);
            else if (p.rpp > 1) hipLaunchKernelGGL((k_render_sm<false, false, 6, true, false, false, 256, true>), grid, dim3(256), top_lds, rs, p);
            else if (nt == 512) { PT_LAUNCH_WIDE_G(512, 6) }
            else if (nt == 768) { PT_LAUNCH_WIDE_G(768, 6) }
            else if (nt == 1024) { PT_LAUNCH_WIDE_G(1024, 4) }
            else if (mw == 5) { PT_LAUNCH_WIDE_G(256, 5) }
            else if (mw == 7) { PT_LAUNCH_WIDE_G(256, 7) }
            else { PT_LAUNCH_WIDE_G(256, 6) }
#undef PT_LAUNCH_WIDE_G
        } else if (nt > 256) {
            if (nt == 512) { PT_LAUNCH_WIDE(512, 6) }
            else if (nt == 768) { PT_LAUNCH_WIDE(768, 6) }
            else { PT_LAUNCH_WIDE(1024, 4) }
#undef PT_LAUNCH_WIDE
        } else {
            bool multi = p.rpp > 1;
            if (use_lds && multi) { PT_LAUNCH_SM(true, true) }
            else if (use_lds) { PT_LAUNCH_SM(true, false) }
            else if (multi) { PT_LAUNCH_SM(false, true) }
            else { PT_LAUNCH_SM(false, false) }
#undef PT_LAUNCH_SM
        }
        if (p.rgb) {
            if (overlap) {
                HIPCHK(c, hipEventRecord(c->ev_rdone[re], rs));
                HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_rdone[re], 0));
            }
            long long px = (long long)c->rows_local * p.W;
            // a presenting caller's view of the new image, written by the same pass (not inside
            // a captured graph: its replays are not followed by pt_present_begin's check)
            p.aces_out = (c->aces_fuse && !frame_dev) ? c->rgba8 : nullptr;
            c->stage_ok = p.aces_out != nullptr;
            if (n_frames > kShortLaunch)
                hipLaunchKernelGGL((k_accum_frames<kAccumPixLong, kAccumFramesLong>),
                                   dim3((unsigned)((px + 256 * kAccumPixLong - 1) / (256 * kAccumPixLong))), dim3(256), 0,
                                   c->stream, p);
            else
                hipLaunchKernelGGL((k_accum_frames<kAccumPix, 1>),
                                   dim3((unsigned)((px + 256 * kAccumPix - 1) / (256 * kAccumPix))), dim3(256), 0,
                                   c->stream, p);
            if (overlap) {
                HIPCHK(c, hipEventRecord(c->ev_adone[re], c->stream));
                c->adone_rec[re] = true;
            }
        }
    }
    // The queue order is recomputed from the accumulated tile costs after every long launch,
    // but only after every kOrderEvery-th short one (the first time after kOrderFirst): a
    // sort after each one-frame 1080p launch cost more than the order gained (adaptive off:
    // +0.5%), while a sorted order, even one 64 frames old, keeps most of the gain
    // (same-process A/B of one-frame launches, against sorting every launch: every 4th
    // +6%, 8th +8.4%, 16th +9.8%, 64th +10.7%).  Captured graphs (frame_dev) sort every replay.
    if (p.tile_cost && c->n_tiles > 1 &&
        (frame_dev || force_sort || n_frames > kShortLaunch ||
         ++c->order_skip >= (c->order_sorted ? kOrderEvery : kOrderFirst))) {
        c->order_skip = 0;
        c->order_sorted = true;
        hipLaunchKernelGGL(k_tile_order, dim3(1), dim3(1024), 0, c->stream, c->d_tile_cost, c->d_tile_perm,
                           c->n_tiles, c->tiles_x);
        if (!frame_dev) {   // later overlapped renders start after the new order
            HIPCHK(c, hipEventRecord(c->ev_fence, c->stream));
            c->fence_rec = true;
        }
    }
    HIPCHK(c, hipGetLastError());
    return PT_OK;
}

// A pair of timing events from the recycled pool, queued for pt_sync.
static int take_events(pt_ctx* c, hipEvent_t ev[2]) {
    for (int i = 0; i < 2; i++) {
        if (c->ev_free.empty()) {
            HIPCHK(c, hipEventCreate(&ev[i]));
        } else {
            ev[i] = c->ev_free.back();
            c->ev_free.pop_back();
        }
    }
    c->ev_pending.emplace_back(ev[0], ev[1]);
    return PT_OK;
}

// Enqueues a render of n_frames as launches of at most launch_frames() frames (one launch
// when the scratch budget and the 32-bit queue ids allow).  Launch j > 0 continues the
// running mean (accumulate = 1), so the image is that of n_frames single dispatches.
static int enqueue_frames(pt_ctx* c, int frame_first, int n_frames, int acc_first, const int* frame_dev,
                          int frame_offset) {
    // A long render on a context whose tile order was never sorted (the first render after an
    // upload) would run in raster order.  Its first kProbeFrames frames go first as a short
    // launch whose tile costs are sorted at once, so the remaining frames already run most-
    // expensive-tile-first; the continuation accumulates, so the image is unchanged.
    if (!frame_dev && c->adaptive && !c->counting && !c->order_sorted && n_frames >= kProbeMin) {
        // the scratch for the launch this render would have been: the next identical render
        // then finds it in place instead of freeing and mapping ~25 GB (1.5 s measured on one
        // box) in front of its kernel
        const int full = launch_frames(c, n_frames);
        if (split_mode(c, full, plan_group(c, full))) {
            int rc = ensure_rgb(c, full);
            if (rc) return rc;
        }
        int rc = enqueue_render(c, frame_first, kProbeFrames, acc_first, nullptr, 0, true);
        if (rc) return rc;
        frame_first += kProbeFrames;
        n_frames -= kProbeFrames;
        acc_first = 1;
    }
    const int step = launch_frames(c, n_frames);
    for (int done = 0; done < n_frames; done += step) {
        const int n = std::min(step, n_frames - done);
        int rc = enqueue_render(c, frame_first + done, n, done ? 1 : acc_first, frame_dev, frame_offset + done);
        if (rc) return rc;
    }
    return PT_OK;
}

int pt_render_async(pt_ctx* c, int frame_first, int n_frames, int acc_first) {
    if (!c) return PT_E_ARG;
    if (!c->scene_ok) return fail(c, PT_E_STATE, "pt_render before pt_upload_scene");
    if (n_frames <= 0) return fail(c, PT_E_ARG, "n_frames must be > 0");
    HIPCHK(c, hipSetDevice(c->cfg.device));
    {
        int rc0 = ensure_tiles(c);
        if (rc0) return rc0;
    }
    if (c->counting) HIPCHK(c, hipMemsetAsync(c->d_counters, 0, 16 * sizeof(unsigned long long), c->stream));
    hipEvent_t ev[2];
    int rc = take_events(c, ev);
    if (rc) return rc;
    HIPCHK(c, hipEventRecord(ev[0], c->stream));
    // a caller that presented after its previous render gets the ACES view from this render's
    // accumulate pass (pt_present_begin then only copies it)
    c->aces_fuse = c->presented;
    c->presented = false;
    rc = enqueue_frames(c, frame_first, n_frames, acc_first, nullptr, 0);
    if (rc) return rc;
    HIPCHK(c, hipEventRecord(ev[1], c->stream));
    c->count_pending = c->counting;
    return PT_OK;
}

static void drop_graph(pt_ctx* c) {
    if (c->graph_exec) (void)hipGraphExecDestroy(c->graph_exec);
    if (c->graph) (void)hipGraphDestroy(c->graph);
    c->graph_exec = nullptr;
    c->graph = nullptr;
    c->graph_rgb = nullptr;
    if (!c->graph_owned.empty()) {      // scratch only the dropped graph still referenced
        (void)hipSetDevice(c->cfg.device);
        (void)hipStreamSynchronize(c->stream);
        for (float* b : c->graph_owned) (void)hipFree(b);
        c->graph_owned.clear();
    }
}

int pt_progressive_setup(pt_ctx* c, int frames_per_launch, int launches_per_replay) {
    if (!c) return PT_E_ARG;
    c->stage_ok = false;
    if (!c->scene_ok) return fail(c, PT_E_STATE, "pt_progressive_setup before pt_upload_scene");
    if (frames_per_launch <= 0 || launches_per_replay <= 0) return fail(c, PT_E_ARG, "counts must be > 0");
    if (c->counting) return fail(c, PT_E_STATE, "counting is not supported in graph replay");
    HIPCHK(c, hipSetDevice(c->cfg.device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    drop_graph(c);
    {
        int rc0 = ensure_tiles(c);
        if (rc0) return rc0;
    }
    if (!c->d_frame) HIPCHK(c, hipMalloc(&c->d_frame, 64));
    {   // no allocation inside the capture: the scratch of the largest sub-launch first
        const int n = launch_frames(c, frames_per_launch);
        if (split_mode(c, n, plan_group(c, n))) {
            int rc0 = ensure_rgb(c, n);
            if (rc0) return rc0;
        }
    }
    HIPCHK(c, hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
    int rc = PT_OK;
    for (int i = 0; i < launches_per_replay && rc == PT_OK; i++)
        rc = enqueue_frames(c, 0, frames_per_launch, 0, c->d_frame, i * frames_per_launch);
    if (rc == PT_OK) {
        hipLaunchKernelGGL(k_advance_frames, dim3(1), dim3(64), 0, c->stream, c->d_frame,
                           frames_per_launch * launches_per_replay);
    }
    hipGraph_t g = nullptr;
    hipError_t e = hipStreamEndCapture(c->stream, &g);
    if (rc != PT_OK) { if (g) (void)hipGraphDestroy(g); return rc; }
    if (e != hipSuccess) return fail(c, PT_E_HIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(e));
    c->graph = g;
    HIPCHK(c, hipGraphInstantiate(&c->graph_exec, g, nullptr, nullptr, 0));
    c->graph_rgb = c->d_rgb;
    c->graph_frames = frames_per_launch * launches_per_replay;
    return pt_progressive_reset(c, 1);
}

int pt_progressive_reset(pt_ctx* c, int next_frame) {
    if (!c) return PT_E_ARG;
    if (!c->d_frame) return fail(c, PT_E_STATE, "pt_progressive_setup first");
    if (next_frame < 1) return fail(c, PT_E_ARG, "frames start at 1");
    HIPCHK(c, hipSetDevice(c->cfg.device));
    HIPCHK(c, hipMemcpyAsync(c->d_frame, &next_frame, sizeof(int), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return PT_OK;
}

int pt_progressive_run(pt_ctx* c, int replays) {
    if (!c) return PT_E_ARG;
    c->stage_ok = false;
    if (!c->graph_exec) return fail(c, PT_E_STATE, "pt_progressive_setup first");
    if (replays <= 0) return fail(c, PT_E_ARG, "replays must be > 0");
    HIPCHK(c, hipSetDevice(c->cfg.device));
    hipEvent_t ev[2];
    for (int i = 0; i < 2; i++) {
        if (c->ev_free.empty()) {
            HIPCHK(c, hipEventCreate(&ev[i]));
        } else {
            ev[i] = c->ev_free.back();
            c->ev_free.pop_back();
        }
    }
    c->ev_pending.emplace_back(ev[0], ev[1]);
    HIPCHK(c, hipEventRecord(ev[0], c->stream));
    for (int r = 0; r < replays; r++) HIPCHK(c, hipGraphLaunch(c->graph_exec, c->stream));
    HIPCHK(c, hipEventRecord(c->ev_fence, c->stream));   // the replays sort the tile order
    c->fence_rec = true;
    HIPCHK(c, hipEventRecord(ev[1], c->stream));
    return PT_OK;
}

int pt_sync(pt_ctx* c) {
    if (!c) return PT_E_ARG;
    HIPCHK(c, hipSetDevice(c->cfg.device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (auto& pr : c->ev_pending) {
        float ms = 0;
        HIPCHK(c, hipEventElapsedTime(&ms, pr.first, pr.second));
        c->last_ms = ms;
        c->total_ms += ms;
        c->n_launches++;
        c->ev_free.push_back(pr.first);
        c->ev_free.push_back(pr.second);
    }
    c->ev_pending.clear();
    if (c->count_pending) {
        HIPCHK(c, hipMemcpy(c->last_counts, c->d_counters, 16 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        c->count_pending = false;
    }
    return PT_OK;
}

int pt_render(pt_ctx* c, int frame_first, int n_frames, int acc_first) {
    int rc = pt_render_async(c, frame_first, n_frames, acc_first);
    if (rc) return rc;
    return pt_sync(c);
}

int pt_rows(const pt_ctx* c, int* rows_local, int* row0, int* row_stride) {
    if (!c) return PT_E_ARG;
    if (rows_local) *rows_local = c->rows_local;
    if (row0) *row0 = c->cfg.rank;
    if (row_stride) *row_stride = c->cfg.world;
    return PT_OK;
}

int pt_get_config(const pt_ctx* c, pt_config* out) {
    if (!c || !out) return PT_E_ARG;
    *out = c->cfg;
    return PT_OK;
}

// Scene replication for pt_group_upload_scene (pt_group.hip, not part of the public ABI):
// gives `dst` a device scene of exactly `src`'s layout -- the same host-side facts and
// buffers of the same sizes, contents undefined -- and returns both contexts' buffer pointers
// and sizes, so the caller can fill dst's from src's (an RCCL broadcast across devices or a
// device copy).  Both contexts must have the same width (tile facts are per image).
int pt__scene_replicate_layout(pt_ctx* dst, const pt_ctx* src, void* dptr[10], const void* sptr[10],
                               size_t bytes[10]) {
    if (!dst || !src || !dptr || !sptr || !bytes) return PT_E_ARG;
    if (!src->scene_ok) return fail(dst, PT_E_STATE, "source context has no scene");
    HIPCHK(dst, hipSetDevice(dst->cfg.device));
    HIPCHK(dst, hipStreamSynchronize(dst->stream));
    drop_graph(dst);
    free_scene(dst);
    const size_t nd = 2 * (size_t)std::max(src->n_nodes, 1), nt = 8 * (size_t)std::max(src->n_slots / 2, 1);
    const size_t nm = 3 * (size_t)std::max(src->n_mats, 1), ns = 2 * (size_t)std::max(src->n_spheres, 1);
    const size_t nw = 16 * (size_t)src->walk_np, nk = src->d_walk_sk ? 18 * (size_t)src->walk_np : 0;
    const size_t ni = src->wide_ok ? (size_t)src->n_wide : 0;   // the wide walk's arrays (pt_wide.h)
    const size_t sz[10] = {nd, nt, nm, ns, nw, nk, kWideStride * ni, 2 * ni, ni ? nd : 0, 8 * ni};
    float4** mine[10] = {&dst->d_nodes, &dst->d_tris, &dst->d_mats, &dst->d_spheres, &dst->d_walk_lds, &dst->d_walk_sk,
                         &dst->d_wrec, &dst->d_wlbox, &dst->d_nodesw, &dst->d_trisw};
    const float4* theirs[10] = {src->d_nodes, src->d_tris, src->d_mats, src->d_spheres, src->d_walk_lds, src->d_walk_sk,
                                src->d_wrec, src->d_wlbox, src->d_nodesw, src->d_trisw};
    for (int i = 0; i < 10; i++) {
        bytes[i] = sz[i] * sizeof(float4);
        sptr[i] = theirs[i];
        if (sz[i]) HIPCHK(dst, hipMalloc(mine[i], bytes[i]));
        dptr[i] = *mine[i];
    }
    dst->n_nodes = src->n_nodes;
    dst->n_spheres = src->n_spheres;
    dst->n_mats = src->n_mats;
    dst->n_slots = src->n_slots;
    dst->n_top = src->n_top;
    dst->scene_fast = src->scene_fast;
    dst->walk_nested = src->walk_nested;
    std::memcpy(dst->cons_m, src->cons_m, sizeof(dst->cons_m));
    dst->wide_ok = src->wide_ok;
    dst->leaf_cert_ok = src->leaf_cert_ok;
    dst->n_wide = src->n_wide;
    std::memcpy(dst->wide_cw, src->wide_cw, sizeof(dst->wide_cw));
    dst->walk_np = src->walk_np;
    dst->lds_bytes = src->lds_bytes;
    dst->lds_bytes_sk = src->lds_bytes_sk;
    std::memcpy(dst->root_box, src->root_box, sizeof(dst->root_box));
    dst->root_child = src->root_child;
    dst->order_sorted = false;
    dst->order_skip = 0;
    // scene_ok stays false until the caller has filled the buffers (pt__scene_set_ready): a
    // failed broadcast or copy must not leave a context rendering from uninitialised memory
    dst->scene_ok = false;
    return PT_OK;
}

// ACES epilogue of n RGBA32F pixels on a caller's stream (pt_group's gathered frame; the
// same k_aces as pt_read_rgba8_aces and pt_present_*).  Internal, not part of the public ABI.
int pt__aces_launch(const void* src, void* dst, long long n, void* stream) {
    if (!src || !dst || n < 0) return PT_E_ARG;
    if (n == 0) return PT_OK;
    hipLaunchKernelGGL(k_aces, dim3((unsigned)((n + 256 * kAcesPix - 1) / (256 * kAcesPix))), dim3(256), 0, (hipStream_t)stream,
                       (const float4*)src, (uchar4*)dst, n);
    return hipGetLastError() == hipSuccess ? PT_OK : PT_E_HIP;
}

int pt__scene_set_ready(pt_ctx* c, int ready) {
    if (!c) return PT_E_ARG;
    c->scene_ok = ready != 0 && c->d_mats != nullptr;
    return PT_OK;
}

int pt_read_rgba32f(pt_ctx* c, float* dst, size_t bytes) {
    if (!c || !dst) return PT_E_ARG;
    size_t need = (size_t)c->rows_local * c->cfg.width * sizeof(float4);
    if (bytes < need) return fail(c, PT_E_ARG, "destination too small");
    HIPCHK(c, hipSetDevice(c->cfg.device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(dst, c->accum, need, hipMemcpyDeviceToHost));
    return PT_OK;
}

int pt_write_rgba32f(pt_ctx* c, const float* src, size_t bytes) {
    if (!c || !src) return PT_E_ARG;
    c->stage_ok = false;
    size_t need = (size_t)c->rows_local * c->cfg.width * sizeof(float4);
    if (bytes < need) return fail(c, PT_E_ARG, "source too small");
    HIPCHK(c, hipSetDevice(c->cfg.device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(c->accum, src, need, hipMemcpyHostToDevice));
    return PT_OK;
}

int pt_read_rgba8_aces(pt_ctx* c, unsigned char* dst, size_t bytes) {
    if (!c || !dst) return PT_E_ARG;
    long long n = (long long)c->rows_local * c->cfg.width;
    if (bytes < (size_t)n * 4) return fail(c, PT_E_ARG, "destination too small");
    if (n == 0) return PT_OK;
    HIPCHK(c, hipSetDevice(c->cfg.device));
    // the view the last render's accumulate pass wrote when the caller also read (or presented)
    // after the render before it (pt_present_begin), else the ACES pass here
    if (!c->stage_ok) {
        hipLaunchKernelGGL(k_aces, dim3((unsigned)((n + 256 * kAcesPix - 1) / (256 * kAcesPix))), dim3(256), 0,
                           c->stream, c->accum, c->rgba8, n);
        HIPCHK(c, hipGetLastError());
    }
    c->stage_ok = true;     // rgba8 is the view of the current image
    c->presented = true;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(dst, c->rgba8, (size_t)n * 4, hipMemcpyDeviceToHost));
    return PT_OK;
}

// Asynchronous presentation for a viewer that shows every frame (ogl_path_trace.h:189-192
// draws each frame's texture on the GPU that rendered it; a headless caller reads it back).
// begin: the ACES epilogue of the current image on the context stream (after every render
// issued so far and its running mean), then a copy into pinned host memory on a separate
// stream, so renders issued after it run while the image crosses PCIe.  end: waits for that
// copy and hands out the pinned pixels.
int pt_present_begin(pt_ctx* c, int buf) {
    if (!c) return PT_E_ARG;
    if (buf < 0 || buf >= kPresentBufs) return fail(c, PT_E_ARG, "present buffer must be 0..3");
    const long long n = (long long)c->rows_local * c->cfg.width;
    HIPCHK(c, hipSetDevice(c->cfg.device));
    if (!c->present_host[buf]) {
        HIPCHK(c, hipHostMalloc((void**)&c->present_host[buf], std::max<long long>(n, 1) * sizeof(uchar4),
                                hipHostMallocDefault));
        HIPCHK(c, hipEventCreateWithFlags(&c->ev_copied[buf], hipEventDisableTiming));
    }
    // a buffer begun again before its end: its previous copy must land first
    if (c->present_pending[buf]) HIPCHK(c, hipEventSynchronize(c->ev_copied[buf]));
    c->present_pending[buf] = false;
    // the view of the current image: written by the last render's accumulate pass when the
    // caller presented after the render before it (stage_ok), else the ACES pass here
    if (n > 0 && !c->stage_ok) {
        hipLaunchKernelGGL(k_aces, dim3((unsigned)((n + 256 * kAcesPix - 1) / (256 * kAcesPix))), dim3(256), 0,
                           c->stream, c->accum, c->rgba8, n);
        HIPCHK(c, hipGetLastError());
    }
    c->stage_ok = true;     // rgba8 is the view of the current image
    c->presented = true;
    // the copy on the context stream itself: a copy stream waiting on an event started each
    // copy about 150 us after the view was ready (one-frame loop with lag 2: 0.578 -> 0.537
    // ms per frame); the next render's accumulate pass, which rewrites the view, follows it
    if (n > 0)
        HIPCHK(c, hipMemcpyAsync(c->present_host[buf], c->rgba8, (size_t)n * sizeof(uchar4), hipMemcpyDeviceToHost,
                                 c->stream));
    HIPCHK(c, hipEventRecord(c->ev_copied[buf], c->stream));
    c->present_pending[buf] = true;
    return PT_OK;
}

int pt_present_end(pt_ctx* c, int buf, const unsigned char** pixels) {
    if (!c || !pixels) return PT_E_ARG;
    if (buf < 0 || buf >= kPresentBufs) return fail(c, PT_E_ARG, "present buffer must be 0..3");
    if (!c->present_pending[buf]) return fail(c, PT_E_STATE, "pt_present_end without pt_present_begin");
    HIPCHK(c, hipSetDevice(c->cfg.device));
    HIPCHK(c, hipEventSynchronize(c->ev_copied[buf]));
    c->present_pending[buf] = false;
    *pixels = c->present_host[buf];
    return PT_OK;
}

int pt_accum_device(pt_ctx* c, void** ptr, size_t* bytes) {
    if (!c) return PT_E_ARG;
    c->stage_ok = false;   // the caller may write the image through this pointer
    if (ptr) *ptr = c->accum;
    if (bytes) *bytes = (size_t)c->rows_local * c->cfg.width * sizeof(float4);
    return PT_OK;
}

int pt_copy_rows_device(pt_ctx* c, void* dst, size_t bytes) {
    if (!c || !dst) return PT_E_ARG;
    size_t need = (size_t)c->rows_local * c->cfg.width * sizeof(float4);
    if (bytes < need) return fail(c, PT_E_ARG, "destination too small");
    HIPCHK(c, hipSetDevice(c->cfg.device));
    HIPCHK(c, hipMemcpyAsync(dst, c->accum, need, hipMemcpyDeviceToDevice, c->stream));
    return pt_sync(c);
}

int pt_timing(pt_ctx* c, double* total_ms, int* n, int reset) {
    if (!c) return PT_E_ARG;
    if (total_ms) *total_ms = c->total_ms;
    if (n) *n = c->n_launches;
    if (reset) { c->total_ms = 0.0; c->n_launches = 0; }
    return PT_OK;
}

int pt_stream(pt_ctx* c, void** s) {
    if (!c || !s) return PT_E_ARG;
    c->stage_ok = false;   // ... or queue work on this stream that does
    *s = (void*)c->stream;
    return PT_OK;
}

#ifdef PT_WAVE_TRACE
extern "C" int pt_debug_wave_trace(unsigned long long* out, int max_waves, int reset) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    const int n = max_waves < kWaveTraceMax ? max_waves : kWaveTraceMax;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wave_trace), sizeof(unsigned long long) * 4 * n) != hipSuccess) return -1;
    if (reset) {
        std::vector<unsigned long long> z(4 * (size_t)kWaveTraceMax, 0ull);
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_wave_trace), z.data(), z.size() * 8) != hipSuccess) return -1;
    }
    return n;
}
#endif

#ifdef PT_PHASE_CLOCK
extern "C" int pt_debug_phase_clock(unsigned long long out[8], int reset) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase_clk), sizeof(unsigned long long) * 8) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_phase_clk), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif


int pt_stats_ex(pt_ctx* c, unsigned long long out[16]) {
    if (!c || !out) return PT_E_ARG;
    std::memcpy(out, c->last_counts, sizeof(c->last_counts));
    out[13] = c->lds_bytes;
    out[14] = c->walk_nested ? c->lds_bytes_sk : 0;
    out[15] = cons_walk_on(c);               // the scene's LDS walk culls (slab_oct_cons)
    return PT_OK;
}

int pt_stats(pt_ctx* c, double* ms, unsigned long long out[5]) {
    if (!c) return PT_E_ARG;
    if (ms) *ms = c->last_ms;
    if (out) std::memcpy(out, c->last_counts, 5 * sizeof(unsigned long long));
    return PT_OK;
}

}  // extern "C"
