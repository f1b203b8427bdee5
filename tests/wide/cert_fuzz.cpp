// TEST INFRASTRUCTURE: adversarial check of the leaf re-test certificate (pt_wide.h
// ptw::leaf_certificate) against the reference's exact slab test (bvh_intersect,
// computeShader.c:309-365) of a leaf box that is the bounding box of its two triangles
// (bvh.h:29-52).  Rays are aimed at points ON the triangles -- vertices, edges, a few ulps
// inside or outside -- from near and far origins, with axis-aligned (flat) triangles among
// them; the hit is hit_triangle's (computeShader.c:274-307).  For every hit that could move t
// (t_h in (1e-4, t)), at t = t_h's successor and at larger t: certificate => exact test
// passes.  Exit status 0 = no violation; prints one JSON line.
//   usage: cert_fuzz [cases] [seed]
#include "../../opengl-path-tracing_amd/csrc/pt_wide.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

using pt::f3;
using pt::mk;

namespace {

uint64_t rs = 88172645463325252ull;
uint64_t nx() { rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17; return rs; }
float uni() { return (float)((nx() >> 40) * 0x1p-24); }                 // [0, 1)
float sym() { return 2.0f * uni() - 1.0f; }
float nudge(float v, int k) {                                            // k ulps away
    for (int i = 0; i < std::abs(k); i++) v = std::nextafter(v, k > 0 ? INFINITY : -INFINITY);
    return v;
}

bool slab_exact(const float* lo, const float* hi, f3 o, f3 d, float cur_t) {   // :309-365
    float tmin = (lo[0] - o.x) / d.x, tmax = (hi[0] - o.x) / d.x;
    if (tmin > tmax) std::swap(tmin, tmax);
    float tymin = (lo[1] - o.y) / d.y, tymax = (hi[1] - o.y) / d.y;
    if (tymin > tymax) std::swap(tymin, tymax);
    if ((tmin > tymax) || (tymin > tmax)) return false;
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    float tzmin = (lo[2] - o.z) / d.z, tzmax = (hi[2] - o.z) / d.z;
    if (tzmin > tzmax) std::swap(tzmin, tzmax);
    if ((tmin > tzmax) || (tzmin > tmax)) return false;
    if (tzmin > tmin) tmin = tzmin;
    return !(tmin > cur_t);
}

// hit_triangle (:274-307): -1 on a miss; n out
float hit_triangle(f3 o, f3 d, f3 v0, f3 v1, f3 v2, f3& n) {
    n = pt::normalize(pt::cross(v1 - v0, v2 - v0));
    const float dd = -pt::dot(n, v0);
    const float t = -(pt::dot(n, o) + dd) / pt::dot(n, d);
    if (t < 0.0f) return -1.0f;
    const f3 p = o + d * t;
    if (pt::dot(n, pt::cross(v1 - v0, p - v0)) > 0.0f && pt::dot(n, pt::cross(v2 - v1, p - v1)) > 0.0f &&
        pt::dot(n, pt::cross(v0 - v2, p - v2)) > 0.0f)
        return t;
    return -1.0f;
}

bool in_guard(f3 o, f3 d) {
    auto g0 = [](float v) { float a = std::fabs(v); return v == 0.0f || (a >= 0x1p-40f && a <= 0x1p60f); };
    auto g1 = [](float v) { float a = std::fabs(v); return a >= 0x1p-20f && a <= 2.0f; };
    return g0(o.x) && g0(o.y) && g0(o.z) && g1(d.x) && g1(d.y) && g1(d.z);
}

f3 rand_tri_vertex(f3 c, float s, int flat_axis, float flat_v) {
    f3 v = mk(c.x + s * sym(), c.y + s * sym(), c.z + s * sym());
    if (flat_axis == 0) v.x = flat_v;
    if (flat_axis == 1) v.y = flat_v;
    if (flat_axis == 2) v.z = flat_v;
    return v;
}

}  // namespace

int main(int argc, char** argv) {
    const long cases = argc > 1 ? std::atol(argv[1]) : 200000;
    if (argc > 2) rs ^= (uint64_t)std::atoll(argv[2]) * 0x9e3779b97f4a7c15ull;
    long hits = 0, certified = 0, violations = 0, exact_fail = 0, flat_hits = 0, flat_cert = 0;
    for (long k = 0; k < cases; k++) {
        // the leaf: two triangles around a centre at a random scale and offset
        const float scale = std::ldexp(1.0f, (int)(nx() % 12) - 6);
        const float off = (nx() % 4 == 0) ? std::ldexp(1.0f, (int)(nx() % 12)) * sym() : 0.0f;
        const f3 c = mk(off + sym(), off * 0.5f + sym(), sym());
        const int flat = (int)(nx() % 5) - 2;          // -2, -1: none; 0..2: flat axis (both triangles)
        const float fv = (flat == 0 ? c.x : flat == 1 ? c.y : c.z) + (nx() % 2 ? 0.0f : scale * sym());
        f3 V[6];
        for (int i = 0; i < 6; i++) V[i] = rand_tri_vertex(c, scale, flat >= 0 ? flat : -1, fv);
        if (nx() % 3 == 0) { V[3] = V[0]; V[4] = V[2]; }      // a quad's two halves share an edge
        float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int i = 0; i < 6; i++) {                          // bvh.h:29-52
            const float a[3] = {V[i].x, V[i].y, V[i].z};
            for (int q = 0; q < 3; q++) { lo[q] = std::fmin(lo[q], a[q]); hi[q] = std::fmax(hi[q], a[q]); }
        }
        // the target: a vertex, an edge point or an interior point of either triangle, nudged
        const int tri = (int)(nx() % 2);
        const f3 A = V[3 * tri], B = V[3 * tri + 1], Cc = V[3 * tri + 2];
        f3 tg;
        const uint64_t kind = nx() % 4;
        if (kind == 0) tg = (nx() % 3 == 0) ? A : (nx() % 2 ? B : Cc);
        else if (kind == 1) { const float w = uni(); tg = A * (1.0f - w) + B * w; }
        else { float a = uni(), b = uni(); if (a + b > 1.0f) { a = 1.0f - a; b = 1.0f - b; } tg = A + (B - A) * a + (Cc - A) * b; }
        tg = mk(nudge(tg.x, (int)(nx() % 7) - 3), nudge(tg.y, (int)(nx() % 7) - 3), nudge(tg.z, (int)(nx() % 7) - 3));
        // the origin: near or far, sometimes on an axis plane of the box
        const float dist = std::ldexp(1.0f, (int)(nx() % 16) - 4);
        f3 o = mk(tg.x + dist * sym(), tg.y + dist * sym(), tg.z + dist * sym());
        if (nx() % 8 == 0) o.x = lo[0];
        if (nx() % 8 == 0) o.y = hi[1];
        f3 d = tg - o;
        if (nx() % 6 == 0) d.x = d.x * 1e-4f;                // near-axis directions
        if (pt::dot(d, d) == 0.0f) continue;
        d = pt::normalize(d);
        if (!in_guard(o, d)) continue;
        f3 n;
        const f3 T0 = V[3 * tri], T1 = V[3 * tri + 1], T2 = V[3 * tri + 2];
        const float th = hit_triangle(o, d, T0, T1, T2, n);
        if (!(th > 0.0001f)) continue;
        hits++;
        const f3 p = o + d * th;
        const bool cert = ptw::leaf_certificate(p, n, T0, T1, T2, ptw::abs_max3(o));
        const bool fl = flat >= 0;
        flat_hits += fl;
        for (int r = 0; r < 3; r++) {                          // t just above t_h, and larger
            const float t = r == 0 ? std::nextafter(th, INFINITY) : (r == 1 ? th * 1.5f : INFINITY);
            const bool ex = slab_exact(lo, hi, o, d, t);
            if (!ex) exact_fail++;
            if (cert && !ex) {
                if (violations < 10)
                    std::fprintf(stderr, "VIOLATION o=(%a,%a,%a) d=(%a,%a,%a) th=%a t=%a\n", o.x, o.y, o.z, d.x, d.y, d.z,
                                 th, t);
                violations++;
            }
        }
        certified += cert;
        flat_cert += cert && fl;
    }
    std::printf("{\"hits\": %ld, \"certified\": %ld, \"flat_hits\": %ld, \"flat_certified\": %ld, "
                "\"exact_fail\": %ld, \"violations\": %ld}\n", hits, certified, flat_hits, flat_cert, exact_fail,
                violations);
    return violations ? 1 : 0;
}
