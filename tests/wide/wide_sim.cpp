// TEST INFRASTRUCTURE: CPU model of the wide global-memory walk (pt_wide.h) against the
// reference's binary walk (calculateRayCollision, computeShader.c:367-432; bvh_intersect
// :309-365; hit_triangle :274-307).  It runs the SAME per-lane functions the kernel runs
// (ptw::wide_hits / wide_visit / wide_pop) on the host and, for every ray segment of a set of
// diffuse paths and of adversarial rays, checks that
//   (1) the wide walk ends with the reference walk's t (bitwise) and triangle,
//   (2) every record child whose exact box test passes at the visit's t is accepted by the
//       conservative test (the superset property the argument of pt_wide.h rests on),
// and reports the work per segment of both walks.
//
// usage: wide_sim scene.bin [stride] [bounces] [adversarial_rays]
//   scene.bin: int32 n_tris, n_nodes, n_spheres, then float32 tris (16 per), nodes (12 per),
//   spheres (8 per), camera (12: pos, dir, 0...) -- written by tests/test_wide_walk.py.
// Exit status 0 = no mismatch.  Output: one JSON line of statistics.
#include "../../opengl-path-tracing_amd/csrc/pt_wide.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using pt::f3;
using pt::mk;

namespace {

std::vector<float> tris, nodes, sph;
int nt = 0, nn = 0, ns = 0;
float cam[12];

// computeShader.c:309-365 in IEEE division (the reference's exact test)
bool slab_exact(const float* lo, const float* hi, f3 o, f3 d, float cur_t) {
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
bool node_exact(int i, f3 o, f3 d, float t) {
    const float* b = &nodes[12 * (size_t)i];
    return slab_exact(b, b + 4, o, d, t);
}

f3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }

// :274-307
float hit_triangle(f3 o, f3 d, int ti) {
    const float* tr = &tris[16 * (size_t)ti];
    const f3 v0 = ld3(tr), v1 = ld3(tr + 4), v2 = ld3(tr + 8);
    const f3 n = pt::normalize(pt::cross(v1 - v0, v2 - v0));
    const float dd = -pt::dot(n, v0);
    const float t = -(pt::dot(n, o) + dd) / pt::dot(n, d);
    if (t < 0.0f) return -1.0f;
    const f3 p = o + d * t;
    if (pt::dot(n, pt::cross(v1 - v0, p - v0)) > 0.0f && pt::dot(n, pt::cross(v2 - v1, p - v1)) > 0.0f &&
        pt::dot(n, pt::cross(v0 - v2, p - v2)) > 0.0f)
        return t;
    return -1.0f;
}

float sphere_t(f3 o, f3 d) {   // :372-385 (the closest sphere hit in (1e-4, inf), else inf)
    float t = INFINITY;
    for (int si = 0; si < ns; si++) {
        const float* s = &sph[8 * (size_t)si];
        const f3 oc = o - ld3(s);
        const float a = pt::dot(d, d), hb = pt::dot(oc, d), c = pt::dot(oc, oc) - s[3] * s[3];
        const float disc = hb * hb - a * c;
        const float ht = disc < 0.0f ? -1.0f : (-hb - std::sqrt(disc)) / a;
        if (ht > 0.0001f && ht < t) t = ht;
    }
    return t;
}

struct Leaf { float t; int tri; };
// the leaf's 2-way choice (:411-428) at t; returns whether t moves
bool leaf_choice(int bnode, f3 o, f3 d, float t, float& nt_, int& ntri) {
    const float* b = &nodes[12 * (size_t)bnode];
    const int t0 = (int)b[8], t1 = (int)b[9];
    const float h1 = hit_triangle(o, d, t0), h2 = hit_triangle(o, d, t1);
    if (h1 > 0.0001f && h1 < t && (h1 < h2 || h2 < 0.0001f)) { nt_ = h1; ntri = t0; return true; }
    if (h2 > 0.0001f && h2 < t) { nt_ = h2; ntri = t1; return true; }
    return false;
}

struct RefOut { float t; int tri; long visits, leaves, top; };
std::vector<unsigned char> ref_top_set;   // the binary walk's LDS top nodes (768 breadth-first)
RefOut ref_walk(f3 o, f3 d, float t0) {
    RefOut r{t0, -1, 0, 0, 0};
    for (int bi = 0; bi > -1;) {
        const float* b = &nodes[12 * (size_t)bi];
        const bool hb = node_exact(bi, o, d, r.t);
        r.visits++;
        if (ref_top_set[bi]) r.top++;
        const int next = hb ? (int)b[10] : (int)b[11];
        if (hb && b[8] > -1.0f) {
            r.leaves++;
            float t2;
            int tri;
            if (leaf_choice(bi, o, d, r.t, t2, tri)) { r.t = t2; r.tri = tri; }
        }
        bi = next;
    }
    return r;
}

ptw::WideTree W;
long cons_violations = 0;
struct WideOut { float t; int tri; long visits, resumes, leaves, retests, retest_fail, pops, top_visits, lines, certified; };
long cert_violations = 0;

// the exact-reciprocal guard, ray half
bool in_guard(f3 o, f3 d) {
    auto g0 = [](float v) { float a = std::fabs(v); return v == 0.0f || (a >= 0x1p-40f && a <= 0x1p60f); };
    auto g1 = [](float v) { float a = std::fabs(v); return a >= 0x1p-20f && a <= 2.0f; };
    return g0(o.x) && g0(o.y) && g0(o.z) && g1(d.x) && g1(d.y) && g1(d.z);
}

int top_records = 512;   // indices below this are staged in LDS by the kernel

WideOut wide_walk(f3 o, f3 d, float t0) {
    WideOut r{t0, -1, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    const f3 rd = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    const ptw::WRay wr = ptw::make_wray(o, rd, W.cw, std::signbit(d.x), std::signbit(d.y), std::signbit(d.z));
    int cur = 0, R = -1;
#ifndef STACK_K
#define STACK_K ptw::kStack   // the kernel's depth (pt_wide.h)
#endif
    uint32_t e[STACK_K] = {};
    long last_line = -1;
    for (;;) {
        if (cur >= 0) {
            const int N = cur >> 3, s = cur & 7;
            uint32_t u[16];
            std::memcpy(u, &W.rec[(size_t)N * 16], 64);
            float O[3];
            std::memcpy(O, u, 12);
            const uint32_t pend = ptw::wide_hits(O[0], O[1], O[2], u[3], u[4], u[5], u[6], u[7], u[8], u[9], wr, r.t, s);
            // superset check against the exact tests of the children's own boxes
            const uint32_t types = u[3] >> 24;
            for (int j = s; j < 4; j++) {
                if (!((types >> (2 * j)) & 3u)) continue;
                const int bnode = W.bn_of[(int)u[10] + j];
                if (node_exact(bnode, o, d, r.t) && !((pend >> (2 * j)) & 3u)) cons_violations++;
            }
            r.visits++;
            if (s) r.resumes++;
            if (N < top_records) r.top_visits++;
            else if (N / 2 != last_line) { r.lines++; last_line = N / 2; }
            cur = ptw::wide_visit<STACK_K>(cur, pend, (int)u[10], (int)u[11], e, R);
            continue;
        }
        if (cur == -1) break;
        const int code = -2 - cur, g = code >> 1;
        r.leaves++;
        float t2;
        int tri;
        if (leaf_choice(W.bn_of[g], o, d, r.t, t2, tri)) {
            r.retests++;
            const float* lb = &W.lbox[(size_t)g * 8];
            const float lo[3] = {lb[0], lb[2], lb[4]}, hi[3] = {lb[1], lb[3], lb[5]};
            const bool exact = slab_exact(lo, hi, o, d, r.t);
            const float* tr = &tris[16 * (size_t)tri];
            const f3 p = o + d * t2;
            const f3 v0 = ld3(tr), v1 = ld3(tr + 4), v2 = ld3(tr + 8);
            const f3 n = pt::normalize(pt::cross(v1 - v0, v2 - v0));
            if (ptw::leaf_certificate(p, n, v0, v1, v2, ptw::abs_max3(o))) {
                r.certified++;
                if (!exact) cert_violations++;
            }
            if (exact) { r.t = t2; r.tri = tri; }
            else r.retest_fail++;
        }
        r.pops++;
        cur = ptw::wide_pop<STACK_K>(e, R);
    }
    return r;
}

struct Acc { double segs = 0, rv = 0, rl = 0, wv = 0, wr = 0, wl = 0, wt = 0, wf = 0, top = 0, lines = 0, ref_top = 0, wc = 0; };

long mismatches = 0, slow = 0;
void segment(f3 o, f3 d, Acc& A, float* t_out, int* tri_out) {
    const float t0 = sphere_t(o, d);
    const RefOut ro = ref_walk(o, d, t0);
    *t_out = ro.t;
    *tri_out = ro.tri;
    A.segs++;
    A.rv += ro.visits;
    A.rl += ro.leaves;
    A.ref_top += ro.top;
    if (!in_guard(o, d)) { slow++; return; }
    const WideOut wo = wide_walk(o, d, t0);
    uint32_t a, b;
    std::memcpy(&a, &ro.t, 4);
    std::memcpy(&b, &wo.t, 4);
    if (a != b || ro.tri != wo.tri) {
        if (mismatches < 10)
            std::fprintf(stderr, "MISMATCH o=(%a,%a,%a) d=(%a,%a,%a): ref t=%a tri=%d, wide t=%a tri=%d\n", o.x, o.y, o.z,
                         d.x, d.y, d.z, ro.t, ro.tri, wo.t, wo.tri);
        mismatches++;
    }
    A.wv += wo.visits;
    A.wr += wo.resumes;
    A.wl += wo.leaves;
    A.wt += wo.retests;
    A.wf += wo.retest_fail;
    A.top += wo.top_visits;
    A.lines += wo.lines;
    A.wc += wo.certified;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) { std::fprintf(stderr, "usage: wide_sim scene.bin [stride] [bounces] [adversarial]\n"); return 2; }
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) return 2;
    int hdr[3];
    if (std::fread(hdr, 4, 3, f) != 3) return 2;
    nt = hdr[0]; nn = hdr[1]; ns = hdr[2];
    tris.resize(16 * (size_t)nt); nodes.resize(12 * (size_t)nn); sph.resize(8 * (size_t)ns);
    if (std::fread(tris.data(), 4, tris.size(), f) != tris.size() || std::fread(nodes.data(), 4, nodes.size(), f) != nodes.size() ||
        std::fread(sph.data(), 4, sph.size(), f) != sph.size() || std::fread(cam, 4, 12, f) != 12)
        return 2;
    std::fclose(f);
    const int stride = argc > 2 ? std::atoi(argv[2]) : 16;
    const int bounces = argc > 3 ? std::atoi(argv[3]) : 8;
    const long adversarial = argc > 4 ? std::atol(argv[4]) : 0;
    if (argc > 5) top_records = std::atoi(argv[5]);
    // the leaf flags of pt_upload_scene: both triangles' (n, d0) equal
    std::vector<unsigned char> cop(nn, 0);
    for (int i = 0; i < nn; i++) {
        const float* b = &nodes[12 * (size_t)i];
        if (!(b[8] > -1.0f)) continue;
        float nd[2][4];
        for (int k = 0; k < 2; k++) {
            const float* tr = &tris[16 * (size_t)(int)b[8 + k]];
            const f3 v0 = ld3(tr), v1 = ld3(tr + 4), v2 = ld3(tr + 8);
            const f3 n = pt::normalize(pt::cross(v1 - v0, v2 - v0));
            nd[k][0] = n.x; nd[k][1] = n.y; nd[k][2] = n.z; nd[k][3] = -pt::dot(n, v0);
        }
        cop[i] = nd[0][0] == nd[1][0] && nd[0][1] == nd[1][1] && nd[0][2] == nd[1][2] && nd[0][3] == nd[1][3];
    }
    {   // pt_upload_scene's breadth-first top numbering (kTopNodes = 768)
        ref_top_set.assign(nn, 0);
        std::vector<int> q{0};
        ref_top_set[0] = 1;
        int cnt = 1;
        for (size_t qi = 0; qi < q.size() && cnt < 768; qi++)
            for (int l = 10; l < 12; l++) {
                const int t = (int)nodes[12 * (size_t)q[qi] + l];
                if (t >= 0 && !ref_top_set[t] && cnt < 768) { ref_top_set[t] = 1; cnt++; q.push_back(t); }
            }
    }
    if (ptw::wide_build(nodes.data(), nn, cop.data(), W) != 0) {
        std::printf("{\"built\": false}\n");
        return 3;
    }
    // camera basis (computeShader.c:517-522), 1920x1080 grid sampled every `stride` pixels
    const int Wd = 1920, Hd = 1080;
    const f3 pos = mk(cam[0], cam[1], cam[2]);
    const f3 fwd = pt::normalize(mk(cam[4], cam[5], cam[6]));
    const f3 right = pt::normalize(pt::cross(fwd, mk(0, 0, 1)));
    const f3 up = (pt::normalize(pt::cross(right, fwd)) * (float)Hd) / (float)Wd;
    Acc A;
    for (int y = 0; y < Hd; y += stride)
        for (int x = 0; x < Wd; x += stride) {
            uint32_t st = pt::seed(x, y, 1);
            const float u = ((float)x + pt::random01(st)) / (float)Wd - 0.5f;
            const float v = ((float)y + pt::random01(st)) / (float)Hd - 0.5f;
            f3 o = pos, d = pt::normalize((fwd + right * u) + up * v);
            for (int bnc = 0; bnc <= bounces; bnc++) {
                float t;
                int tri;
                segment(o, d, A, &t, &tri);
                if (tri < 0) break;   // (a sphere hit ends the path here: the model follows triangles)
                const float* tr = &tris[16 * (size_t)tri];
                const f3 v0 = ld3(tr), v1 = ld3(tr + 4), v2 = ld3(tr + 8);
                f3 n = pt::normalize(pt::cross(v1 - v0, v2 - v0));
                if (pt::dot(n, d) > 0.0f) n = n * -1.0f;
                o = o + d * t;
                d = pt::normalize(n + pt::random_unit_vector(st));
            }
        }
    const double path_segs = A.segs;
    // adversarial rays: origins on box planes / corners of random nodes, directions toward
    // other nodes' corners, random and near-axis directions
    uint32_t st = 12345u;
    for (long k = 0; k < adversarial; k++) {
        const float* a = &nodes[12 * (size_t)(pt::next_random(st) % (uint32_t)nn)];
        const float* b = &nodes[12 * (size_t)(pt::next_random(st) % (uint32_t)nn)];
        auto pick = [&](const float* nd, int q) {
            const uint32_t r = pt::next_random(st) % 4u;
            if (r == 0) return nd[q];
            if (r == 1) return nd[4 + q];
            return nd[q] + (nd[4 + q] - nd[q]) * pt::random01(st);
        };
        f3 o = mk(pick(a, 0), pick(a, 1), pick(a, 2));
        f3 tg = mk(pick(b, 0), pick(b, 1), pick(b, 2));
        f3 d = tg - o;
        if (pt::next_random(st) % 8u == 0) d = pt::random_unit_vector(st);
        if (pt::dot(d, d) == 0.0f) continue;
        if (pt::next_random(st) % 16u == 0) d.x = d.x * 1e-3f;
        d = pt::normalize(d);
        float t;
        int tri;
        segment(o, d, A, &t, &tri);
    }
    const double s = A.segs - slow;
    std::printf("{\"n_tris\": %d, \"n_nodes\": %d, \"records\": %d, \"index\": %d, \"depth\": %d, \"segments\": %.0f, "
                "\"path_segments\": %.0f, \"slow\": %ld, \"mismatches\": %ld, \"cons_violations\": %ld, "
                "\"ref_visits\": %.3f, \"ref_leaves\": %.3f, \"ref_top\": %.3f, \"wide_visits\": %.3f, \"wide_resumes\": %.3f, "
                "\"wide_leaves\": %.3f, \"wide_retests\": %.3f, \"wide_retest_fail\": %.4f, \"wide_top\": %.3f, "
                "\"wide_lines\": %.3f, \"wide_certified\": %.4f, \"cert_violations\": %ld}\n",
                nt, nn, W.n_records, W.n_index, W.depth, A.segs, path_segs, slow, mismatches, cons_violations,
                A.rv / A.segs, A.rl / A.segs, A.ref_top / A.segs, A.wv / s, A.wr / s, A.wl / s, A.wt / s, A.wf / s, A.top / s, A.lines / s, A.wc / s, cert_violations);
    return (mismatches || cons_violations || cert_violations) ? 1 : 0;
}
