// pt_wide.cpp -- host builder of the 4-wide quantised tree of the global-memory walk
// (pt_wide.h).  Input: the reference's threaded binary tree (bvh.h:173-268
// builds it; computeShader.c:389-431 walks it), which must be nested (pt_bvh_culling_ok).
#include "pt_wide.h"

#include <algorithm>
#include <array>
#include <cmath>
#include <cstring>
#include <functional>

namespace ptw {
namespace {

// Record frontiers (wide_build): the surface-area-optimal cut of each record's binary subtree
// into at most 4 members.  Every leaf is a member of exactly one cut, so its cost term is the
// same for every choice of cuts: only the record visits, weighted by area, decide.
// (Measured against the round-4 greedy frontier -- the member of largest area expanded until
// four -- with the walk's other settings equal: +0.8% / +1.5% on the C3 / C4 stand-ins.)
constexpr double kCostRec = 1.0;

struct BN {
    float lo[3], hi[3];
    int left = -1, right = -1;
    bool leaf = false;
};

// Sign of (O + q 2^e) - b, exactly: q 2^e is exact in binary64 and TwoSum gives the rounding
// error of the sum, so the comparison with the binary32 b is exact (no overflow here).
int cmp_plane(float O, int q, int e, float b) {
    const double a = (double)O, c = std::ldexp((double)q, e);
    const double s = a + c, bb = s - a;
    const double err = (a - (s - bb)) + (c - bb);
    const double B = (double)b;
    if (s < B) return -1;
    if (s > B) return 1;
    return err < 0.0 ? -1 : (err > 0.0 ? 1 : 0);
}

// Smallest e in [-100, 100] with L + 255 * 2^e >= H (the codes of a record's axis then span
// its box).
int axis_exp(float L, float H) {
    const double ext = (double)H - (double)L;
    int e = -100;
    if (ext > 0.0) e = std::max(-100, (int)std::ceil(std::log2(ext / 255.0)));
    while (e < 100 && cmp_plane(L, 255, e, H) < 0) e++;
    while (e > -100 && cmp_plane(L, 255, e - 1, H) >= 0) e--;
    return e;
}

// Outward codes of the child interval [cl, ch] on an axis with origin L and step 2^e:
// the largest q with L + q 2^e <= cl, the smallest with L + q 2^e >= ch.
void codes(float L, int e, float cl, float ch, int& qlo, int& qhi) {
    const double st = std::ldexp(1.0, e);
    qlo = (int)std::floor(((double)cl - (double)L) / st);
    qlo = std::min(255, std::max(0, qlo));
    while (qlo > 0 && cmp_plane(L, qlo, e, cl) > 0) qlo--;
    while (qlo < 255 && cmp_plane(L, qlo + 1, e, cl) <= 0) qlo++;
    qhi = (int)std::ceil(((double)ch - (double)L) / st);
    qhi = std::min(255, std::max(0, qhi));
    while (qhi < 255 && cmp_plane(L, qhi, e, ch) < 0) qhi++;
    while (qhi > 0 && cmp_plane(L, qhi - 1, e, ch) >= 0) qhi--;
}

double area(const BN& b) {
    const double dx = (double)b.hi[0] - b.lo[0], dy = (double)b.hi[1] - b.lo[1], dz = (double)b.hi[2] - b.lo[2];
    return dx * dy + dy * dz + dz * dx;
}

int link_of(float v, int n) {
    if (!(v >= -1.0f && v < (float)n) || v != (float)(int)v) return -2;
    return (int)v;
}

float round_up_f(double v) {
    float f = (float)v;
    if ((double)f < v) f = std::nextafter(f, INFINITY);
    return f;
}

}  // namespace

int wide_build(const float* bvh, int n_nodes, const unsigned char* leaf_cop, WideTree& out) {
    out = WideTree();
    if (n_nodes <= 0) return -1;
    std::vector<BN> bn(n_nodes);
    for (int i = 0; i < n_nodes; i++) {
        const float* nd = bvh + 12 * (size_t)i;
        for (int q = 0; q < 3; q++) {
            bn[i].lo[q] = nd[q];
            bn[i].hi[q] = nd[4 + q];
            // finite, ordered boxes only (the quantisation steps and codes are computed from
            // them; the walk needs the scene half of the exact-reciprocal guard anyway)
            if (!std::isfinite(nd[q]) || !std::isfinite(nd[4 + q]) || !(nd[q] <= nd[4 + q])) return -1;
        }
        bn[i].leaf = nd[8] > -1.0f;
    }
    // children of the internal nodes reachable from the root (the threading of a nested tree:
    // hit link = left child, the left child's miss link = the right child)
    {
        std::vector<int> st{0};
        std::vector<unsigned char> seen(n_nodes, 0);
        while (!st.empty()) {
            const int x = st.back();
            st.pop_back();
            if (x < 0 || x >= n_nodes || seen[x]) return -1;
            seen[x] = 1;
            if (bn[x].leaf) continue;
            const int l = link_of(bvh[12 * (size_t)x + 10], n_nodes);
            if (l < 0) return -1;
            const int r = link_of(bvh[12 * (size_t)l + 11], n_nodes);
            if (r < 0) return -1;
            bn[x].left = l;
            bn[x].right = r;
            st.push_back(r);
            st.push_back(l);
        }
    }
    // F[y][k]: least cost of covering subtree y with at most k cut members (a member leaf
    // costs 0 here, see kCostRec; a member internal node costs area(y) * (kCostRec + its own
    // best cut's cost)), bottom-up; split[y][k] = how many of the k go left (0: y itself)
    std::vector<std::array<double, 5>> F(n_nodes, {0, 0, 0, 0, 0});
    std::vector<std::array<signed char, 5>> split(n_nodes, {0, 0, 0, 0, 0});
    {
        std::vector<int> order, st{0};
        while (!st.empty()) {               // preorder; reversed it is a valid bottom-up order
            const int x = st.back();
            st.pop_back();
            order.push_back(x);
            if (!bn[x].leaf) { st.push_back(bn[x].left); st.push_back(bn[x].right); }
        }
        for (auto it = order.rbegin(); it != order.rend(); ++it) {
            const int y = *it;
            if (bn[y].leaf) continue;
            const int l = bn[y].left, r = bn[y].right;
            double best = 1e300;                  // y as a record: its own best cut below
            for (int k1 = 1; k1 <= 3; k1++) best = std::min(best, F[l][k1] + F[r][4 - k1]);
            F[y][1] = (area(bn[y]) + 1e-30) * kCostRec + best;
            for (int k = 2; k <= 4; k++) {
                F[y][k] = F[y][k - 1];
                split[y][k] = split[y][k - 1];
                for (int k1 = 1; k1 < k; k1++) {
                    const double c = F[l][k1] + F[r][k - k1];
                    if (c < F[y][k]) { F[y][k] = c; split[y][k] = (signed char)k1; }
                }
            }
        }
    }
    // expands subtree y into at most k members, in preorder
    std::function<void(int, int, int*, int&)> expand = [&](int y, int k, int* f, int& n) {
        const int k1 = bn[y].leaf ? 0 : split[y][k];
        if (k1 == 0) { f[n++] = y; return; }
        expand(bn[y].left, k1, f, n);
        expand(bn[y].right, k - k1, f, n);
    };
    // a record's frontier: the best cut of its two children's subtrees (in preorder)
    auto frontier = [&](int x, int* f) {
        if (bn[x].leaf) { f[0] = x; return 1; }   // a root leaf: a record with that one child
        const int l = bn[x].left, r = bn[x].right;
        int bk = 1;
        double best = 1e300;
        for (int k1 = 1; k1 <= 3; k1++)
            if (F[l][k1] + F[r][4 - k1] < best) { best = F[l][k1] + F[r][4 - k1]; bk = k1; }
        int n = 0;
        expand(l, bk, f, n);
        expand(r, 4 - bk, f, n);
        return n;
    };
    // numbering: a record's children take consecutive indices (cbase + j).  Best-first: the
    // pending record of largest box area (the likeliest to be visited by an incoherent ray)
    // has its group allocated next, so the first indices -- the ones the kernel stages in LDS
    // -- hold the most visited records.  (Measured against breadth-first numbering: +0.3% on
    // the C3 / C4 stand-ins, 13% fewer global-memory record visits in the CPU model; numbering
    // each subtree below the LDS top depth-first or breadth-first inside it: within 0.3%.)
    out.g_of.assign(n_nodes, -1);
    std::vector<int> recs{0}, rdepth{0};          // binary node of each record, in discovery order
    std::vector<int> parent_g{-1}, parent_slot{0};
    std::vector<int> g_of_rec;                     // record (discovery index) -> g
    std::vector<std::array<int, 4>> kids(1);
    std::vector<int> nkids(1, 0);
    out.g_of[0] = 0;
    int next = 1;
    g_of_rec.push_back(0);
    bool overflow = false;
    // allocates record ri's child group; returns the discovery indices of its record children
    auto process = [&](size_t ri, std::vector<int>* found) {
        int f[4];
        const int n = frontier(recs[ri], f);
        std::array<int, 4> k = {-1, -1, -1, -1};
        for (int j = 0; j < n; j++) {
            k[j] = f[j];
            if (next >= kMaxRecords) { overflow = true; return; }
            out.g_of[f[j]] = next++;
            if (!bn[f[j]].leaf) {
                if (found) found->push_back((int)recs.size());
                recs.push_back(f[j]);
                rdepth.push_back(rdepth[ri] + 1);
                parent_g.push_back(g_of_rec[ri]);
                parent_slot.push_back(j);
                g_of_rec.push_back(out.g_of[f[j]]);
                kids.emplace_back();
                nkids.push_back(0);
            }
        }
        kids[ri] = k;
        nkids[ri] = n;
    };
    {
        std::vector<std::pair<double, int>> heap{{area(bn[recs[0]]), 0}};
        std::vector<int> found;
        while (!heap.empty() && !overflow) {
            std::pop_heap(heap.begin(), heap.end());
            const int ri = heap.back().second;
            heap.pop_back();
            found.clear();
            process((size_t)ri, &found);
            for (int c : found) {
                heap.emplace_back(area(bn[recs[c]]), c);
                std::push_heap(heap.begin(), heap.end());
            }
        }
    }
    if (overflow) return -1;
    out.n_index = next;
    out.bn_of.assign(next, -1);
    for (int i = 0; i < n_nodes; i++)
        if (out.g_of[i] >= 0) out.bn_of[out.g_of[i]] = i;
    out.bn_of[0] = 0;
    out.n_records = (int)recs.size();
    out.depth = 0;
    for (int d : rdepth) out.depth = std::max(out.depth, d + 1);
    out.rec.assign((size_t)next * 16, 0.0f);
    out.lbox.assign((size_t)next * 8, 0.0f);
    std::vector<int> exit_of(next, -1), pos_of(next, -1);
    for (size_t qi = 0; qi < recs.size(); qi++) pos_of[g_of_rec[qi]] = (int)qi;
    for (size_t qi = 0; qi < recs.size(); qi++) {
        const int x = recs[qi], g = g_of_rec[qi];
        const int n = nkids[qi];
        if (qi > 0) {   // resume the parent after this slot; after its last slot, the parent's exit
            const int pg = parent_g[qi], ps = parent_slot[qi];
            exit_of[g] = ps + 1 < nkids[pos_of[pg]] ? ((pg << 3) | (ps + 1)) : exit_of[pg];
        }
        float* r = &out.rec[(size_t)g * 16];
        int e[3];
        for (int i = 0; i < 3; i++) e[i] = axis_exp(bn[x].lo[i], bn[x].hi[i]);
        uint32_t lo_w[3] = {0, 0, 0}, hi_w[3] = {0, 0, 0}, types = 0;
        for (int j = 0; j < n; j++) {
            const BN& c = bn[kids[qi][j]];
            for (int i = 0; i < 3; i++) {
                int ql, qh;
                codes(bn[x].lo[i], e[i], c.lo[i], c.hi[i], ql, qh);
                lo_w[i] |= (uint32_t)ql << (8 * j);
                hi_w[i] |= (uint32_t)qh << (8 * j);
            }
            const uint32_t ty = c.leaf ? (2u | (leaf_cop && leaf_cop[kids[qi][j]] ? 1u : 0u)) : 1u;
            types |= ty << (2 * j);
        }
        const uint32_t w = ((uint32_t)(e[0] & 0xff)) | ((uint32_t)(e[1] & 0xff) << 8) |
                           ((uint32_t)(e[2] & 0xff) << 16) | (types << 24);
        const int cbase = out.g_of[kids[qi][0]];
        const uint32_t u[12] = {0, 0, 0, w, lo_w[0], hi_w[0], lo_w[1], hi_w[1], lo_w[2], hi_w[2],
                                (uint32_t)cbase, (uint32_t)exit_of[g]};
        std::memcpy(r, u, sizeof(u));
        r[0] = bn[x].lo[0];
        r[1] = bn[x].lo[1];
        r[2] = bn[x].lo[2];
        for (int j = 0; j < n; j++) {
            const int c = kids[qi][j];
            if (!bn[c].leaf) continue;
            float* b = &out.lbox[(size_t)out.g_of[c] * 8];
            b[0] = bn[c].lo[0]; b[1] = bn[c].hi[0]; b[2] = bn[c].lo[1]; b[3] = bn[c].hi[1];
            b[4] = bn[c].lo[2]; b[5] = bn[c].hi[2];
            out.n_leaves++;
        }
    }
    for (int q = 0; q < 3; q++) {
        const double m = std::max(std::fabs((double)bn[0].lo[q]), std::fabs((double)bn[0].hi[q]));
        out.cw[q] = round_up_f(std::ldexp(m, -18));
    }
    return 0;
}

}  // namespace ptw
