// pt_bvh_gpu.hip -- the reference's SAH BVH builder (bvh.h:173-268) on the GPU
// ("optional GPU build").  Output identical to pt_bvh_build
// (pt_scene.cpp), which is itself checked node for node against the oracle's literal
// restatement of buildSAHTree.
//
// The host builder recurses node by node; here every node of one tree level is split at
// once:
//   * the chained stable centroid sorts of find_split (x, then y on the x order, then z on
//     the y order; bvh.h:185-189) are three stable radix sorts over all positions, keyed by
//     (node rank, centroid sum mapped to an order-preserving integer with -0 == +0 like the
//     comparator), so every node of the level is sorted within its own range at once;
//   * the prefix / suffix boxes behind each candidate's surface areas are segmented
//     inclusive scans (forward, and over the reversed arrays) with the host's exact union:
//     keep the left operand unless the right one is strictly smaller (larger), which is
//     associative, so the scans give the host loop's bits, signed zeros included;
//   * the <= 60 candidates per axis and the strict-< first minimum (bvh.h:191-214) are one
//     thread per node, in double, with the host's operation order (-ffp-contract=off).
// The host keeps the level bookkeeping (which children are leaves, the level's segment
// table) and at the end numbers the nodes as the reference allocates them -- a node's two
// children get the next two indices when the node is processed, left subtree first
// (bvh.h:243-246) -- and threads the hit / miss links (bvh.h:84-98).
#include "../../include/pt_scene.h"
#include "../../include/pt_api.h"

#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <limits>
#include <string>
#include <thread>
#include <vector>

namespace pt_internal {
// pt_scene.cpp: index of the first triangle equal (all 16 floats, -0 == +0) to each one,
// the leaf index of buildSAHTreeHelper's std::find (bvh.h:231-232); fails on non-finite data.
int first_equal_indices(const float* tris, int n, std::vector<int>& out, std::string& err);
// pt_scene.cpp: the builders' last error (pt_bvh_last_error).
void set_bvh_error(const std::string& msg);
}

namespace {

struct GBox {
    float mn[3], mx[3];
};

// The host builder's grow(): a coordinate is replaced only by a strictly smaller (larger)
// one, so the kept value is the first extreme in sequence order.
struct BoxUnion {
    __host__ __device__ GBox operator()(const GBox& a, const GBox& b) const {
        GBox r;
        for (int k = 0; k < 3; k++) {
            r.mn[k] = b.mn[k] < a.mn[k] ? b.mn[k] : a.mn[k];
            r.mx[k] = b.mx[k] > a.mx[k] ? b.mx[k] : a.mx[k];
        }
        return r;
    }
};

// bvh.h:21-27 as in pt_scene.cpp: float extents promoted to double.
__device__ __forceinline__ double area(const GBox& b) {
    double x = (float)(b.mx[0] - b.mn[0]);
    double y = (float)(b.mx[1] - b.mn[1]);
    double z = (float)(b.mx[2] - b.mn[2]);
    return 2.0 * (x * y + y * z + x * z);
}

__global__ void k_prep(const float* __restrict__ T, int n, GBox* __restrict__ box, unsigned* __restrict__ key) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float* t = T + 16 * (size_t)i;
    GBox b;
    const float inf = __builtin_huge_valf();
    for (int a = 0; a < 3; a++) { b.mn[a] = inf; b.mx[a] = -inf; }
    for (int v = 0; v < 3; v++)
        for (int a = 0; a < 3; a++) {
            const float c = t[4 * v + a];
            if (c < b.mn[a]) b.mn[a] = c;
            if (c > b.mx[a]) b.mx[a] = c;
        }
    box[i] = b;
    for (int a = 0; a < 3; a++) {
        float c = (t[a] + t[4 + a]) + t[8 + a];    // the centroid sum the comparator orders
        c = c + 0.0f;                               // -0 -> +0: the comparator's ties
        const unsigned u = __float_as_uint(c);
        key[(size_t)a * n + i] = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    }
}

// Sort keys of one axis pass: (position-ordered segment rank) << 32 | centroid key.  Active
// node j's positions get rank 2j + 1, the finished positions after it 2j + 2, so one stable
// radix sort over all positions sorts every active node's range in place and leaves the
// ranges where they are (finished ranges are reordered inside themselves, and never read).
__global__ void k_gather_keys(const int* __restrict__ vals, const unsigned* __restrict__ key,
                              const int* __restrict__ seg, int n, unsigned long long* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = ((unsigned long long)(unsigned)seg[i] << 32) | key[vals[i]];
}

// Window-relative (position off + i): the active node of the position (-1 / -2 outside
// them, alternating so that no two outside positions form one scan run) and its sort rank.
__global__ void k_seg_of(const int* __restrict__ beg, const int* __restrict__ end, int k, int off, int len,
                         int* __restrict__ seg, int* __restrict__ rank) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= len) return;
    const int p = off + i;
    int lo = 0, hi = k - 1, s = -1;
    while (lo <= hi) {
        const int mid = (lo + hi) >> 1;
        if (beg[mid] <= p) { s = mid; lo = mid + 1; } else hi = mid - 1;
    }
    const bool in = s >= 0 && p < end[s];
    seg[i] = in ? s : -1 - (i & 1);
    rank[i] = in ? 2 * s + 1 : 2 * s + 2;
}

// Boxes in a given order, forward and reversed, with the reversed segment keys.
__global__ void k_boxes(const int* __restrict__ ord, const GBox* __restrict__ box, const int* __restrict__ seg, int n,
                        GBox* __restrict__ fwd, GBox* __restrict__ rev, int* __restrict__ rseg) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const GBox b = box[ord[i]];
    fwd[i] = b;
    rev[n - 1 - i] = b;
    rseg[n - 1 - i] = seg[i];
}

// find_split (bvh.h:173-218) for one node per thread: SA of the node box (its own order),
// the candidates split = 1, 1+s, ... (s = m/60 + 1) per axis, the first strict minimum.
// out: {axis (0..2, 3 = no finite cost), split} per node; nbox: the node's bounds.
__global__ void k_decide(const int* __restrict__ beg, const int* __restrict__ end, int k, int off, int len,
                         const GBox* __restrict__ own, const GBox* __restrict__ pre0, const GBox* __restrict__ pre1,
                         const GBox* __restrict__ pre2, const GBox* __restrict__ rsuf0,
                         const GBox* __restrict__ rsuf1, const GBox* __restrict__ rsuf2, int2* __restrict__ out,
                         GBox* __restrict__ nbox) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= k) return;
    const int st = beg[j] - off, m = end[j] - beg[j];      // window-relative start
    const GBox ov = own[st + m - 1];
    nbox[j] = ov;
    const double SA = area(ov);
    double best = __builtin_huge_val();
    int best_axis = 3, best_split = m / 2;
    const GBox* pre[3] = {pre0, pre1, pre2};
    const GBox* suf[3] = {rsuf0, rsuf1, rsuf2};
    const int step = m / 60 + 1;
    for (int a = 0; a < 3; a++) {
        for (int s = 1; s < m; s += step) {
            const double SA1 = area(pre[a][st + s - 1]);
            const double SA2 = area(suf[a][len - 1 - (st + s)]);   // reversed-scan index
            const double cost = 1.0 + (SA1 / SA) * s * 1.0 + (SA2 / SA) * (double)(m - s) * 1.0;
            if (cost < best) { best = cost; best_axis = a; best_split = s; }
        }
    }
    out[j] = make_int2(best_axis, best_split);
}

// The chosen order becomes each split node's element order (its children's sequences).
__global__ void k_apply(const int* __restrict__ seg, const int2* __restrict__ dec, const int* __restrict__ o0,
                        const int* __restrict__ o1, const int* __restrict__ o2, int len, int* __restrict__ cur) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;   // o0..o2, cur: window base
    if (i >= len) return;
    const int s = seg[i];
    if (s < 0) return;
    const int a = dec[s].x;
    cur[i] = a == 0 ? o0[i] : (a == 1 ? o1[i] : o2[i]);   // axis 3 (degenerate): the z order
}

// The node table, indexed by creation id: each split node j of the level gets children
// base + 2j, base + 2j + 1.  A child of at most 2 triangles is a leaf: its bounds over its
// elements in order and its first / last triangle (buildSAHTreeHelper :224-237).
struct DNode {
    GBox b;
    int left, right;   // children (creation ids), -1 at a leaf
    int t0, t1;        // leaf triangles (input indices, before the first-equal mapping)
};

__device__ __forceinline__ void make_leaf(DNode& d, const int* cur, const GBox* box, int st, int m) {
    GBox b = box[cur[st]];
    for (int q = 1; q < m; q++) b = BoxUnion()(b, box[cur[st + q]]);
    d.b = b;
    d.left = d.right = -1;
    d.t0 = cur[st];
    d.t1 = cur[st + m - 1];
}

__global__ void k_root_leaf(const int* __restrict__ cur, const GBox* __restrict__ box, int n, DNode* __restrict__ nodes) {
    if (blockIdx.x == 0 && threadIdx.x == 0) make_leaf(nodes[0], cur, box, 0, n);
}

__global__ void k_children(const int* __restrict__ beg, const int* __restrict__ end, const int* __restrict__ id, int k,
                           int base, const int2* __restrict__ dec, const GBox* __restrict__ nbox,
                           const int* __restrict__ cur, const GBox* __restrict__ box, DNode* __restrict__ nodes) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= k) return;
    const int st = beg[j], m = end[j] - st, s = dec[j].y;
    const int l = base + 2 * j, r = l + 1;
    DNode& d = nodes[id[j]];
    d.b = nbox[j];
    d.left = l;
    d.right = r;
    d.t0 = d.t1 = -1;
    if (s <= 2) make_leaf(nodes[l], cur, box, st, s);
    if (m - s <= 2) make_leaf(nodes[r], cur, box, st + s, m - s);
}

struct Seg {
    int start, size, node;
};

template <typename T>
struct DBuf {
    T* p = nullptr;
    size_t n = 0;
    hipError_t alloc(size_t count) {
        if (count <= n) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        hipError_t e = hipMalloc(&p, std::max<size_t>(count, 1) * sizeof(T));
        if (e == hipSuccess) n = count;
        return e;
    }
    ~DBuf() { if (p) (void)hipFree(p); }
};

thread_local std::string g_err;   // this builder's message, handed to pt_bvh_last_error

#define GCHK(call)                                                      \
    do {                                                                \
        hipError_t e_ = (call);                                         \
        if (e_ != hipSuccess) {                                         \
            g_err = std::string(#call) + ": " + hipGetErrorString(e_);  \
            return PT_E_HIP;                                            \
        }                                                               \
    } while (0)

inline unsigned blocks_for(long long n) { return (unsigned)((n + 255) / 256); }

int build(const float* T, int n, int device, std::vector<DNode>& nodes) {
    int prev_device = 0;
    GCHK(hipGetDevice(&prev_device));
    struct DeviceGuard { int d; ~DeviceGuard() { (void)hipSetDevice(d); } } dg{prev_device};   // the caller's device back
    GCHK(hipSetDevice(device));
    hipStream_t sm;
    GCHK(hipStreamCreateWithFlags(&sm, hipStreamNonBlocking));
    struct StreamGuard { hipStream_t s; ~StreamGuard() { (void)hipStreamDestroy(s); } } sg{sm};

    // every buffer at its largest size up front (a reallocation mid-build drains the device)
    const int kmax = n / 3 + 2, nn_max = 2 * n;
    DBuf<float> d_tris;
    DBuf<GBox> d_box, d_fwd[3], d_rev, d_pre[3], d_rsuf[3], d_own, d_nbox;
    DBuf<unsigned> d_key;
    DBuf<unsigned long long> d_kin, d_kout;
    DBuf<int> d_cur, d_ord[3], d_seg, d_rseg, d_rank, d_lvl;
    DBuf<int2> d_dec;
    DBuf<DNode> d_nodes;
    DBuf<char> d_tmp;
    GCHK(d_tris.alloc(16 * (size_t)n));
    GCHK(d_box.alloc(n));
    GCHK(d_key.alloc(3 * (size_t)n));
    GCHK(d_kin.alloc(n));
    GCHK(d_kout.alloc(n));
    GCHK(d_cur.alloc(n));
    GCHK(d_seg.alloc(n));
    GCHK(d_rseg.alloc(n));
    GCHK(d_rank.alloc(n));
    GCHK(d_rev.alloc(n));
    GCHK(d_own.alloc(n));
    for (int a = 0; a < 3; a++) {
        GCHK(d_ord[a].alloc(n));
        GCHK(d_fwd[a].alloc(n));
        GCHK(d_pre[a].alloc(n));
        GCHK(d_rsuf[a].alloc(n));
    }
    GCHK(d_lvl.alloc(3 * (size_t)kmax));     // per active node: start, end, creation id
    GCHK(d_dec.alloc(kmax));
    GCHK(d_nbox.alloc(kmax));
    GCHK(d_nodes.alloc(nn_max));
    {
        size_t b1 = 0, b2 = 0;
        GCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, b1, d_kin.p, d_kout.p, d_cur.p, d_ord[0].p, n, 0, 64, sm));
        GCHK(hipcub::DeviceScan::InclusiveScanByKey(nullptr, b2, d_seg.p, d_fwd[0].p, d_pre[0].p, BoxUnion(), n,
                                                    hipcub::Equality(), sm));
        GCHK(d_tmp.alloc(std::max(b1, b2)));
    }
    const bool prof = getenv("PT_BVH_PROFILE") != nullptr;   // per-level timing on stderr
    GCHK(hipMemcpyAsync(d_tris.p, T, 16 * (size_t)n * sizeof(float), hipMemcpyHostToDevice, sm));
    hipLaunchKernelGGL(k_prep, dim3(blocks_for(n)), dim3(256), 0, sm, d_tris.p, n, d_box.p, d_key.p);
    {
        std::vector<int> ident(n);
        for (int i = 0; i < n; i++) ident[i] = i;
        GCHK(hipMemcpyAsync(d_cur.p, ident.data(), (size_t)n * sizeof(int), hipMemcpyHostToDevice, sm));
    }

    int n_nodes = 1;
    std::vector<Seg> active;
    if (n >= 3) active.push_back({0, n, 0});
    else hipLaunchKernelGGL(k_root_leaf, dim3(1), dim3(64), 0, sm, d_cur.p, d_box.p, n, d_nodes.p);

    int level = 0;
    auto t_level = std::chrono::steady_clock::now();
    std::vector<int> hlvl;
    std::vector<int2> hdec;
    while (!active.empty()) {
        const int k = (int)active.size();
        hlvl.resize(3 * (size_t)k);
        for (int j = 0; j < k; j++) {
            hlvl[j] = active[j].start;
            hlvl[k + j] = active[j].start + active[j].size;
            hlvl[2 * k + j] = active[j].node;
        }
        const int* d_beg = d_lvl.p;
        const int* d_end = d_lvl.p + k;
        const int* d_id = d_lvl.p + 2 * k;
        GCHK(hipMemcpyAsync(d_lvl.p, hlvl.data(), 3 * (size_t)k * sizeof(int), hipMemcpyHostToDevice, sm));
        // only the window spanned by the level's active nodes is processed
        const int off = hlvl[0], len = hlvl[2 * k - 1] - hlvl[0];
        hipLaunchKernelGGL(k_seg_of, dim3(blocks_for(len)), dim3(256), 0, sm, d_beg, d_end, k, off, len, d_seg.p,
                           d_rank.p);
        int rank_bits = 1;
        while ((1ll << rank_bits) <= 2ll * k + 2) rank_bits++;
        // the three chained stable sorts (bvh.h:185-189): x on the node order, y on the x
        // order, z on the y order
        const int* src = d_cur.p + off;
        for (int a = 0; a < 3; a++) {
            hipLaunchKernelGGL(k_gather_keys, dim3(blocks_for(len)), dim3(256), 0, sm, src, d_key.p + (size_t)a * n,
                               d_rank.p, len, d_kin.p);
            size_t bytes = d_tmp.n;
            GCHK(hipcub::DeviceRadixSort::SortPairs(d_tmp.p, bytes, d_kin.p, d_kout.p, src, d_ord[a].p + off, len, 0,
                                                    32 + rank_bits, sm));
            src = d_ord[a].p + off;
        }
        // prefix boxes in each axis order, suffix boxes by scanning the reversed arrays, and
        // the node boxes in the nodes' own order
        for (int a = 0; a < 4; a++) {
            const int* ord = (a < 3 ? d_ord[a].p : d_cur.p) + off;
            GBox* fwd = a < 3 ? d_fwd[a].p : d_fwd[0].p;
            hipLaunchKernelGGL(k_boxes, dim3(blocks_for(len)), dim3(256), 0, sm, ord, d_box.p, d_seg.p, len, fwd,
                               d_rev.p, d_rseg.p);
            GBox* pre = a < 3 ? d_pre[a].p : d_own.p;
            size_t bytes = d_tmp.n;
            GCHK(hipcub::DeviceScan::InclusiveScanByKey(d_tmp.p, bytes, d_seg.p, fwd, pre, BoxUnion(), len,
                                                        hipcub::Equality(), sm));
            if (a < 3) {
                bytes = d_tmp.n;
                GCHK(hipcub::DeviceScan::InclusiveScanByKey(d_tmp.p, bytes, d_rseg.p, d_rev.p, d_rsuf[a].p, BoxUnion(),
                                                            len, hipcub::Equality(), sm));
            }
        }
        hipLaunchKernelGGL(k_decide, dim3(blocks_for(k)), dim3(256), 0, sm, d_beg, d_end, k, off, len, d_own.p,
                           d_pre[0].p, d_pre[1].p, d_pre[2].p, d_rsuf[0].p, d_rsuf[1].p, d_rsuf[2].p, d_dec.p,
                           d_nbox.p);
        hipLaunchKernelGGL(k_apply, dim3(blocks_for(len)), dim3(256), 0, sm, d_seg.p, d_dec.p, d_ord[0].p + off,
                           d_ord[1].p + off, d_ord[2].p + off, len, d_cur.p + off);
        hipLaunchKernelGGL(k_children, dim3(blocks_for(k)), dim3(256), 0, sm, d_beg, d_end, d_id, k, n_nodes, d_dec.p,
                           d_nbox.p, d_cur.p, d_box.p, d_nodes.p);
        hdec.resize(k);
        GCHK(hipMemcpyAsync(hdec.data(), d_dec.p, k * sizeof(int2), hipMemcpyDeviceToHost, sm));
        GCHK(hipStreamSynchronize(sm));
        std::vector<Seg> next;
        next.reserve(2 * (size_t)k);
        for (int j = 0; j < k; j++) {
            const Seg& g = active[j];
            const int s = hdec[j].y, l = n_nodes + 2 * j;
            if (s >= 3) next.push_back({g.start, s, l});
            if (g.size - s >= 3) next.push_back({g.start + s, g.size - s, l + 1});
        }
        n_nodes += 2 * k;
        if (prof) {
            const auto t1 = std::chrono::steady_clock::now();
            std::fprintf(stderr, "level %d: %d active nodes, window %d, %.3f ms\n", level, k, len,
                         std::chrono::duration<double>(t1 - t_level).count() * 1e3);
            t_level = t1;
        }
        level++;
        active.swap(next);
    }
    nodes.resize(n_nodes);
    GCHK(hipMemcpyAsync(nodes.data(), d_nodes.p, (size_t)n_nodes * sizeof(DNode), hipMemcpyDeviceToHost, sm));
    GCHK(hipStreamSynchronize(sm));
    return PT_OK;
}

}  // namespace

extern "C" int pt_bvh_build_gpu(const float* tris, int n_tris, float* nodes_out, int max_nodes, int* n_nodes,
                                int device) {
    auto fail = [](int code, const std::string& msg) { pt_internal::set_bvh_error(msg); return code; };
    if (!tris || n_tris <= 0 || !n_nodes) return fail(PT_E_ARG, "empty triangle list");
    if (n_tris > (1 << 23)) return fail(PT_E_SCENE, "more than 2^23 triangles (float index limit)");
    const bool prof = getenv("PT_BVH_PROFILE") != nullptr;
    auto t0 = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
        if (!prof) return;
        const auto t1 = std::chrono::steady_clock::now();
        std::fprintf(stderr, "%s: %.3f ms\n", what, std::chrono::duration<double>(t1 - t0).count() * 1e3);
        t0 = t1;
    };
    // the first-equal map (host hashing) runs on a second host thread under the device build
    std::vector<int> first;
    std::string err;
    int rc_first = PT_OK;
    std::thread fe([&] { rc_first = pt_internal::first_equal_indices(tris, n_tris, first, err); });
    std::vector<DNode> tree;
    int rc = build(tris, n_tris, device, tree);
    lap("device build");
    fe.join();
    lap("first-equal map (host thread, after the build)");
    if (rc_first) return fail(rc_first, err);
    if (rc) return fail(rc, g_err);
    // the reference's numbering: processing a node (root first, left subtree before right)
    // gives its children the next two indices (bvh.h:243-246); then build_links (bvh.h:84-98)
    const int nn = (int)tree.size();
    *n_nodes = nn;
    if (!nodes_out) return PT_OK;
    if (nn > max_nodes) return fail(PT_E_ARG, "node buffer too small");
    std::vector<int> idx(nn, -1);
    idx[0] = 0;
    int next = 1;
    std::vector<int> st;
    st.push_back(0);
    while (!st.empty()) {
        const int c = st.back();
        st.pop_back();
        const DNode& h = tree[c];
        if (h.left < 0) continue;
        idx[h.left] = next++;
        idx[h.right] = next++;
        st.push_back(h.right);
        st.push_back(h.left);
    }
    const float inf = std::numeric_limits<float>::infinity();
    for (int c = 0; c < nn; c++) {
        const DNode& h = tree[c];
        float* nd = nodes_out + 12 * (size_t)idx[c];
        nd[0] = h.b.mn[0]; nd[1] = h.b.mn[1]; nd[2] = h.b.mn[2]; nd[3] = inf;
        nd[4] = h.b.mx[0]; nd[5] = h.b.mx[1]; nd[6] = h.b.mx[2]; nd[7] = -inf;
        nd[8] = h.left < 0 ? (float)first[h.t0] : -1.0f;
        nd[9] = h.left < 0 ? (float)first[h.t1] : -1.0f;
    }
    std::vector<std::pair<int, int>> ls;
    ls.emplace_back(0, -1);
    while (!ls.empty()) {
        const auto [c, next_right] = ls.back();
        ls.pop_back();
        const DNode& h = tree[c];
        float* nd = nodes_out + 12 * (size_t)idx[c];
        if (h.left >= 0) {
            nd[10] = (float)idx[h.left];
            nd[11] = (float)next_right;
            ls.emplace_back(h.right, next_right);
            ls.emplace_back(h.left, idx[h.right]);
        } else {
            nd[10] = (float)next_right;
            nd[11] = (float)next_right;
        }
    }
    lap("numbering + links (host)");
    return PT_OK;
}
