// pt_group.hip -- multi-context image assembly over RCCL (include/pt_group.h).
//
// One process drives G contexts of one image, row-interleaved (context rank r of world G owns
// rows y = r + k*G).  The reference has a single GL context and no collective
// (ogl_path_trace.h:183-192); here:
//   * one RCCL communicator spans the distinct devices of the contexts (ncclCommInitAll);
//     the first context's device is rank 0, the root of every collective;
//   * scene upload: pt_upload_scene's validation + transposition runs once (first context);
//     each device's first context receives the device scene by ncclBroadcast, other contexts
//     on a device copy it on the device;
//   * gather: each device packs its contexts' rows into padded row blocks (one block of
//     rows_max = ceil(H/G) rows per context slot), ncclGather collects the blocks on the root,
//     and k_interleave_rows writes the full frame (HBM-bound copy, 16 B per pixel each way).
// Every step is stream-ordered after the contexts' renders (events), so no host round trip
// sits between the last render and the gather.
#include "../../include/pt_api.h"
#include "../../include/pt_group.h"
#include "pt_group_plan.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <string>
#include <vector>

// internal hooks of pt_render.hip (not part of the public ABI): kSceneBufs device scene
// buffers of a context, and the flag that lets a replicated context render
constexpr int kSceneBufs = 10;
extern "C" int pt__scene_replicate_layout(pt_ctx* dst, const pt_ctx* src, void* dptr[kSceneBufs],
                                          const void* sptr[kSceneBufs], size_t bytes[kSceneBufs]);
extern "C" int pt__scene_set_ready(pt_ctx* c, int ready);
extern "C" int pt__aces_launch(const void* src, void* dst, long long n, void* stream);

constexpr int kGroupPresentBufs = 4;   // pt_group_present_begin buffers

namespace {

// Full frame from the gathered blocks: row y comes from image rank r = y mod G, local row
// y div G, stored in block table[r] of rows_max rows (ptg::interleave_src, the function
// pt_group_interleave_host runs on the CPU).  One float4 per thread, coalesced.
__global__ __launch_bounds__(256) void k_interleave_rows(const float4* __restrict__ blocks, const int* __restrict__ table,
                                                         float4* __restrict__ out, int W, int world, int rows_max) {
    const int x = blockIdx.x * 256 + threadIdx.x;
    const int y = blockIdx.y;
    if (x >= W) return;
    out[(size_t)y * (size_t)W + (size_t)x] = blocks[ptg::interleave_src(x, y, W, world, rows_max, table)];
}

}  // namespace

struct pt_group {
    std::vector<pt_ctx*> ctx;
    int W = 0, H = 0, world = 0, rows_max = 0, max_slots = 0;
    std::vector<int> devs;                  // distinct devices; devs[0] = ctx[0]'s (the root)
    std::vector<int> dev_idx, slot;         // per context: device index, slot on that device
    std::vector<int> rows_local;            // per context
    std::vector<ncclComm_t> comm;
    std::vector<hipStream_t> stream;        // per device
    std::vector<float4*> send;              // per device: max_slots blocks
    float4* recv = nullptr;                 // root: devs.size() * max_slots blocks
    float4* frame = nullptr;                // root: the frame for host destinations
    int* d_table = nullptr;                 // root: image rank -> block index
    std::vector<hipEvent_t> ctx_ev;         // per context, on its device
    std::vector<hipEvent_t> packed_ev;      // per device: its contexts' rows are packed
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // pipelined ACES presentation (pt_group_present_*): per buffer an RGBA8 frame on the root
    // device, its pinned host copy and the copy's event (on the root's group stream)
    uchar4* present_dev[kGroupPresentBufs] = {};
    unsigned char* present_host[kGroupPresentBufs] = {};
    hipEvent_t ev_copied[kGroupPresentBufs] = {};
    hipEvent_t ev_g0[kGroupPresentBufs] = {}, ev_g1[kGroupPresentBufs] = {};   // its gather's timer
    bool present_pending[kGroupPresentBufs] = {};
    uchar4* rgba8 = nullptr;                // root: the ACES frame of pt_group_gather_rgba8_aces
    double last_ms = 0.0;
    std::string err;
};

static int gfail(pt_group* g, int code, const std::string& msg) {
    if (g) g->err = msg;
    return code;
}
#define GHIP(g, call)                                                                          \
    do {                                                                                       \
        hipError_t e_ = (call);                                                                \
        if (e_ != hipSuccess) return gfail(g, PT_E_HIP, std::string(#call ": ") + hipGetErrorString(e_)); \
    } while (0)
#define GNCCL(g, call)                                                                         \
    do {                                                                                       \
        ncclResult_t r_ = (call);                                                              \
        if (r_ != ncclSuccess) return gfail(g, PT_E_RCCL, std::string(#call ": ") + ncclGetErrorString(r_)); \
    } while (0)

static size_t block_floats(const pt_group* g) { return (size_t)g->rows_max * (size_t)g->W * 4; }

extern "C" {

void pt_group_destroy(pt_group* g) {
    if (!g) return;
    for (size_t d = 0; d < g->devs.size(); d++) {
        (void)hipSetDevice(g->devs[d]);
        if (d < g->stream.size() && g->stream[d]) (void)hipStreamSynchronize(g->stream[d]);
        if (d < g->comm.size() && g->comm[d]) (void)ncclCommDestroy(g->comm[d]);
        if (d < g->send.size()) (void)hipFree(g->send[d]);
        if (d < g->stream.size() && g->stream[d]) (void)hipStreamDestroy(g->stream[d]);
    }
    for (size_t i = 0; i < g->ctx_ev.size(); i++) {
        if (!g->ctx_ev[i]) continue;
        (void)hipSetDevice(g->devs[g->dev_idx[i]]);
        (void)hipEventDestroy(g->ctx_ev[i]);
    }
    for (size_t d = 0; d < g->packed_ev.size(); d++) {
        if (!g->packed_ev[d]) continue;
        (void)hipSetDevice(g->devs[d]);
        (void)hipEventDestroy(g->packed_ev[d]);
    }
    if (!g->devs.empty()) {
        (void)hipSetDevice(g->devs[0]);
        for (int b = 0; b < kGroupPresentBufs; b++) {
            (void)hipFree(g->present_dev[b]);
            if (g->present_host[b]) (void)hipHostFree(g->present_host[b]);
            if (g->ev_copied[b]) (void)hipEventDestroy(g->ev_copied[b]);
            if (g->ev_g0[b]) (void)hipEventDestroy(g->ev_g0[b]);
            if (g->ev_g1[b]) (void)hipEventDestroy(g->ev_g1[b]);
        }
        (void)hipFree(g->rgba8);
        (void)hipFree(g->recv);
        (void)hipFree(g->frame);
        (void)hipFree(g->d_table);
        if (g->ev0) (void)hipEventDestroy(g->ev0);
        if (g->ev1) (void)hipEventDestroy(g->ev1);
    }
    delete g;
}

const char* pt_group_last_error(const pt_group* g) { return g ? g->err.c_str() : "null group"; }

int pt_group_create(pt_ctx* const* ctxs, int n, pt_group** out) {
    if (!out) return PT_E_ARG;
    *out = nullptr;
    pt_group* g = new pt_group();
    *out = g;
    if (!ctxs || n < 1) return gfail(g, PT_E_ARG, "need at least one context");
    std::vector<pt_config> cfg(n);
    for (int i = 0; i < n; i++) {
        if (!ctxs[i] || pt_get_config(ctxs[i], &cfg[i])) return gfail(g, PT_E_ARG, "null context");
        g->ctx.push_back(ctxs[i]);
    }
    g->W = cfg[0].width;
    g->H = cfg[0].height;
    g->world = cfg[0].world;
    if (g->world != n) return gfail(g, PT_E_ARG, "the contexts' world size must equal their count");
    std::vector<int> seen(n, 0);
    for (int i = 0; i < n; i++) {
        if (cfg[i].width != g->W || cfg[i].height != g->H || cfg[i].world != g->world)
            return gfail(g, PT_E_ARG, "contexts of one group need the same width, height and world");
        // the gathered frame is one render only if every context renders the same way
        if (cfg[i].max_bounce != cfg[0].max_bounce || cfg[i].display_mode != cfg[0].display_mode ||
            cfg[i].flags != cfg[0].flags || cfg[i].rays_per_pixel != cfg[0].rays_per_pixel)
            return gfail(g, PT_E_ARG, "contexts of one group need the same max_bounce, display_mode, flags and "
                                      "rays_per_pixel");
        if (cfg[i].rank < 0 || cfg[i].rank >= n || seen[cfg[i].rank]++)
            return gfail(g, PT_E_ARG, "context ranks must be 0..world-1, each once");
    }
    g->rows_max = ptg::rows_max(g->H, g->world);
    // devices, slots and the block table: pt_group_plan (host arithmetic, CPU-tested)
    std::vector<int> dev_of(n), rank_of(n), devs(n), table(n);
    for (int i = 0; i < n; i++) {
        dev_of[i] = cfg[i].device;
        rank_of[i] = cfg[i].rank;
    }
    g->dev_idx.assign(n, 0);
    g->slot.assign(n, 0);
    int n_dev = 0;
    if (pt_group_plan(dev_of.data(), rank_of.data(), n, devs.data(), &n_dev, g->dev_idx.data(), g->slot.data(),
                      &g->max_slots, table.data()))
        return gfail(g, PT_E_ARG, "group plan");
    g->devs.assign(devs.begin(), devs.begin() + n_dev);
    g->rows_local.assign(n, 0);
    for (int i = 0; i < n; i++) pt_rows(ctxs[i], &g->rows_local[i], nullptr, nullptr);
    const int nd = (int)g->devs.size();
    g->comm.assign(nd, nullptr);
    GNCCL(g, ncclCommInitAll(g->comm.data(), nd, g->devs.data()));
    g->stream.assign(nd, nullptr);
    g->send.assign(nd, nullptr);
    g->packed_ev.assign(nd, nullptr);
    const size_t blk = block_floats(g) * sizeof(float);
    for (int d = 0; d < nd; d++) {
        GHIP(g, hipSetDevice(g->devs[d]));
        GHIP(g, hipStreamCreateWithFlags(&g->stream[d], hipStreamNonBlocking));
        GHIP(g, hipEventCreateWithFlags(&g->packed_ev[d], hipEventDisableTiming));
        GHIP(g, hipMalloc(&g->send[d], std::max<size_t>(blk * (size_t)g->max_slots, 16)));
    }
    g->ctx_ev.assign(n, nullptr);
    for (int i = 0; i < n; i++) {
        GHIP(g, hipSetDevice(cfg[i].device));
        GHIP(g, hipEventCreateWithFlags(&g->ctx_ev[i], hipEventDisableTiming));
    }
    GHIP(g, hipSetDevice(g->devs[0]));
    GHIP(g, hipMalloc(&g->recv, std::max<size_t>(blk * (size_t)g->max_slots * (size_t)nd, 16)));
    GHIP(g, hipMalloc(&g->frame, std::max<size_t>((size_t)g->W * (size_t)g->H * sizeof(float4), 16)));
    GHIP(g, hipMalloc(&g->d_table, table.size() * sizeof(int)));
    GHIP(g, hipMemcpy(g->d_table, table.data(), table.size() * sizeof(int), hipMemcpyHostToDevice));
    GHIP(g, hipEventCreate(&g->ev0));
    GHIP(g, hipEventCreate(&g->ev1));
    return PT_OK;
}

int pt_group_upload_scene(pt_group* g, const float* tris, int n_tris, const float* bvh, int n_nodes,
                          const float* mats, int n_mats, const float* spheres, int n_spheres) {
    if (!g || g->ctx.empty()) return PT_E_ARG;
    pt_ctx* root = g->ctx[0];
    int rc = pt_upload_scene(root, tris, n_tris, bvh, n_nodes, mats, n_mats, spheres, n_spheres);
    if (rc) return gfail(g, rc, std::string("pt_upload_scene: ") + pt_last_error(root));
    const int n = (int)g->ctx.size(), nd = (int)g->devs.size();
    std::vector<std::vector<void*>> dptr(n, std::vector<void*>(kSceneBufs, nullptr));
    const void* sptr[kSceneBufs] = {nullptr};
    size_t bytes[kSceneBufs] = {0};
    // the replicated contexts render only once their buffers are filled (set below, after the
    // streams have drained without error)
    for (int i = 1; i < n; i++) {
        rc = pt__scene_replicate_layout(g->ctx[i], root, dptr[i].data(), sptr, bytes);
        if (rc) return gfail(g, rc, std::string("scene layout: ") + pt_last_error(g->ctx[i]));
    }
    if (n == 1) return PT_OK;
    // the first context on each device receives the broadcast (the root device: ctx 0 itself)
    std::vector<int> leader(nd, -1);
    for (int i = 0; i < n; i++)
        if (leader[g->dev_idx[i]] < 0) leader[g->dev_idx[i]] = i;
    for (int b = 0; b < kSceneBufs; b++) {
        if (!bytes[b]) continue;
        if (nd > 1) {
            GNCCL(g, ncclGroupStart());
            for (int d = 0; d < nd; d++) {
                void* buf = d == 0 ? const_cast<void*>(sptr[b]) : dptr[leader[d]][b];
                if (hipSetDevice(g->devs[d]) != hipSuccess) { (void)ncclGroupEnd(); return gfail(g, PT_E_HIP, "hipSetDevice"); }
                ncclResult_t r = ncclBroadcast(buf, buf, bytes[b], ncclChar, 0, g->comm[d], g->stream[d]);
                if (r != ncclSuccess) { (void)ncclGroupEnd(); return gfail(g, PT_E_RCCL, std::string("ncclBroadcast: ") + ncclGetErrorString(r)); }
            }
            GNCCL(g, ncclGroupEnd());
        }
        for (int i = 1; i < n; i++) {
            const int d = g->dev_idx[i];
            if (leader[d] == i) continue;
            const void* from = d == 0 ? sptr[b] : dptr[leader[d]][b];
            GHIP(g, hipSetDevice(g->devs[d]));
            GHIP(g, hipMemcpyAsync(dptr[i][b], from, bytes[b], hipMemcpyDeviceToDevice, g->stream[d]));
        }
    }
    for (int d = 0; d < nd; d++) {
        GHIP(g, hipSetDevice(g->devs[d]));
        GHIP(g, hipStreamSynchronize(g->stream[d]));
    }
    for (int i = 1; i < n; i++) pt__scene_set_ready(g->ctx[i], 1);
    return PT_OK;
}

}  // extern "C"

// The gather, stream-ordered on the root device's stream: every device stream waits for its
// contexts' pending renders, packs their rows, ncclGather collects the blocks on the root and
// k_interleave_rows writes the frame to `out` (root device memory).  Each context's stream
// then waits for its device's pack, so renders queued after this call cannot overwrite rows
// that are still being packed.  Nothing is synchronised here.
static int gather_core(pt_group* g, float4* out, hipEvent_t e0, hipEvent_t e1) {
    const int n = (int)g->ctx.size(), nd = (int)g->devs.size();
    const size_t blk = block_floats(g);
    // the device streams wait for every context's pending renders first; the timer starts
    // after those waits, at the first pack copy (pt_group.h), not while renders still run
    for (int i = 0; i < n; i++) {
        const int d = g->dev_idx[i];
        void* cs = nullptr;
        pt_stream(g->ctx[i], &cs);
        GHIP(g, hipSetDevice(g->devs[d]));
        GHIP(g, hipEventRecord(g->ctx_ev[i], (hipStream_t)cs));
        GHIP(g, hipStreamWaitEvent(g->stream[d], g->ctx_ev[i], 0));
    }
    for (int i = 0; i < n; i++) {   // the root stream also waits for the other devices' renders
        if (g->dev_idx[i] == 0) continue;
        GHIP(g, hipSetDevice(g->devs[0]));
        GHIP(g, hipStreamWaitEvent(g->stream[0], g->ctx_ev[i], 0));
    }
    GHIP(g, hipSetDevice(g->devs[0]));
    GHIP(g, hipEventRecord(e0, g->stream[0]));
    // pack: each context's rows into its block
    for (int i = 0; i < n; i++) {
        const int d = g->dev_idx[i];
        void* acc = nullptr;
        size_t ab = 0;
        pt_accum_device(g->ctx[i], &acc, &ab);
        GHIP(g, hipSetDevice(g->devs[d]));
        if (ab) GHIP(g, hipMemcpyAsync(g->send[d] + (size_t)g->slot[i] * blk / 4, acc, ab, hipMemcpyDeviceToDevice,
                                       g->stream[d]));
    }
    for (int d = 0; d < nd; d++) {
        GHIP(g, hipSetDevice(g->devs[d]));
        GHIP(g, hipEventRecord(g->packed_ev[d], g->stream[d]));
    }
    for (int i = 0; i < n; i++) {
        void* cs = nullptr;
        pt_stream(g->ctx[i], &cs);
        GHIP(g, hipSetDevice(g->devs[g->dev_idx[i]]));
        GHIP(g, hipStreamWaitEvent((hipStream_t)cs, g->packed_ev[g->dev_idx[i]], 0));
    }
    GNCCL(g, ncclGroupStart());
    for (int d = 0; d < nd; d++) {
        if (hipSetDevice(g->devs[d]) != hipSuccess) { (void)ncclGroupEnd(); return gfail(g, PT_E_HIP, "hipSetDevice"); }
        ncclResult_t r = ncclGather(g->send[d], d == 0 ? (void*)g->recv : nullptr, blk * (size_t)g->max_slots, ncclFloat,
                                    0, g->comm[d], g->stream[d]);
        if (r != ncclSuccess) { (void)ncclGroupEnd(); return gfail(g, PT_E_RCCL, std::string("ncclGather: ") + ncclGetErrorString(r)); }
    }
    GNCCL(g, ncclGroupEnd());
    GHIP(g, hipSetDevice(g->devs[0]));
    if (g->H > 0 && g->W > 0) {
        hipLaunchKernelGGL(k_interleave_rows, dim3((unsigned)((g->W + 255) / 256), (unsigned)g->H), dim3(256), 0,
                           g->stream[0], g->recv, g->d_table, out, g->W, g->world, g->rows_max);
        GHIP(g, hipGetLastError());
    }
    GHIP(g, hipEventRecord(e1, g->stream[0]));
    return PT_OK;
}

// Drains the device streams (last one the root) and records the gather time.
static int gather_finish(pt_group* g) {
    for (int d = (int)g->devs.size() - 1; d >= 0; d--) {
        GHIP(g, hipSetDevice(g->devs[d]));
        GHIP(g, hipStreamSynchronize(g->stream[d]));
    }
    float ms = 0.0f;
    GHIP(g, hipEventElapsedTime(&ms, g->ev0, g->ev1));
    g->last_ms = ms;
    return PT_OK;
}

extern "C" {

int pt_group_gather_rgba32f(pt_group* g, float* dst, size_t bytes, int dst_on_device) {
    if (!g || !dst || g->ctx.empty()) return PT_E_ARG;
    const size_t frame_bytes = (size_t)g->W * (size_t)g->H * sizeof(float4);
    if (bytes < frame_bytes) return gfail(g, PT_E_ARG, "destination too small");
    float4* out = dst_on_device ? (float4*)dst : g->frame;
    int rc = gather_core(g, out, g->ev0, g->ev1);
    if (rc) return rc;
    if (!dst_on_device) GHIP(g, hipMemcpyAsync(dst, g->frame, frame_bytes, hipMemcpyDeviceToHost, g->stream[0]));
    return gather_finish(g);
}

int pt_group_gather_rgba8_aces(pt_group* g, unsigned char* dst, size_t bytes, int dst_on_device) {
    if (!g || !dst || g->ctx.empty()) return PT_E_ARG;
    const long long n = (long long)g->W * (long long)g->H;
    if (bytes < (size_t)n * 4) return gfail(g, PT_E_ARG, "destination too small");
    GHIP(g, hipSetDevice(g->devs[0]));
    if (!g->rgba8 && !dst_on_device) GHIP(g, hipMalloc(&g->rgba8, std::max<long long>(n, 1) * sizeof(uchar4)));
    int rc = gather_core(g, g->frame, g->ev0, g->ev1);
    if (rc) return rc;
    void* out = dst_on_device ? (void*)dst : (void*)g->rgba8;
    rc = pt__aces_launch(g->frame, out, n, g->stream[0]);
    if (rc) return gfail(g, rc, "k_aces launch");
    if (!dst_on_device && n) GHIP(g, hipMemcpyAsync(dst, g->rgba8, (size_t)n * 4, hipMemcpyDeviceToHost, g->stream[0]));
    return gather_finish(g);
}

int pt_group_present_begin(pt_group* g, int buf) {
    if (!g || g->ctx.empty()) return PT_E_ARG;
    if (buf < 0 || buf >= kGroupPresentBufs) return gfail(g, PT_E_ARG, "present buffer must be 0..3");
    const long long n = (long long)g->W * (long long)g->H;
    GHIP(g, hipSetDevice(g->devs[0]));
    // each resource on its own null check: an earlier call that failed part-way (say the
    // pinned allocation after the device one) must not leave later calls recording on null events
    if (!g->present_dev[buf])
        GHIP(g, hipMalloc(&g->present_dev[buf], std::max<long long>(n, 1) * sizeof(uchar4)));
    if (!g->present_host[buf])
        GHIP(g, hipHostMalloc((void**)&g->present_host[buf], std::max<long long>(n, 1) * sizeof(uchar4),
                              hipHostMallocDefault));
    if (!g->ev_copied[buf]) GHIP(g, hipEventCreateWithFlags(&g->ev_copied[buf], hipEventDisableTiming));
    if (!g->ev_g0[buf]) GHIP(g, hipEventCreate(&g->ev_g0[buf]));
    if (!g->ev_g1[buf]) GHIP(g, hipEventCreate(&g->ev_g1[buf]));
    // a buffer begun again before its end: its previous copy must land first
    if (g->present_pending[buf]) GHIP(g, hipEventSynchronize(g->ev_copied[buf]));
    g->present_pending[buf] = false;
    int rc = gather_core(g, g->frame, g->ev_g0[buf], g->ev_g1[buf]);
    if (rc) return rc;
    GHIP(g, hipSetDevice(g->devs[0]));
    rc = pt__aces_launch(g->frame, g->present_dev[buf], n, g->stream[0]);
    if (rc) return gfail(g, rc, "k_aces launch");
    // the copy on the root's group stream, behind the ACES pass: a copy stream waiting on an
    // event started each copy ~150 us late (pt_present_begin); the contexts'
    // renders wait only for the next gather's pack, not for this copy
    if (n) GHIP(g, hipMemcpyAsync(g->present_host[buf], g->present_dev[buf], (size_t)n * 4, hipMemcpyDeviceToHost,
                                  g->stream[0]));
    GHIP(g, hipEventRecord(g->ev_copied[buf], g->stream[0]));
    g->present_pending[buf] = true;
    return PT_OK;
}

int pt_group_present_end(pt_group* g, int buf, const unsigned char** pixels) {
    if (!g || !pixels) return PT_E_ARG;
    if (buf < 0 || buf >= kGroupPresentBufs) return gfail(g, PT_E_ARG, "present buffer must be 0..3");
    if (!g->present_pending[buf]) return gfail(g, PT_E_STATE, "pt_group_present_end without pt_group_present_begin");
    GHIP(g, hipSetDevice(g->devs[0]));
    GHIP(g, hipEventSynchronize(g->ev_copied[buf]));
    g->present_pending[buf] = false;
    // this buffer's own gather timer (a later begin re-records only its own buffer's events)
    float ms = 0.0f;
    GHIP(g, hipEventElapsedTime(&ms, g->ev_g0[buf], g->ev_g1[buf]));
    g->last_ms = ms;
    *pixels = g->present_host[buf];
    return PT_OK;
}

int pt_group_stats(const pt_group* g, double* gather_ms, size_t* bytes_per_device) {
    if (!g) return PT_E_ARG;
    if (gather_ms) *gather_ms = g->last_ms;
    if (bytes_per_device) *bytes_per_device = block_floats(g) * (size_t)g->max_slots * sizeof(float);
    return PT_OK;
}

int pt_gather_rgba32f(pt_ctx* const* ctxs, int n, float* dst, size_t bytes, int dst_on_device) {
    pt_group* g = nullptr;
    int rc = pt_group_create(ctxs, n, &g);
    if (!rc) rc = pt_group_gather_rgba32f(g, dst, bytes, dst_on_device);
    if (rc && n > 0 && ctxs && ctxs[0]) std::fprintf(stderr, "pt_gather_rgba32f: %s\n", pt_group_last_error(g));
    pt_group_destroy(g);
    return rc;
}

}  // extern "C"
