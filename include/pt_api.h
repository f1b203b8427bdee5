/* pt_api.h -- C ABI of the MI355X path-tracing hot path (HIP kernels for gfx950).
 *
 * Drop-in for the reference's GL compute-program interface:
 *   ComputeShader("computeShader.c")                 shader_c.h:14-60          -> pt_create
 *   SSBOs at bindings 4..8 (glMapBufferRange)        ogl_path_trace.h:383-529  -> pt_upload_scene
 *   camera SSBO re-upload (glBufferData)             ogl_path_trace.h:322-326  -> pt_set_camera
 *   setInt("frame"/"accumulate"/"displayMode"...)    ogl_path_trace.h:174-182  -> pt_render args
 *   glDispatchCompute(W/10, H/10, 1)                 ogl_path_trace.h:183      -> pt_render
 *   glMemoryBarrier + textured quad readback         ogl_path_trace.h:186-192  -> pt_read_rgba32f
 *   ACESFilm fragment shader                         screenQuadFrag.c:12-33    -> pt_read_rgba8_aces
 *
 * No torch / C++ types cross this boundary.  Every call is synchronous w.r.t. the host
 * unless named *_async.  A context is not thread-safe: one context per thread.
 * Return 0 on success, a negative PT_E* code otherwise; pt_last_error() explains.
 */
#ifndef PT_API_H
#define PT_API_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PT_OK 0
#define PT_E_ARG (-1)      /* bad argument / size */
#define PT_E_IO (-2)       /* file could not be opened */
#define PT_E_PARSE (-3)    /* OBJ/MTL line too long or malformed */
#define PT_E_SCENE (-4)    /* scene violates a limit or layout assumption */
#define PT_E_HIP (-5)      /* HIP runtime error (no device, OOM, launch failure) */
#define PT_E_STATE (-6)    /* call out of order (e.g. render before upload) */

/* Flags mirroring the shader's compile-time toggles (computeShader.c:77-82). */
#define PT_FLAG_NO_AA 1          /* antiAlias = false */
#define PT_FLAG_NO_SKY 2         /* EnvironmentEnabled = false */
#define PT_FLAG_NO_SPHERES 4     /* render_spheres = false */
#define PT_FLAG_NO_TRIANGLES 8   /* render_triangles = false */
#define PT_FLAG_REF_DISPATCH 16  /* write only the 10x10-group footprint of
                                    glDispatchCompute(W/10, H/10) (ogl_path_trace.h:183) */
#define PT_FLAG_MOLLER_TRUMBORE 32 /* opt-in fast mode: the reference's (dead) Moller-Trumbore
                                    RayIntersectsTriangle (computeShader.c:228-272) replaces the
                                    live hit_triangle (:274-307).  NOT the reference's image:
                                    pixels differ where the two tests disagree (tolerance in
                                    tests/test_gpu_parity.py); bit-exact to the oracle's MT mode */
#define PT_FLAG_ALL 63

typedef struct pt_ctx pt_ctx;

typedef struct {
    int width, height;       /* framebuffer (TEXTURE_WIDTH/HEIGHT, ogl_path_trace.h:45-46) */
    int max_bounce;          /* maxBounceCount; loop is i <= max_bounce (computeShader.c:74,447) */
    int display_mode;        /* 1 shaded, 2 normals, 3 albedo, 4 distance (computeShader.c:454-481) */
    int flags;               /* PT_FLAG_* */
    int rays_per_pixel;      /* raysPerPixel (computeShader.c:507); 1 in the reference */
    int device;              /* HIP device ordinal */
    int rank, world;         /* image partition: this context owns rows y = rank + k*world */
} pt_config;

int pt_create(const pt_config* cfg, pt_ctx** out);
void pt_destroy(pt_ctx* ctx);
const char* pt_last_error(const pt_ctx* ctx);

/* Scene upload in the reference's std140 layouts (see pt_scene.h).  The library validates
 * links/indices and transposes to its device layouts. */
int pt_upload_scene(pt_ctx* ctx, const float* tris, int n_tris, const float* bvh, int n_nodes,
                    const float* mats, int n_mats, const float* spheres, int n_spheres);

/* cam: 12 floats {position.xyzw, direction.xyzw, data.xyzw} (computeShader.c:50-55). */
int pt_set_camera(pt_ctx* ctx, const float cam[12]);
/* Uniform displayMode (1..4), set per frame by the reference (ogl_path_trace.h:182; the
 * keys 1-4 change it, :261-265).  Replaces pt_config.display_mode for later renders. */
int pt_set_display_mode(pt_ctx* ctx, int display_mode);

/* Equivalent to n_frames reference dispatches with frame = frame_first .. frame_first+n-1;
 * only the first uses accumulate = accumulate_first, the rest accumulate = 1 (running
 * mean, computeShader.c:548-551).  Bit-identical to n_frames separate calls, for any
 * n_frames: a render too large for one launch's scratch is split (tuning key 8). */
int pt_render(pt_ctx* ctx, int frame_first, int n_frames, int accumulate_first);
/* Same, enqueued on the context's stream without waiting (timing / overlap). */
int pt_render_async(pt_ctx* ctx, int frame_first, int n_frames, int accumulate_first);
int pt_sync(pt_ctx* ctx);

/* Progressive rendering as a replayed hipGraph (the reference's endless render loop,
 * ogl_path_trace.h:160-204, without a host round trip per frame): setup captures
 * `launches_per_replay` launches of `frames_per_launch` frames each plus a device-side
 * frame-counter advance; every replay renders the next frames_per_launch*launches frames.
 * Frame 1 is rendered with accumulate = 0 (a reset), later frames accumulate.  reset()
 * sets the next frame number (1 = restart accumulation).  The graph is dropped whenever
 * the scene, camera, kernel or tuning changes.  run() is asynchronous (pt_sync waits). */
int pt_progressive_setup(pt_ctx* ctx, int frames_per_launch, int launches_per_replay);
int pt_progressive_reset(pt_ctx* ctx, int next_frame);
int pt_progressive_run(pt_ctx* ctx, int replays);

/* Local rows owned by this context: rows y = rank + k*world, k < rows_local. */
int pt_rows(const pt_ctx* ctx, int* rows_local, int* row0, int* row_stride);
/* The context's configuration as created (display_mode as last set). */
int pt_get_config(const pt_ctx* ctx, pt_config* out);

/* Copies the local accumulation rows (rows_local * width * 4 floats, local row 0 =
 * image row `rank`, image row 0 = bottom). */
int pt_read_rgba32f(pt_ctx* ctx, float* host_dst, size_t bytes);
/* ACES-tonemapped RGBA8 of the local rows, computed on the device. */
int pt_read_rgba8_aces(pt_ctx* ctx, unsigned char* host_dst, size_t bytes);
/* Asynchronous presentation, for a loop that shows every frame (the reference draws each
 * frame's texture, ogl_path_trace.h:189-192).  pt_present_begin(buf) enqueues the ACES
 * epilogue of the image as of the renders issued so far, and its copy into the context's
 * pinned host buffer `buf` (0..3), both on the context stream; it does not wait, and later
 * renders overlap the copy.  When the caller presented after its previous render too, the
 * latest render's accumulate pass already wrote the view and only the copy is enqueued (a
 * write through pt_accum_device's pointer or onto pt_stream's stream must therefore come
 * after those calls, not before with a pointer kept from earlier).
 * pt_present_end(buf) waits for that copy and returns the
 * rows_local * width RGBA8 pixels (same bytes as pt_read_rgba8_aces), valid until the next
 * pt_present_begin on `buf` or pt_destroy.  Showing frame f-2 while frames f-1 and f render
 * (three buffers in rotation) keeps renders in flight, as the render-only loop does.
 * A buffer begun again before its end first waits for its previous copy.
 * PT_E_STATE: end without a begin. */
int pt_present_begin(pt_ctx* ctx, int buf);
int pt_present_end(pt_ctx* ctx, int buf, const unsigned char** pixels);
/* Overwrites the local accumulation rows (resume from a checkpoint / seed a test). */
int pt_write_rgba32f(pt_ctx* ctx, const float* host_src, size_t bytes);

/* Device pointer + size of the local accumulation buffer (for RCCL gathers). */
int pt_accum_device(pt_ctx* ctx, void** dev_ptr, size_t* bytes);
/* Stream-ordered device-to-device copy of the local rows into caller device memory
 * (e.g. an RCCL send buffer); returns after the copy completed. */
int pt_copy_rows_device(pt_ctx* ctx, void* dst_dev, size_t bytes);
/* The hipStream_t the context renders on (as void*). */
int pt_stream(pt_ctx* ctx, void** stream);

/* Statistics of the last pt_render*: kernel ms (HIP events on the render stream), and
 * when counting is enabled the reference-semantics work counts:
 * out[0] segments, [1] node visits, [2] triangle tests, [3] sphere tests, [4] hits. */
int pt_set_counting(pt_ctx* ctx, int enable);
int pt_stats(pt_ctx* ctx, double* kernel_ms, unsigned long long out[5]);
/* Counting-build diagnostics of the last render: out[0..4] as pt_stats, then per kernel
 * phase (traversal step, leaf test, segment) the wave iterations and the active lanes
 * summed over them: [5] trav waves, [6] trav lanes, [7] leaf waves, [8] leaf lanes,
 * [9] segment waves, [10] segment lanes (persistent kernels; 0 for the tiled kernel),
 * [11] segments outside the exact-reciprocal guard (state-machine kernel), [12] segments
 * that met a NaN.  Scene facts (any build): [13] bytes of the LDS scene copy, [14] the same
 * with the culling walk's sink image (0 when the tree does not qualify); [15] 1 when the
 * uploaded tree qualifies for the culling walk, it is on (tuning key 15) and the sink image
 * costs no resident workgroup per CU at the set waves per SIMD (key 3), else 0. */
int pt_stats_ex(pt_ctx* ctx, unsigned long long out[16]);
/* Sum of render-kernel durations (HIP events on the render stream) and the number of
 * launches since the last reset; reset != 0 clears both after reading. */
int pt_timing(pt_ctx* ctx, double* total_kernel_ms, int* n_launches, int reset);

/* Kernel variant selection: 0 = the state-machine kernel (default), 3 = the same kernel with
 * the scene kept in global memory even when it would fit LDS (A/B of the LDS staging). */
int pt_set_kernel(pt_ctx* ctx, int variant);
/* Scheduling knobs of the state-machine kernel:
 * key 0 = run the leaf phase once this many lanes wait at leaves (1..64, 0 = auto),
 * key 1 = run the shading phase once this many lanes finished their segment (1..64, 0 = auto),
 * key 2 = adaptive tile order (1 default: 8x8 tiles are queued most-expensive-first using
 *         the segment counts of the previous renders; 0 = raster order),
 * key 3 = resident waves per SIMD the kernel is compiled for (5..8; 0 = auto: 7 for scenes
 *         staged in LDS, 6 for global-memory scenes),
 * key 4 = queue ids a wave reserves per queue atomic in frame-split mode (1..1024; 0 = auto:
 *         256 / 64 for LDS-staged scenes with items of 1 / 2 frames, else about the launch's
 *         queue ids per resident wave / (8 x frames per item), clamped to 32..256).
 * key 5 = frames per work item (>= 1; 0 = auto, 2..8): a pixel's frames are spread over
 *         several lanes and the running mean is applied by a second kernel in frame order;
 *         a value >= n_frames gives each lane whole pixels (running mean in registers).
 *         In automatic mode launches of at most 16 frames always take the split path (its
 *         batched queue reservations), whatever their group.
 * key 6 = walk floor (1..64, 0 = auto): a walk phase ends once fewer lanes than this still
 *         walk, and the leaf (or shading) phase runs even below its threshold.
 * key 7 = leaf-phase compaction limit (0..63, default 63): the edge tests of a wave's leaf
 *         phase are packed onto its first lanes when at most this many (lane, triangle) pairs
 *         need them; 0 = every lane tests its own triangles.
 * key 8 = frame-split scratch budget in MiB (0 = automatic: min(32 GiB, device memory / 4)).
 *         A render whose per-frame colours (12 B per pixel-frame) exceed it -- or whose
 *         32-bit work-queue ids would overflow -- runs as back-to-back launches, the first
 *         with the caller's accumulate flag and the rest accumulating: the same image.
 * key 9 = overlapped short launches: render slots 2..4, 1 = off, 0 = automatic (3).  Renders
 *         of at most 16 frames (the reference's one dispatch per displayed frame) run their
 *         render kernel on one of these extra streams, so the next render fills the CUs that
 *         this one's launch tail frees; the running mean is still applied on the context's
 *         stream in frame order.
 * key 15 = culling walk (0 = automatic, 1 = off).  When the uploaded tree is a full binary
 *         tree threaded in preorder whose internal boxes contain their children's, the
 *         LDS-staged walk tests nodes with a cheaper conservative slab test and re-tests a
 *         leaf's box exactly before one of its triangles may move t.
 * key 16 = wide global-memory walk (0 = automatic, 1 = off: the binary walk).  Scenes too
 *         large for LDS with a nested tree walk a 4-wide tree of quantised child boxes
 *         (DESIGN.md §5.10).
 * key 17 = threads per workgroup of the wide walk: 256, 512, 768 or 1024 (0 = automatic, 256).
 * key 18 = overlapped short renders: 256-thread blocks per CU, 1..8 (0 = automatic: 3 with
 *         three or more render slots, 5 when the caller presents every frame).
 * key 19 = leaf re-test certificate (0 = automatic, 1 = off).  The wide walk skips the exact
 *         leaf-box re-test for a hit whose triangle data proves it passes;
 *         only for uploaded trees whose leaf boxes contain their triangles' vertices.
 * key 20 = work-queue tile shape: 1 = 8x8, 2 = 16x4, 3 = 32x2, 4 = 64x1 pixels (columns x local
 *         rows), 0 = automatic (8x8).  A change drains the context's streams and
 *         drops a captured graph.
 * None of these change the image (each pixel's frames stay in order in one lane). */
int pt_set_tuning(pt_ctx* ctx, int key, int value);

#ifdef __cplusplus
}
#endif
#endif /* PT_API_H */
