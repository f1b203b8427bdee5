/* pt_group.h -- one process driving an image split over several contexts:
 * a scene broadcast and the frame gather over RCCL (xGMI between the MI355X devices).
 *
 * The reference renders on one GL context: glDispatchCompute + glMemoryBarrier
 * (ogl_path_trace.h:183-186) and a textured-quad blit of the one image (:189-192).  Split
 * across G contexts (pt_config rank r of world G owns rows y = r, r + G, ...), the image is
 * assembled here:
 *   pt_group_create        one RCCL communicator over the contexts' distinct devices
 *                          (ncclCommInitAll); several contexts may share a device
 *   pt_group_upload_scene  pt_upload_scene's validation and layout transposition run once,
 *                          on the first context; its device scene is broadcast (ncclBroadcast)
 *                          to one context per device and copied on-device to the rest
 *   pt_group_gather_rgba32f every context's rows are gathered on the first context's device
 *                          (ncclGather of padded row blocks) and interleaved there by a
 *                          device kernel into the full RGBA32F frame, row 0 = bottom; the
 *                          result goes to host memory or stays in device memory
 *   pt_group_gather_rgba8_aces / pt_group_present_*  the same frame through the reference's
 *                          ACES view (screenQuadFrag.c:12-33), synchronous or pipelined
 * The gather waits for every context's stream (stream-ordered, no host round trip in
 * between) and returns once the frame is in `dst`.  The assembled frame is bit-identical to
 * a single context's render: each pixel's RNG depends only on (x, y, frame)
 * (computeShader.c:514-515).  Return 0 or a negative PT_E* code; pt_group_last_error explains.
 */
#ifndef PT_GROUP_H
#define PT_GROUP_H

#include <stddef.h>

#include "pt_api.h"

#ifdef __cplusplus
extern "C" {
#endif

#define PT_E_RCCL (-7)     /* RCCL error (communicator setup or a collective) */

typedef struct pt_group pt_group;

/* ctxs[0..n): contexts of one image (equal width, height and world = n, ranks 0..n-1 in any
 * order).  The frame is assembled on ctxs[0]'s device.  The contexts must outlive the group. */
int pt_group_create(pt_ctx* const* ctxs, int n, pt_group** out);
void pt_group_destroy(pt_group* g);
const char* pt_group_last_error(const pt_group* g);

/* pt_upload_scene for every context of the group (same arguments and checks). */
int pt_group_upload_scene(pt_group* g, const float* tris, int n_tris, const float* bvh, int n_nodes,
                          const float* mats, int n_mats, const float* spheres, int n_spheres);

/* Full frame (height * width * 4 floats = `bytes` or more).  dst_on_device != 0: dst is device
 * memory on ctxs[0]'s device; else host memory. */
int pt_group_gather_rgba32f(pt_group* g, float* dst, size_t bytes, int dst_on_device);

/* The reference's view of the frame: the gathered frame through the ACES epilogue
 * (screenQuadFrag.c:12-33) on the root device, RGBA8 with alpha 255 (height * width * 4
 * bytes), in host or root-device memory -- the multi-GPU form of pt_read_rgba8_aces, so a
 * display loop never tonemaps the 16-B-per-pixel frame on the host. */
int pt_group_gather_rgba8_aces(pt_group* g, unsigned char* dst, size_t bytes, int dst_on_device);

/* Pipelined presentation (the multi-GPU pt_present_begin / pt_present_end): begin enqueues the
 * gather and the ACES epilogue of the frame as every context's stream has it now, then a copy
 * into pinned host buffer `buf` (0..3) behind it on the root's group stream, and returns at
 * once; renders queued afterwards wait only for the row packing.  end waits for that copy and returns the
 * pinned pixels (valid until the buffer is begun again); pt_group_stats then reports that
 * buffer's gather time. */
int pt_group_present_begin(pt_group* g, int buf);
int pt_group_present_end(pt_group* g, int buf, const unsigned char** pixels);

/* Device time of the last gather (ms, from the first pack copy to the interleaved frame on the
 * root device, HIP events) and the bytes each device sent. */
int pt_group_stats(const pt_group* g, double* gather_ms, size_t* bytes_per_device);

/* One-shot form: create a group, gather, destroy (sets up a communicator on every call). */
int pt_gather_rgba32f(pt_ctx* const* ctxs, int n, float* dst, size_t bytes, int dst_on_device);

/* The gather plan pt_group_create computes -- host arithmetic only, no device is touched, so
 * the multi-device layouts can be checked on any machine.  Contexts i = 0..n-1 live on
 * device[i] with image rank rank[i] (world n, ranks 0..n-1 each once).  Out (n ints each):
 * the distinct devices in first-use order (devices_out[0] = device[0], the root of the
 * collectives) and their count, each context's device index and slot on that device, the
 * slots per device (every device sends max_slots padded row blocks of ceil(H/n) rows), and
 * table[rank] = dev_idx * max_slots + slot, the rank's block in the gathered buffer.
 * Returns 0 or PT_E_ARG. */
int pt_group_plan(const int* device, const int* rank, int n, int* devices_out, int* n_devices, int* dev_idx,
                  int* slot, int* max_slots, int* table);

/* The root's interleave on the host: frame (height x width RGBA32F) from n_blocks gathered
 * blocks of ceil(height/world) x width RGBA32F by the plan's table -- the index function of
 * the device kernel (csrc/pt_group_plan.h).  Returns 0 or PT_E_ARG (a table entry outside
 * the blocks). */
int pt_group_interleave_host(const float* blocks, size_t n_blocks, const int* table, int world, int width,
                             int height, float* frame);

#ifdef __cplusplus
}
#endif
#endif /* PT_GROUP_H */
