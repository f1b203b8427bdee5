// pt_group_plan.h -- the index arithmetic of pt_group's gather (include/pt_group.h), shared by
// the device kernel (pt_group.hip: k_interleave_rows) and the host planner / host interleave
// (pt_group_plan.cpp), so the CPU suite checks the very functions the GPU runs.
//
// Layout (the reference has one GL context, ogl_path_trace.h:183-192):
//   context of image rank r (world G) owns rows y = r + k*G, k < rows_local(r);
//   every context has a slot on its device; a device's send buffer holds max_slots blocks of
//   rows_max = ceil(H/G) rows (its contexts' rows, padded); ncclGather concatenates the send
//   buffers in device order on the root, so rank r's block is table[r] = dev_idx * max_slots +
//   slot; the frame's row y is block table[y mod G], local row y div G.
#pragma once

#include <stddef.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define PTG_HD __host__ __device__ __forceinline__
#else
#define PTG_HD inline
#endif

namespace ptg {

// rows of image rank r of world G (the pt_create partition: y = r, r + G, ...)
PTG_HD int rows_local(int H, int r, int G) { return H > r ? (H - r + G - 1) / G : 0; }

// padded block height
PTG_HD int rows_max(int H, int G) { return (H + G - 1) / G; }

// float4 index, in the gathered blocks, of frame pixel (x, y)
PTG_HD size_t interleave_src(int x, int y, int W, int G, int rmax, const int* table) {
    const int r = y % G, k = y / G;
    return ((size_t)table[r] * (size_t)rmax + (size_t)k) * (size_t)W + (size_t)x;
}

}  // namespace ptg
