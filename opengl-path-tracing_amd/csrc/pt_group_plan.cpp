// pt_group_plan.cpp -- host planning of pt_group's scene broadcast and frame gather
// (include/pt_group.h).  Plain host code: pt_group_create uses it on the GPU path, and the CPU
// suite (tests/test_group_plan.py) runs it with the host interleave for device layouts no
// one-GPU box can create (several devices, any rank order).
#include "pt_group_plan.h"

#include "../../include/pt_group.h"

#include <cstring>
#include <vector>

extern "C" {

int pt_group_plan(const int* device, const int* rank, int n, int* devices_out, int* n_devices, int* dev_idx,
                  int* slot, int* max_slots, int* table) {
    if (!device || !rank || n < 1 || !devices_out || !n_devices || !dev_idx || !slot || !max_slots || !table)
        return PT_E_ARG;
    std::vector<int> seen(n, 0);
    for (int i = 0; i < n; i++)
        if (rank[i] < 0 || rank[i] >= n || seen[rank[i]]++) return PT_E_ARG;   // ranks 0..n-1, each once
    int nd = 0;
    std::vector<int> used;
    for (int i = 0; i < n; i++) {
        int d = 0;
        while (d < nd && devices_out[d] != device[i]) d++;
        if (d == nd) {               // first use: devices in first-use order, [0] = the root
            devices_out[nd++] = device[i];
            used.push_back(0);
        }
        dev_idx[i] = d;
        slot[i] = used[d]++;
    }
    int ms = 0;
    for (int u : used) ms = u > ms ? u : ms;
    for (int i = 0; i < n; i++) table[rank[i]] = dev_idx[i] * ms + slot[i];
    *n_devices = nd;
    *max_slots = ms;
    return PT_OK;
}

int pt_group_interleave_host(const float* blocks, size_t n_blocks, const int* table, int world, int width,
                             int height, float* frame) {
    if (!blocks || !table || !frame || world < 1 || width < 0 || height < 0) return PT_E_ARG;
    for (int r = 0; r < world; r++)
        if (table[r] < 0 || (size_t)table[r] >= n_blocks) return PT_E_ARG;
    const int rmax = ptg::rows_max(height, world);
    for (int y = 0; y < height; y++)
        for (int x = 0; x < width; x++)
            std::memcpy(frame + 4 * ((size_t)y * (size_t)width + (size_t)x),
                        blocks + 4 * ptg::interleave_src(x, y, width, world, rmax, table), 16);
    return PT_OK;
}

}  // extern "C"
