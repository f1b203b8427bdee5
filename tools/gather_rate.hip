// Random-gather rate of record layouts on gfx950: every lane loads one record per iteration at
// a hashed index into a table (L2-resident or larger), as the wide walk's global-memory record
// visits do, in several record sizes / load shapes.  Prints one JSON line per (table, shape):
// records per second chip-wide and ns per wave-level record load.
//   hipcc -O3 --offload-arch=gfx950 -o gather_rate tools/gather_rate.hip && ./gather_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define ITERS 512

__device__ __forceinline__ unsigned hash(unsigned x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

// SHAPE: 0 = 3 x 16 B (48-B stride), 1 = 2 x 16 B + 8 B (40-B stride), 2 = 2 x 16 B (32 B),
// 3 = 3 x 16 B on a 64-B stride, 4 = 4 x 16 B (64 B), 5 = 2 x 16 B + 8 B on a 48-B stride
template <int SHAPE>
__global__ __launch_bounds__(256) void k_gather(const unsigned char* __restrict__ tab, unsigned n, unsigned* out) {
    const unsigned tid = blockIdx.x * blockDim.x + threadIdx.x;
    constexpr unsigned stride = SHAPE == 0 ? 48 : SHAPE == 1 ? 40 : SHAPE == 2 ? 32 : SHAPE == 5 ? 48 : 64;
    unsigned acc = 0, s = tid * 2654435761u;
    for (int i = 0; i < ITERS; i++) {
        s = hash(s + (unsigned)i);
        const unsigned idx = s % n;
        const unsigned char* r = tab + (size_t)idx * stride;
        const uint4 a = *(const uint4*)r;
        const uint4 b = *(const uint4*)(r + 16);
        acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w;
        if (SHAPE == 0 || SHAPE == 3 || SHAPE == 4) {
            const uint4 c = *(const uint4*)(r + 32);
            acc ^= c.x ^ c.y ^ c.z ^ c.w;
        }
        if (SHAPE == 4) {
            const uint4 c = *(const uint4*)(r + 48);
            acc ^= c.x ^ c.y ^ c.z ^ c.w;
        }
        if (SHAPE == 1 || SHAPE == 5) {
            const uint2 c = *(const uint2*)(r + 32);
            acc ^= c.x ^ c.y;
        }
        s ^= acc & 1u;   // keep the loads live (and the chain honest)
    }
    out[tid] = acc;
}

typedef void (*KF)(const unsigned char*, unsigned, unsigned*);

int main() {
    const char* names[] = {"48B_3x16", "40B_2x16+8", "32B_2x16", "64Bstride_3x16", "64B_4x16", "48Bstride_2x16+8"};
    KF ks[] = {k_gather<0>, k_gather<1>, k_gather<2>, k_gather<3>, k_gather<4>, k_gather<5>};
    const size_t max_bytes = (size_t)64 << 20;
    unsigned char* tab;
    unsigned* out;
    if (hipMalloc(&tab, max_bytes) != hipSuccess) return 1;
    if (hipMemset(tab, 0x5a, max_bytes) != hipSuccess) return 1;
    const int blocks = 256 * 6, threads = 256;   // 6 waves per SIMD
    if (hipMalloc(&out, (size_t)blocks * threads * 4) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return 1;
    for (size_t tbytes : {(size_t)2 << 20, (size_t)8 << 20, (size_t)48 << 20}) {
        for (int k = 0; k < 6; k++) {
            const unsigned stride = k == 0 ? 48 : k == 1 ? 40 : k == 2 ? 32 : k == 5 ? 48 : 64;
            const unsigned n = (unsigned)(tbytes / stride) - 1;
            float best = 1e30f;
            for (int rep = 0; rep < 4; rep++) {
                if (hipEventRecord(e0) != hipSuccess) return 1;
                hipLaunchKernelGGL(ks[k], dim3(blocks), dim3(threads), 0, 0, tab, n, out);
                if (hipEventRecord(e1) != hipSuccess || hipEventSynchronize(e1) != hipSuccess) return 1;
                float ms;
                if (hipEventElapsedTime(&ms, e0, e1) != hipSuccess) return 1;
                if (rep && ms < best) best = ms;
            }
            const double recs = (double)blocks * threads * ITERS;
            printf("{\"table_mib\": %zu, \"shape\": \"%s\", \"ms\": %.4f, \"grecords_per_s\": %.2f, \"gb_per_s\": %.1f}\n",
                   tbytes >> 20, names[k], best, recs / best / 1e6, recs * (k == 2 ? 32 : k == 1 || k == 5 ? 40 : k == 4 ? 64 : 48) / best / 1e6);
        }
    }
    return 0;
}
