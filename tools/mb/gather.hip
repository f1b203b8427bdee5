// Microbenchmark: cost of scattered 16-B global loads (the global-memory BVH walk's node
// fetch) as a function of the active lanes per wave-instruction and of the loads per step.
// Each active lane chases a dependent chain through a table of float4 "nodes" (random
// successor per entry, like a walk's next-node index), so every load depends on the last.
//   mode k: lanes with (lane % 64) < k are active (exec mask), k = 64, 32, 16, 8, 4, 1
//   halves: 1 = one dwordx4 per step, 2 = two dwordx4 of the same 32-B record per step
// Prints lane-loads and wave-load-instructions per CU per cycle (2.4 GHz assumed).
// hipcc -O3 --offload-arch=gfx950 -o gather gather.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

template <int HALVES, int CHAINS>
__global__ __launch_bounds__(256) void k_chase(const float4* __restrict__ tab, unsigned n, int active, int iters,
                                               float* out) {
    const int lane = threadIdx.x & 63;
    unsigned idx[CHAINS];
    for (int c = 0; c < CHAINS; c++) idx[c] = ((blockIdx.x * 256u + threadIdx.x) * 4u + c) * 2654435761u % n;
    float acc = 0.0f;
    if (lane < active) {
        for (int i = 0; i < iters; i++) {
#pragma unroll
            for (int c = 0; c < CHAINS; c++) {
                const float4 a = tab[2 * idx[c]];
                float s = a.x + a.y;
                unsigned nx = __float_as_uint(a.w);
                if (HALVES == 2) {
                    const float4 b = tab[2 * idx[c] + 1];
                    s += b.x;
                    nx ^= __float_as_uint(b.w) & 1u;
                }
                acc += s;
                idx[c] = nx;
            }
        }
    }
    if (acc == 1234.5f) out[0] = acc;
}

int main(int argc, char** argv) {
    const unsigned n = argc > 1 ? (unsigned)atoi(argv[1]) : 78000u;   // C3-like node count (2.5 MB)
    std::vector<float> h(8 * (size_t)n);
    srand(1);
    for (unsigned i = 0; i < n; i++) {
        unsigned nx = ((unsigned)rand() * 65536u + (unsigned)rand()) % n;
        float* r = &h[8 * (size_t)i];
        for (int k = 0; k < 8; k++) r[k] = 0.001f * (float)k;
        unsigned u = nx;
        std::memcpy(&r[3], &u, 4);
        unsigned z = 0;
        std::memcpy(&r[7], &z, 4);
    }
    float4* d;
    float* o;
    (void)hipMalloc(&d, h.size() * 4);
    (void)hipMalloc(&o, 4);
    (void)hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    hipEvent_t s, t;
    (void)hipEventCreate(&s);
    (void)hipEventCreate(&t);
    const int iters = 2000;
    const int blocks_list[2] = {256 * 6, 256 * 2};   // 24 and 8 waves per CU
    for (int bi = 0; bi < 2; bi++) {
        const int blocks = blocks_list[bi];
        for (int cfg = 0; cfg < 4; cfg++) {
            const int halves = 1 + (cfg & 1), chains = cfg < 2 ? 1 : 4;
            const int acts[6] = {64, 32, 16, 8, 4, 1};
            for (int a : acts) {
                for (int rep = 0; rep < 2; rep++) {
                    (void)hipEventRecord(s);
                    if (cfg == 0) hipLaunchKernelGGL((k_chase<1, 1>), dim3(blocks), dim3(256), 0, 0, d, n, a, iters, o);
                    if (cfg == 1) hipLaunchKernelGGL((k_chase<2, 1>), dim3(blocks), dim3(256), 0, 0, d, n, a, iters, o);
                    if (cfg == 2) hipLaunchKernelGGL((k_chase<1, 4>), dim3(blocks), dim3(256), 0, 0, d, n, a, iters, o);
                    if (cfg == 3) hipLaunchKernelGGL((k_chase<2, 4>), dim3(blocks), dim3(256), 0, 0, d, n, a, iters, o);
                    (void)hipEventRecord(t);
                    (void)hipEventSynchronize(t);
                    float ms;
                    (void)hipEventElapsedTime(&ms, s, t);
                    if (rep == 0) continue;
                    const double cycles = ms * 1e-3 * 2.4e9;
                    const double waves_per_cu = blocks * 4.0 / 256.0;
                    const double instr = waves_per_cu * iters * halves * chains;  // per CU
                    printf("waves/CU %2.0f chains %d halves %d active %2d: %8.3f ms  wave-instr/CU/cyc %.4f  lane-loads/CU/cyc %.3f"
                           "  cyc/instr/CU %.1f\n", waves_per_cu, chains, halves, a, ms, instr / cycles, instr * a / cycles,
                           cycles / instr);
                    (void)chains;
                }
            }
        }
    }
    return 0;
}
