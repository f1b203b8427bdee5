// Throughput of v_fma_mix_f32 (binary16 operand converted in the fma) against v_fma_f32 on
// gfx950: 8 independent chains per lane, 4096 iterations, one kernel each; prints ns per
// wave-instruction per SIMD.  hipcc -O3 --offload-arch=gfx950 -o fmamix fmamix.hip
#include <hip/hip_runtime.h>
#include <cstdio>
template <int MIX>
__global__ __launch_bounds__(256) void k(float* out, unsigned h, float b, int iters) {
    float a[8];
    for (int i = 0; i < 8; i++) a[i] = threadIdx.x * 0.001f + i;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            if (MIX) asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,0]" : "+v"(a[i]) : "v"(h), "v"(b));
            else asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[i]) : "v"(__uint_as_float(h)), "v"(b));
        }
    }
    float s = 0;
    for (int i = 0; i < 8; i++) s += a[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
int main() {
    float* out;
    hipMalloc(&out, 256 * 4096 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 4096, blocks = 256 * 8;   // 8 blocks x 4 waves per CU = 8 waves per SIMD
    for (int rep = 0; rep < 2; rep++) {
        for (int mix = 0; mix < 2; mix++) {
            hipEventRecord(e0);
            if (mix) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, 0x3c003c00u, 1.0001f, iters);
            else hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, 0x3f800000u, 1.0001f, iters);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double winst = (double)blocks * 4 * iters * 8;     // wave-instructions
            printf("%s: %.3f ms, %.3f ns per wave-instruction per SIMD (1024 SIMDs)\n", mix ? "v_fma_mix_f32" : "v_fma_f32",
                   ms, ms * 1e6 * 1024 / winst);
        }
    }
    return 0;
}
