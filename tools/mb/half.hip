#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(256) void k(float* out, int mode, int iters) {
    int lane = threadIdx.x & 63;
    bool on = mode == 0 ? true : mode == 1 ? (lane < 32) : mode == 2 ? ((lane & 1) == 0) : (lane < 16);
    float b = 1.0001f, c = 0.999f;
    float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    if (on) {
        for (int i = 0; i < iters; i++) {
            a0 = __builtin_fmaf(a0, b, c); a1 = __builtin_fmaf(a1, b, c); a2 = __builtin_fmaf(a2, b, c); a3 = __builtin_fmaf(a3, b, c);
            a4 = __builtin_fmaf(a4, b, c); a5 = __builtin_fmaf(a5, b, c); a6 = __builtin_fmaf(a6, b, c); a7 = __builtin_fmaf(a7, b, c);
        }
    }
    if (a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 == 12345.0f) out[0] = a0;
}
int main() {
    float* o; (void)hipMalloc(&o, 4);
    hipEvent_t s, t; (void)hipEventCreate(&s); (void)hipEventCreate(&t);
    for (int rep = 0; rep < 2; rep++)
    for (int mode = 0; mode < 4; mode++) {
        hipLaunchKernelGGL(k, dim3(256 * 8), dim3(256), 0, 0, o, mode, 10000);
        (void)hipEventRecord(s);
        hipLaunchKernelGGL(k, dim3(256 * 8), dim3(256), 0, 0, o, mode, 10000);
        (void)hipEventRecord(t); (void)hipEventSynchronize(t);
        float ms; (void)hipEventElapsedTime(&ms, s, t);
        printf("mode %d (%s): %.3f ms  (%.2f cycles/wave-fma at 2.4 GHz)\n", mode, mode == 0 ? "all 64" : mode == 1 ? "lanes 0-31" : mode == 2 ? "even lanes" : "lanes 0-15", ms,
               ms * 1e-3 * 2.4e9 / (8.0 * 10000 * 8));
    }
    return 0;
}
