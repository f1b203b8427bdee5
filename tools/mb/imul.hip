#include <hip/hip_runtime.h>
#include <cstdio>
// Issue cost per wave-op (8 independent chains per lane, 8 waves per SIMD):
// v_fma_f32, v_mul_lo_u32 (+add), v_mul_u32_u24 (+add), the exact 32-bit product by 24-bit
// pieces (s*C mod 2^32 = mul24(s, Clo) + ((mad24(s>>24, Clo, mul24(s, Chi))) << 24)),
// v_rcp_f32, v_sqrt_f32.
template <int MODE>
__global__ __launch_bounds__(256) void k(unsigned* out, int iters) {
    unsigned a[8];
    float f[8];
    for (int i = 0; i < 8; i++) { a[i] = threadIdx.x * 7u + i; f[i] = threadIdx.x * 1e-3f + i + 1.0f; }
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            if (MODE == 0) f[i] = __builtin_fmaf(f[i], 1.0001f, 0.999f);
            if (MODE == 1) a[i] = a[i] * 747796405u + 2891336453u;
            if (MODE == 2) a[i] = __umul24(a[i], 0x5a5a5au) + 12345u;
            if (MODE == 3) {
                const unsigned C = 747796405u, lo = C & 0xffffffu, hi = C >> 24;
                unsigned p0 = __umul24(a[i], lo);
                unsigned p1 = __umul24(a[i] >> 24, lo) + __umul24(a[i], hi);
                a[i] = p0 + (p1 << 24) + 2891336453u;
            }
            if (MODE == 4) f[i] = __builtin_amdgcn_rcpf(f[i]);
            if (MODE == 5) f[i] = __builtin_amdgcn_sqrtf(f[i]);
        }
    }
    unsigned s = 0;
    for (int i = 0; i < 8; i++) s += a[i] + __float_as_uint(f[i]);
    if (s == 0x12345678u) out[0] = s;
}
__global__ void check(unsigned* bad) {
    unsigned x = blockIdx.x * 0x9E3779B9u + threadIdx.x * 0x85EBCA6Bu;
    const unsigned C = 747796405u, lo = C & 0xffffffu, hi = C >> 24;
    unsigned p = __umul24(x, lo) + ((__umul24(x >> 24, lo) + __umul24(x, hi)) << 24);
    if (p != x * C) atomicAdd(bad, 1u);
}
int main() {
    unsigned* o; (void)hipMalloc(&o, 4);
    (void)hipMemset(o, 0, 4);
    hipLaunchKernelGGL(check, dim3(65536), dim3(256), 0, 0, o);
    unsigned bad = 0; (void)hipMemcpy(&bad, o, 4, hipMemcpyDeviceToHost);
    printf("24-bit split product mismatches: %u of %u\n", bad, 65536u * 256u);
    hipEvent_t s, t; (void)hipEventCreate(&s); (void)hipEventCreate(&t);
    const char* nm[6] = {"v_fma_f32", "mul_lo_u32+add", "mul_u24+add", "split 32-bit mul", "v_rcp_f32", "v_sqrt_f32"};
    for (int rep = 0; rep < 2; rep++)
    for (int mode = 0; mode < 6; mode++) {
        auto run = [&]() {
            dim3 g(256 * 8), b(256);
            if (mode == 0) hipLaunchKernelGGL(k<0>, g, b, 0, 0, o, 10000);
            if (mode == 1) hipLaunchKernelGGL(k<1>, g, b, 0, 0, o, 10000);
            if (mode == 2) hipLaunchKernelGGL(k<2>, g, b, 0, 0, o, 10000);
            if (mode == 3) hipLaunchKernelGGL(k<3>, g, b, 0, 0, o, 10000);
            if (mode == 4) hipLaunchKernelGGL(k<4>, g, b, 0, 0, o, 10000);
            if (mode == 5) hipLaunchKernelGGL(k<5>, g, b, 0, 0, o, 10000);
        };
        run();
        (void)hipEventRecord(s); run(); (void)hipEventRecord(t); (void)hipEventSynchronize(t);
        float ms; (void)hipEventElapsedTime(&ms, s, t);
        if (rep) printf("%-18s %.3f ms  %.2f SIMD-cycles per wave-op at 2.4 GHz\n", nm[mode], ms,
                        ms * 1e-3 * 2.4e9 / (8.0 * 10000 * 8));
    }
    return 0;
}
