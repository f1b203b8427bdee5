// Exhaustive check of the guarded fast forms in pt_math.h against the correctly rounded
// IEEE operations (-fhip-fp32-correctly-rounded-divide-sqrt), over EVERY binary32 input
// inside their guards, on the GPU whose v_rcp_f32 / v_sqrt_f32 they refine.
//   rcp_fast(x)  == 1.0f / x     for |x| in [2^-100, 2^100]
//   sqrt_fast(x) == sqrtf(x)     for  x  in [2^-100, 2^100]
//   div_mk(f, 2+f, rcp_fast(2+f)) == f / (2+f)   for |f| in [2^-21, 0.5]  (logf_pinned's
//                                                  quotient; its branch has |f| >= 2^-20)
//   logf_bf(x) == logf_pinned(x)  for x in [2^-32, 1]   (branch-free Box-Muller forms)
//   cosf_bf(x) == cosf_pinned(x)  for x in [0, 2*pi]
// Prints one line per check: "<name> tested=<n> bad=<n> first=<bits>"; exit 1 on any mismatch.
#include "../opengl-path-tracing_amd/csrc/pt_math.h"

#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k_check(unsigned lo, unsigned hi, int which, unsigned long long* bad, unsigned* first) {
    unsigned stride = gridDim.x * blockDim.x;
    unsigned long long nbad = 0;
    for (unsigned u = lo + blockIdx.x * blockDim.x + threadIdx.x; u < hi && u >= lo; u += stride) {
        float x = __uint_as_float(u);
        float got, want;
        if (which == 0) { got = pt::rcp_fast(x); want = 1.0f / x; }
        else if (which == 1) { got = pt::rcp_fast(-x); want = 1.0f / -x; }
        else if (which == 2) { got = pt::sqrt_fast(x); want = __builtin_sqrtf(x); }
        else if (which == 5) { got = pt::logf_bf(x); want = pt::logf_pinned(x); }
        else if (which == 6) { got = pt::cosf_bf(x); want = pt::cosf_pinned(x); }
        else {
            float f = which == 3 ? x : -x, tf = 2.0f + f;
            got = pt::div_mk(f, tf, pt::rcp_fast(tf));
            want = f / tf;
        }
        if (__float_as_uint(got) != __float_as_uint(want)) {
            nbad++;
            atomicMin(first, u);
        }
    }
    if (nbad) atomicAdd(bad, nbad);
}

int main() {
    const unsigned lo = 0x0d800000u;   // 2^-100
    const unsigned hi = 0x71800001u;   // 2^100 inclusive
    const char* names[7] = {"rcp_fast(+x)", "rcp_fast(-x)", "sqrt_fast", "logf quotient(+f)", "logf quotient(-f)",
                            "logf_bf", "cosf_bf"};
    unsigned long long* bad;
    unsigned* first;
    (void)hipMalloc(&bad, 8);
    (void)hipMalloc(&first, 4);
    int rc = 0;
    for (int w = 0; w < 7; w++) {
        unsigned a = w < 3 ? lo : 0x35000000u;   // 2^-21
        unsigned b = w < 3 ? hi : 0x3f000001u;   // 0.5 inclusive
        if (w == 5) { a = 0x2f800000u; b = 0x3f800001u; }   // [2^-32, 1]
        if (w == 6) { a = 0u; b = 0x40c90fdcu; }            // [0, 2*pi] (RN(2*pi) inclusive)
        (void)hipMemset(bad, 0, 8);
        (void)hipMemset(first, 0xff, 4);
        hipLaunchKernelGGL(k_check, dim3(8192), dim3(256), 0, 0, a, b, w, bad, first);
        unsigned long long nb = 0;
        unsigned f = 0;
        (void)hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(&f, first, 4, hipMemcpyDeviceToHost);
        if (hipDeviceSynchronize() != hipSuccess) { std::printf("hip error\n"); return 2; }
        std::printf("%s tested=%u bad=%llu first=0x%08x\n", names[w], b - a, nb, nb ? f : 0u);
        if (nb) rc = 1;
    }
    return rc;
}
