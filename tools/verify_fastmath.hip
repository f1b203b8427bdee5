// Exhaustive GPU checks of pt_math.h over EVERY binary32 input of each domain, on the GPU
// whose instructions the code refines:
//   rcp_fast(x)  == 1.0f / x   for |x| in [2^-100, 2^100]  (v_rcp_f32 + one fma step)
//   sqrt_fast(x) == sqrtf(x)   for  x  in [2^-100, 2^100]  (v_rsq_f32 + one fma step)
//   (the IEEE forms are -fhip-fp32-correctly-rounded-divide-sqrt's)
//   logf_pinned / cosf_pinned on the device == the same functions compiled for the host, for
//   x in {0} U [2^-32, 1] and t in [0, 2 pi]: an order-independent 64-bit checksum of
//   (input, output bits) over the whole domain on both sides (tools/verify_bf.cpp checks the
//   host functions against the oracle's restatement, input by input).
// Prints one line per check: "<name> tested=<n> bad=<n> first=<bits>"; exit 1 on any mismatch.
#include "../opengl-path-tracing_amd/csrc/pt_math.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <thread>
#include <vector>

__host__ __device__ inline unsigned long long mix64(unsigned long long z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
__host__ __device__ inline float pinned(int which, float x) {
    return which == 3 ? pt::logf_pinned(x) : pt::cosf_pinned(x);
}

__global__ void k_check(unsigned lo, unsigned hi, int which, unsigned long long* bad, unsigned* first) {
    unsigned stride = gridDim.x * blockDim.x;
    unsigned long long nbad = 0;
    for (unsigned u = lo + blockIdx.x * blockDim.x + threadIdx.x; u < hi && u >= lo; u += stride) {
        float x = __uint_as_float(u);
        float got, want;
        if (which == 0) { got = pt::rcp_fast(x); want = 1.0f / x; }
        else if (which == 1) { got = pt::rcp_fast(-x); want = 1.0f / -x; }
        else { got = pt::sqrt_fast(x); want = __builtin_sqrtf(x); }
        if (__float_as_uint(got) != __float_as_uint(want)) {
            nbad++;
            atomicMin(first, u);
        }
    }
    if (nbad) atomicAdd(bad, nbad);
}

__global__ void k_sum(unsigned lo, unsigned hi, int which, unsigned long long* sum) {
    unsigned stride = gridDim.x * blockDim.x;
    unsigned long long s = 0;
    for (unsigned u = lo + blockIdx.x * blockDim.x + threadIdx.x; u < hi && u >= lo; u += stride)
        s += mix64(((unsigned long long)u << 32) | __float_as_uint(pinned(which, __uint_as_float(u))));
    atomicAdd(sum, s);
}

static unsigned long long host_sum(unsigned lo, unsigned hi, int which) {
    const unsigned nthr = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::atomic<unsigned long long> total{0};
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nthr; t++)
        th.emplace_back([&, t]() {
            unsigned long long s = 0;
            for (unsigned long long u = (unsigned long long)lo + t; u < hi; u += nthr)
                s += mix64((u << 32) | pt::fbits(pinned(which, pt::bitsf((uint32_t)u))));
            total += s;
        });
    for (auto& x : th) x.join();
    return total.load();
}

int main() {
    const unsigned lo = 0x0d800000u;   // 2^-100
    const unsigned hi = 0x71800001u;   // 2^100 inclusive
    const char* names[5] = {"rcp_fast(+x)", "rcp_fast(-x)", "sqrt_fast", "logf_pinned device=host", "cosf_pinned device=host"};
    unsigned long long* bad;
    unsigned* first;
    (void)hipMalloc(&bad, 8);
    (void)hipMalloc(&first, 4);
    int rc = 0;
    for (int w = 0; w < 5; w++) {
        unsigned a = lo, b = hi;
        if (w == 3) { a = 0x2f800000u; b = 0x3f800001u; }   // [2^-32, 1]
        if (w == 4) { a = 0u; b = 0x40c90fddu; }            // [0, the largest angle the draw makes]
        (void)hipMemset(bad, 0, 8);
        (void)hipMemset(first, 0xff, 4);
        unsigned long long nb = 0;
        unsigned f = 0;
        if (w < 3) {
            hipLaunchKernelGGL(k_check, dim3(8192), dim3(256), 0, 0, a, b, w, bad, first);
            (void)hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost);
            (void)hipMemcpy(&f, first, 4, hipMemcpyDeviceToHost);
        } else {
            hipLaunchKernelGGL(k_sum, dim3(8192), dim3(256), 0, 0, a, b, w, bad);
            unsigned long long dev = 0;
            (void)hipMemcpy(&dev, bad, 8, hipMemcpyDeviceToHost);
            nb = dev != host_sum(a, b, w) ? 1 : 0;     // (a log-zero check rides along below)
            if (w == 3 && pt::fbits(pt::logf_pinned(0.0f)) != 0xff800000u) nb = 1;
        }
        if (hipDeviceSynchronize() != hipSuccess) { std::printf("hip error\n"); return 2; }
        std::printf("%s tested=%u bad=%llu first=0x%08x\n", names[w], b - a, nb, nb ? f : 0u);
        if (nb) rc = 1;
    }
    return rc;
}
