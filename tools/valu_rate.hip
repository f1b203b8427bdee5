// VALU issue-rate microbenchmark: time per wave-instruction of a few f32 / int forms on gfx950
// (tools/valu_rate.hip; hipcc -O3 --offload-arch=gfx950 -o valu_rate valu_rate.hip; profiles/ab/r05g_valu_rate.jsonl).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define ITERS 4096
#define BODY8(I) I I I I I I I I
template <int K>
__global__ __launch_bounds__(1024) void kern(float* out, unsigned long long* cyc, float seed) {
    float a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    float b = seed * 0.5f, c = seed * 0.25f;
    unsigned w = threadIdx.x * 0x01020304u;
    unsigned long long t0 = clock64();
    for (int i = 0; i < ITERS; i++) {
        if (K == 0) {  // v_fma_f32
#define F(x) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x) : "v"(b), "v"(c));
            F(a0) F(a1) F(a2) F(a3) F(a4) F(a5) F(a6) F(a7)
#undef F
        } else if (K == 1) {  // v_pk_fma_f32 on pairs: 4 instr = 8 fmas
            typedef float f2 __attribute__((ext_vector_type(2)));
            f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}; f2 bb = {b, c};
#define F(x) asm volatile("v_pk_fma_f32 %0, %1, %1, %0" : "+v"(x) : "v"(bb));
            F(p0) F(p1) F(p2) F(p3) F(p0) F(p1) F(p2) F(p3)
#undef F
            a0 = p0.x; a1 = p0.y; a2 = p1.x; a3 = p1.y; a4 = p2.x; a5 = p2.y; a6 = p3.x; a7 = p3.y;
        } else if (K == 2) {  // v_fma_mix_f32
#define F(x) asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,0]" : "+v"(x) : "v"(w), "v"(b));
            F(a0) F(a1) F(a2) F(a3) F(a4) F(a5) F(a6) F(a7)
#undef F
        } else if (K == 3) {  // v_cvt_f32_ubyte0
#define F(x) asm volatile("v_cvt_f32_ubyte1 %0, %1" : "=v"(x) : "v"(w)); asm volatile("" :: "v"(x));
            F(a0) F(a1) F(a2) F(a3) F(a4) F(a5) F(a6) F(a7)
#undef F
        } else if (K == 4) {  // v_max3_f32
#define F(x) asm volatile("v_max3_f32 %0, %1, %2, %0" : "+v"(x) : "v"(b), "v"(c));
            F(a0) F(a1) F(a2) F(a3) F(a4) F(a5) F(a6) F(a7)
#undef F
        } else if (K == 5) {  // v_perm_b32
            unsigned u0 = w, u1 = w + 1, u2 = w + 2, u3 = w + 3, u4 = w + 4, u5 = w + 5, u6 = w + 6, u7 = w + 7;
#define F(x) asm volatile("v_perm_b32 %0, %1, %0, %2" : "+v"(x) : "v"(w), "v"(0x05040100u));
            F(u0) F(u1) F(u2) F(u3) F(u4) F(u5) F(u6) F(u7)
#undef F
            a0 += __uint_as_float(u0 ^ u1 ^ u2 ^ u3 ^ u4 ^ u5 ^ u6 ^ u7);
        } else if (K == 6) {  // v_cndmask_b32
#define F(x) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(b));
            F(a0) F(a1) F(a2) F(a3) F(a4) F(a5) F(a6) F(a7)
#undef F
        } else if (K == 7) {  // v_ldexp_f32
#define F(x) asm volatile("v_ldexp_f32 %0, %0, %1" : "+v"(x) : "v"(w));
            F(a0) F(a1) F(a2) F(a3) F(a4) F(a5) F(a6) F(a7)
#undef F
        }
    }
    unsigned long long t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}
int main() {
    int ncu = 256;
    const char* names[] = {"v_fma_f32", "v_pk_fma_f32", "v_fma_mix_f32", "v_cvt_f32_ubyte", "v_max3_f32", "v_perm_b32", "v_cndmask_b32", "v_ldexp_f32"};
    float* out; unsigned long long* cyc;
    hipMalloc(&out, ncu * 1024 * 4 * 8); hipMalloc(&cyc, ncu * 16 * 8 * 8);
    for (int wps = 1; wps <= 4; wps *= 2) {
        int threads = 256 * wps;   // wps waves per SIMD, one block per CU
        for (int k = 0; k < 8; k++) {
            hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
            for (int rep = 0; rep < 2; rep++) {
                hipEventRecord(e0);
                switch (k) {
                    case 0: kern<0><<<ncu, threads>>>(out, cyc, 1.0f); break;
                    case 1: kern<1><<<ncu, threads>>>(out, cyc, 1.0f); break;
                    case 2: kern<2><<<ncu, threads>>>(out, cyc, 1.0f); break;
                    case 3: kern<3><<<ncu, threads>>>(out, cyc, 1.0f); break;
                    case 4: kern<4><<<ncu, threads>>>(out, cyc, 1.0f); break;
                    case 5: kern<5><<<ncu, threads>>>(out, cyc, 1.0f); break;
                    case 6: kern<6><<<ncu, threads>>>(out, cyc, 1.0f); break;
                    case 7: kern<7><<<ncu, threads>>>(out, cyc, 1.0f); break;
                }
                hipEventRecord(e1); hipEventSynchronize(e1);
            }
            float ms; hipEventElapsedTime(&ms, e0, e1);
            std::vector<unsigned long long> h(ncu * threads / 64);
            hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
            double avg = 0; for (auto v : h) avg += v; avg /= h.size();
            // per SIMD: wps waves each issuing 8*ITERS instructions
            double instr_per_simd = 8.0 * ITERS * wps;
            printf("{\"instr\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"clock64_per_wave\": %.0f, \"clk_per_instr_per_simd\": %.3f, \"ns_per_instr_per_simd\": %.4f}\n",
                   names[k], wps, ms, avg, avg / instr_per_simd, ms * 1e6 / instr_per_simd);
        }
    }
    return 0;
}
