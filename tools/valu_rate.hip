// VALU issue-rate microbenchmark: time per wave-instruction of single f32 / int forms on gfx950
// (hipcc -O3 --offload-arch=gfx950 -o valu_rate tools/valu_rate.hip; profiles/ab/r05*_valu_rate.jsonl).
// Each wave runs 8 independent chains of one instruction form (inline asm, so exactly that
// encoding), one 1024-thread block per CU, 1 / 2 / 4 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define ITERS 4096
#define X8(F) F(a0) F(a1) F(a2) F(a3) F(a4) F(a5) F(a6) F(a7)
#define FORM(NAME, ASM, CONS)                                                                     \
    template <int D> __global__ __launch_bounds__(1024) void k_##NAME(float* out, unsigned long long* cyc, float seed) { \
        float a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,   \
              a6 = a0 + 6, a7 = a0 + 7;                                                               \
        float b = seed * 0.5f, c = seed * 0.25f;                                                      \
        unsigned w = threadIdx.x * 0x01020304u;                                                       \
        unsigned long long m;                                                                         \
        asm volatile("v_cmp_lt_f32 %0, %1, %2" : "=s"(m) : "v"(b), "v"(a0));                           \
        unsigned long long t0 = clock64();                                                            \
        for (int i = 0; i < ITERS; i++) {                                                             \
            _Pragma("unroll") for (int r = 0; r < 1; r++) {                                           \
                X8(ASM)                                                                               \
            }                                                                                         \
        }                                                                                             \
        unsigned long long t1 = clock64();                                                            \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + (float)(m & 1); \
        if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0; \
    }
#define A_FMA(x) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x) : "v"(b), "v"(c));
#define A_FMAC(x) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
#define A_ADD(x) asm volatile("v_add_f32 %0, %1, %0" : "+v"(x) : "v"(b));
#define A_MUL(x) asm volatile("v_mul_f32 %0, %1, %0" : "+v"(x) : "v"(b));
#define A_MIN(x) asm volatile("v_min_f32 %0, %1, %0" : "+v"(x) : "v"(b));
#define A_MAX3(x) asm volatile("v_max3_f32 %0, %1, %2, %0" : "+v"(x) : "v"(b), "v"(c));
#define A_MED3(x) asm volatile("v_med3_f32 %0, %1, %2, %0" : "+v"(x) : "v"(b), "v"(c));
#define A_PKFMA(v) { typedef float f2 __attribute__((ext_vector_type(2))); f2 p = {v, b}; \
    asm volatile("v_pk_fma_f32 %0, %0, %0, %0" : "+v"(p)); v = p[0]; }
#define A_MIX(x) asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,0]" : "+v"(x) : "v"(w), "v"(b));
#define A_CVTUB(x) asm volatile("v_cvt_f32_ubyte1 %0, %0" : "+v"(x));
#define A_CVTU32(x) asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(x));
#define A_LDEXP(x) asm volatile("v_ldexp_f32 %0, %0, %1" : "+v"(x) : "v"(w));
#define A_AND(x) asm volatile("v_and_b32 %0, %1, %0" : "+v"(x) : "v"(w));
#define A_ADDU(x) asm volatile("v_add_u32 %0, %1, %0" : "+v"(x) : "v"(w));
#define A_BFE(x) asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(x));
#define A_PERM(x) asm volatile("v_perm_b32 %0, %1, %0, %2" : "+v"(x) : "v"(w), "v"(0x05040100u));
#define A_CND(x) asm volatile("v_cndmask_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "s"(m));
#define A_CMP(x) asm volatile("v_cmp_le_f32 %0, %1, %2" : "=s"(m) : "v"(x), "v"(b));
#define A_XOR(x) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(x) : "v"(w));
#define A_SHL(x) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(x));
#define A_BITOP3(x) asm volatile("v_bitop3_b32 %0, %1, %0, %2 bitop3:0xca" : "+v"(x) : "v"(w), "v"(b));
#define A_ANDOR(x) asm volatile("v_and_or_b32 %0, %1, %0, %2" : "+v"(x) : "v"(w), "v"(b));
#define A_OR3(x) asm volatile("v_or3_b32 %0, %1, %0, %2" : "+v"(x) : "v"(w), "v"(b));
#define A_MAXI(x) asm volatile("v_max_i32 %0, %1, %0" : "+v"(x) : "v"(w));
#define A_SUBU(x) asm volatile("v_sub_u32 %0, %1, %0" : "+v"(x) : "v"(w));
#define A_FFBL(x) asm volatile("v_ffbl_b32 %0, %0" : "+v"(x));
#define A_CNDV(x) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(b));
#define A_PAIRV(x) asm volatile("v_cmp_le_f32 vcc, %0, %1\n\ts_nop 1\n\tv_cndmask_b32 %0, %0, %2, vcc" : "+v"(x) : "v"(b), "v"(c) : "vcc");
#define A_PAIRS(x) { unsigned long long q_; asm volatile("v_cmp_le_f32 %1, %0, %2\n\ts_nop 1\n\tv_cndmask_b32 %0, %0, %3, %1" : "+v"(x), "=&s"(q_) : "v"(b), "v"(c)); }
#define A_CNDVW(x) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(b));
#define A_MOV(x) asm volatile("v_mov_b32 %0, %1" : "=v"(x) : "v"(b)); asm volatile("" :: "v"(x));
FORM(fma, A_FMA, 0) FORM(fmac, A_FMAC, 0) FORM(add, A_ADD, 0) FORM(mul, A_MUL, 0) FORM(min, A_MIN, 0)
FORM(max3, A_MAX3, 0) FORM(med3, A_MED3, 0) FORM(pkfma, A_PKFMA, 0) FORM(mix, A_MIX, 0) FORM(cvtub, A_CVTUB, 0)
FORM(cvtu32, A_CVTU32, 0) FORM(ldexp, A_LDEXP, 0) FORM(and, A_AND, 0) FORM(addu, A_ADDU, 0) FORM(bfe, A_BFE, 0)
FORM(perm, A_PERM, 0) FORM(cnd, A_CND, 0) FORM(cmp, A_CMP, 0) FORM(mov, A_MOV, 0)
FORM(xor_, A_XOR, 0) FORM(shl, A_SHL, 0) FORM(bitop3, A_BITOP3, 0) FORM(andor, A_ANDOR, 0) FORM(or3, A_OR3, 0)
FORM(pairv, A_PAIRV, 0) FORM(pairs, A_PAIRS, 0)
FORM(maxi, A_MAXI, 0) FORM(subu, A_SUBU, 0) FORM(ffbl, A_FFBL, 0) FORM(cndv, A_CNDV, 0)
typedef void (*KF)(float*, unsigned long long*, float);
int main() {
    const int ncu = 256;
    struct { const char* name; KF f; } forms[] = {
        {"v_fma_f32", k_fma<0>}, {"v_fmac_f32", k_fmac<0>}, {"v_add_f32", k_add<0>}, {"v_mul_f32", k_mul<0>},
        {"v_min_f32", k_min<0>}, {"v_max3_f32", k_max3<0>}, {"v_med3_f32", k_med3<0>}, {"v_pk_fma_f32", k_pkfma<0>},
        {"v_fma_mix_f32", k_mix<0>}, {"v_cvt_f32_ubyte1", k_cvtub<0>}, {"v_cvt_f32_u32", k_cvtu32<0>},
        {"v_ldexp_f32", k_ldexp<0>}, {"v_and_b32", k_and<0>}, {"v_add_u32", k_addu<0>}, {"v_bfe_u32", k_bfe<0>},
        {"v_perm_b32", k_perm<0>}, {"v_cndmask_b32 (sgpr mask)", k_cnd<0>}, {"v_cmp_le_f32 (sgpr dst)", k_cmp<0>},
        {"v_mov_b32", k_mov<0>}, {"v_xor_b32", k_xor_<0>}, {"v_lshlrev_b32", k_shl<0>}, {"v_bitop3_b32", k_bitop3<0>},
        {"v_and_or_b32", k_andor<0>}, {"v_or3_b32", k_or3<0>}, {"v_max_i32", k_maxi<0>}, {"v_sub_u32", k_subu<0>},
        {"v_ffbl_b32", k_ffbl<0>}, {"v_cndmask_b32 (vcc)", k_cndv<0>},
        {"v_cmp vcc + s_nop 1 + v_cndmask vcc (pair)", k_pairv<0>}, {"v_cmp sgpr + s_nop 1 + v_cndmask sgpr (pair)", k_pairs<0>}};
    float* out; unsigned long long* cyc;
    if (hipMalloc(&out, (size_t)ncu * 1024 * 4) != hipSuccess || hipMalloc(&cyc, (size_t)ncu * 16 * 8) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return 1;
    for (int wps : {1, 4}) {
        const int threads = 256 * wps;
        for (auto& fm : forms) {
            float ms = 0.0f;
            for (int rep = 0; rep < 3; rep++) {
                if (hipEventRecord(e0) != hipSuccess) return 1;
                hipLaunchKernelGGL(fm.f, dim3(ncu), dim3(threads), 0, 0, out, cyc, 1.0f);
                if (hipEventRecord(e1) != hipSuccess || hipEventSynchronize(e1) != hipSuccess) return 1;
                if (hipEventElapsedTime(&ms, e0, e1) != hipSuccess) return 1;
            }
            std::vector<unsigned long long> h((size_t)ncu * threads / 64);
            if (hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return 1;
            double avg = 0; for (auto v : h) avg += (double)v; avg /= (double)h.size();
            const double per_simd = 8.0 * ITERS * wps;   // wave-instructions per SIMD
            printf("{\"instr\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"clock64_per_wave_instr\": %.3f, "
                   "\"ns_per_instr_per_simd\": %.4f}\n", fm.name, wps, ms, avg / (8.0 * ITERS), ms * 1e6 / per_simd);
        }
    }
    return 0;
}
