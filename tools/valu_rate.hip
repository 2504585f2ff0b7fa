// valu_rate — issue cost of the VALU instruction forms the ICP pixel loop uses
// (gfx950).  Each wave runs 8 independent dependency chains of ONE
// instruction form (inline asm, so the compiler cannot re-pack, re-encode or
// drop it); the chip is filled with 4 waves/SIMD; the printed cost is wall
// time per wave-instruction per SIMD (ns) and, with the shader clock of that
// run (thread 0 of every workgroup reads s_memtime = shader cycles and
// s_memrealtime = 100 MHz around its loop), cycles per wave-instruction per
// SIMD.  The results are the cost model of DESIGN.md §5
// (profiles/r01/valu_rate.txt: ns; profiles/r03/valu_cycles.txt: cycles).
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/valu_rate.hip -o tools/valu_rate
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

constexpr int kIters = 8192;
typedef float f2 __attribute__((ext_vector_type(2)));

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

// kinds of operand sets an instruction form reads/writes
#define DECL                                                                              \
    float a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,    \
          a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                          \
    f2 p0 = {a0, a1}, p1 = {a1, a2}, p2 = {a2, a3}, p3 = {a3, a4}, p4 = {a4, a5},         \
       p5 = {a5, a6}, p6 = {a6, a7}, p7 = {a7, a0};                                       \
    double d0 = a0, d1 = a1, d2 = a2, d3 = a3, d4 = a4, d5 = a5, d6 = a6, d7 = a7;        \
    const float c = 1.0000001f;                                                           \
    const f2 cc = {c, c};                                                                 \
    const double cd = 1.0000001;                                                          \
    unsigned long long m = __builtin_amdgcn_read_exec() & 0x5555555555555555ull;            \
    float x0 = a0 * 3, x1 = a1 * 3, x2 = a2 * 3, x3 = a3 * 3, x4 = a4 * 3, x5 = a5 * 3,     \
          x6 = a6 * 3, x7 = a7 * 3;                                                       \
    float y0 = a0 * 5, y1 = a1 * 5, y2 = a2 * 5, y3 = a3 * 5, y4 = a4 * 5, y5 = a5 * 5,     \
          y6 = a6 * 5, y7 = a7 * 5;                                                       \
    f2 q0 = p1 * 3, q1 = p2 * 3, q2 = p3 * 3, q3 = p4 * 3, q4 = p5 * 3, q5 = p6 * 3,        \
       q6 = p7 * 3, q7 = p0 * 3;                                                          \
    f2 r0 = p2 * 5, r1 = p3 * 5, r2 = p4 * 5, r3 = p5 * 5, r4 = p6 * 5, r5 = p7 * 5,        \
       r6 = p0 * 5, r7 = p1 * 5;                                                          \
    double e0 = d1 * 3, e1 = d2 * 3, e2 = d3 * 3, e3 = d4 * 3, e4 = d5 * 3, e5 = d6 * 3,   \
           e6 = d7 * 3, e7 = d0 * 3;                                                      \
    double g0 = d2 * 5, g1 = d3 * 5, g2 = d4 * 5, g3 = d5 * 5, g4 = d6 * 5, g5 = d7 * 5,   \
           g6 = d0 * 5, g7 = d1 * 5;

#define SINK                                                                              \
    out[blockIdx.x * blockDim.x + threadIdx.x] =                                          \
        a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + p0.x + p1.y + p2.x + p3.y + p4.x + p5.y + \
        p6.x + p7.y + (float)(d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7) + (float)(m & 1) +  \
        x0 + x7 + y0 + y7 + q0.x + q7.y + r0.x + r7.y + (float)(e0 + e7 + g0 + g7);

// one kernel per form: BODY(k) is the asm statement on chain k
#define FORM(NAME, BODY)                                                                  \
    __global__ __launch_bounds__(256) void k_##NAME(float* out, float seed,              \
                                                    unsigned long long* clk)             \
    {                                                                                     \
        DECL                                                                              \
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();                       \
        const unsigned long long rt0_ = __builtin_amdgcn_s_memrealtime();                   \
        for (int it = 0; it < kIters; ++it) {                                             \
            _Pragma("unroll") for (int u = 0; u < 8; ++u) { REP8(BODY) }                  \
        }                                                                                 \
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();                       \
        const unsigned long long rt1_ = __builtin_amdgcn_s_memrealtime();                   \
        if (threadIdx.x == 0) {                                                           \
            clk[2 * blockIdx.x] = t1 - t0;                                                \
            clk[2 * blockIdx.x + 1] = rt1_ - rt0_;                                            \
        }                                                                                 \
        SINK                                                                              \
    }

#define B_fma(k) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a##k) : "v"(c));
#define B_fmac(k) asm volatile("v_fmac_f32_e32 %0, %1, %1" : "+v"(a##k) : "v"(c));
#define B_mul(k) asm volatile("v_mul_f32_e32 %0, %0, %1" : "+v"(a##k) : "v"(c));
#define B_mul64(k) asm volatile("v_mul_f32_e64 %0, %0, -%1" : "+v"(a##k) : "v"(c));
#define B_add(k) asm volatile("v_add_f32_e32 %0, %0, %1" : "+v"(a##k) : "v"(c));
#define B_pkfma(k) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(p##k) : "v"(cc));
#define B_pkmul(k) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p##k) : "v"(cc));
#define B_pkadd(k) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p##k) : "v"(cc));
#define B_pkfmas(k) \
    asm volatile("v_pk_fma_f32 %0, %0, %1, %0 op_sel_hi:[1,0,1]" : "+v"(p##k) : "s"(cc));
#define B_fma64(k) asm volatile("v_fma_f64 %0, %0, %1, %0" : "+v"(d##k) : "v"(cd));
#define B_fmac64(k) asm volatile("v_fmac_f64_e32 %0, %1, %1" : "+v"(d##k) : "v"(cd));
#define B_add64(k) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d##k) : "v"(cd));
#define B_cvt64(k) asm volatile("v_cvt_f64_f32_e32 %0, %1" : "=v"(d##k) : "v"(a##k));
#define B_cvtfi(k) asm volatile("v_cvt_f32_i32_e32 %0, %0" : "+v"(a##k));
#define B_floor(k) asm volatile("v_floor_f32_e32 %0, %0" : "+v"(a##k));
#define B_rcp(k) asm volatile("v_rcp_f32_e32 %0, %0" : "+v"(a##k));
#define B_mov(k) asm volatile("v_mov_b32_e32 %0, %1" : "=v"(a##k) : "v"(a##k));
#define B_cnd32(k) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(a##k) : "v"(c));
#define B_cnd64(k) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a##k) : "v"(c), "s"(m));
#define B_cmp32(k) asm volatile("v_cmp_lt_f32_e32 vcc, %0, %1" ::"v"(a##k), "v"(c) : "vcc");
#define B_cmp64(k) asm volatile("v_cmp_lt_f32_e64 %0, %1, %2" : "=s"(m) : "v"(a##k), "v"(c));
#define B_dscale(k) asm volatile("v_div_scale_f32 %0, vcc, %0, %1, %0" : "+v"(a##k) : "v"(c) : "vcc");
#define B_dfmas(k) asm volatile("v_div_fmas_f32 %0, %0, %1, %1" : "+v"(a##k) : "v"(c));
#define B_dfix(k) asm volatile("v_div_fixup_f32 %0, %0, %1, %1" : "+v"(a##k) : "v"(c));
#define B_u64(k)                                                                            \
    {                                                                                       \
        unsigned long long q = (unsigned long long)__float_as_uint(a##k);                   \
        asm volatile("v_lshl_add_u64 %0, %0, 4, %0" : "+v"(q));                             \
        a##k = __uint_as_float((unsigned)q);                                                \
    }
#define B_addu(k) asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(a##k) : "v"(c));
// distinct operands (3 different registers / register pairs per instruction)
#define B_fma3(k) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a##k) : "v"(x##k), "v"(y##k));
#define B_pkfma3(k) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p##k) : "v"(q##k), "v"(r##k));
#define B_pkmul2(k) asm volatile("v_pk_mul_f32 %0, %1, %2" : "=v"(p##k) : "v"(q##k), "v"(r##k));
#define B_fmac64d(k) asm volatile("v_fmac_f64_e32 %0, %1, %2" : "+v"(d##k) : "v"(e##k), "v"(g##k));
#define B_fmac3(k) asm volatile("v_fmac_f32_e32 %0, %1, %2" : "+v"(a##k) : "v"(x##k), "v"(y##k));
#define B_mul2(k) asm volatile("v_mul_f32_e32 %0, %1, %2" : "=v"(a##k) : "v"(x##k), "v"(y##k));
#define B_cnd64d(k) asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(a##k) : "v"(x##k), "v"(y##k), "s"(m));
#define B_floor2(k) asm volatile("v_floor_f32_e32 %0, %1" : "=v"(a##k) : "v"(x##k));
#define B_cvtif2(k) asm volatile("v_cvt_i32_f32_e32 %0, %1" : "=v"(a##k) : "v"(x##k));
#define B_cvt64d(k) asm volatile("v_cvt_f64_f32_e32 %0, %1" : "=v"(d##k) : "v"(x##k));
#define B_mu24(k) asm volatile("v_mul_u32_u24_e32 %0, %1, %2" : "=v"(a##k) : "v"(x##k), "v"(y##k));
#define B_and(k) asm volatile("v_and_b32_e32 %0, %1, %2" : "=v"(a##k) : "v"(x##k), "v"(y##k));
#define B_cmpcnd(k)                                                                       \
    asm volatile("v_cmp_lt_f32_e32 vcc, %1, %2\n\tv_cndmask_b32_e32 %0, %0, %2, vcc"     \
                 : "+v"(a##k) : "v"(x##k), "v"(y##k) : "vcc");
#define B_cmpcnd64(k)                                                                      \
    {                                                                                      \
        unsigned long long mm;                                                             \
        asm volatile("v_cmp_lt_f32_e64 %1, %2, %3\n\tv_cndmask_b32_e64 %0, %0, %3, %1"    \
                     : "+v"(a##k), "=&s"(mm) : "v"(x##k), "v"(y##k));                      \
    }

FORM(fma, B_fma)
FORM(fmac, B_fmac)
FORM(mul, B_mul)
FORM(mul64, B_mul64)
FORM(add, B_add)
FORM(pkfma, B_pkfma)
FORM(pkmul, B_pkmul)
FORM(pkadd, B_pkadd)
FORM(pkfmas, B_pkfmas)
FORM(fma64, B_fma64)
FORM(fmac64, B_fmac64)
FORM(add64, B_add64)
FORM(cvt64, B_cvt64)
FORM(cvtfi, B_cvtfi)
FORM(floor, B_floor)
FORM(rcp, B_rcp)
FORM(mov, B_mov)
FORM(cnd32, B_cnd32)
FORM(cnd64, B_cnd64)
FORM(cmp32, B_cmp32)
FORM(cmp64, B_cmp64)
FORM(dscale, B_dscale)
FORM(dfmas, B_dfmas)
FORM(dfix, B_dfix)
FORM(u64, B_u64)
FORM(addu, B_addu)
FORM(fma3, B_fma3)
FORM(pkfma3, B_pkfma3)
FORM(pkmul2, B_pkmul2)
FORM(fmac64d, B_fmac64d)
FORM(cmpcnd, B_cmpcnd)
FORM(cmpcnd64, B_cmpcnd64)
FORM(fmac3, B_fmac3)
FORM(mul2, B_mul2)
FORM(cnd64d, B_cnd64d)
FORM(floor2, B_floor2)
FORM(cvtif2, B_cvtif2)
FORM(cvt64d, B_cvt64d)
FORM(mu24, B_mu24)
FORM(andb, B_and)

int main()
{
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int blocks = cus * 4;  // 4 workgroups x 4 waves per CU -> 4 waves/SIMD
    float* out;
    CK(hipMalloc(&out, (size_t)blocks * 256 * 4));
    unsigned long long* clk;
    CK(hipMalloc(&clk, (size_t)blocks * 2 * sizeof(unsigned long long)));
    unsigned long long* hclk = (unsigned long long*)malloc((size_t)blocks * 2 * sizeof(unsigned long long));
    struct F {
        const char* name;
        void (*k)(float*, float, unsigned long long*);
    } forms[] = {{"v_fma_f32 (VOP3)", k_fma},
                 {"v_fmac_f32_e32 (VOP2)", k_fmac},
                 {"v_mul_f32_e32", k_mul},
                 {"v_mul_f32_e64 (neg)", k_mul64},
                 {"v_add_f32_e32", k_add},
                 {"v_pk_fma_f32", k_pkfma},
                 {"v_pk_mul_f32", k_pkmul},
                 {"v_pk_add_f32", k_pkadd},
                 {"v_pk_fma_f32 s-bcast", k_pkfmas},
                 {"v_fma_f64 (VOP3)", k_fma64},
                 {"v_fmac_f64_e32", k_fmac64},
                 {"v_add_f64", k_add64},
                 {"v_cvt_f64_f32", k_cvt64},
                 {"v_cvt_f32_i32", k_cvtfi},
                 {"v_floor_f32", k_floor},
                 {"v_rcp_f32", k_rcp},
                 {"v_mov_b32", k_mov},
                 {"v_cndmask_b32_e32 vcc", k_cnd32},
                 {"v_cndmask_b32_e64 sgpr", k_cnd64},
                 {"v_cmp_lt_f32_e32 vcc", k_cmp32},
                 {"v_cmp_lt_f32_e64 sgpr", k_cmp64},
                 {"v_div_scale_f32", k_dscale},
                 {"v_div_fmas_f32", k_dfmas},
                 {"v_div_fixup_f32", k_dfix},
                 {"v_lshl_add_u64", k_u64},
                 {"v_add_u32", k_addu},
                 {"v_fma_f32 3 distinct", k_fma3},
                 {"v_pk_fma_f32 3 distinct", k_pkfma3},
                 {"v_pk_mul_f32 2 distinct", k_pkmul2},
                 {"v_fmac_f64 distinct", k_fmac64d},
                 {"cmp_e32+cndmask_e32 (x2)", k_cmpcnd},
                 {"cmp_e64+cndmask_e64 (x2)", k_cmpcnd64},
                 {"v_fmac_f32 distinct", k_fmac3},
                 {"v_mul_f32 distinct", k_mul2},
                 {"v_cndmask_e64 distinct", k_cnd64d},
                 {"v_floor_f32 distinct", k_floor2},
                 {"v_cvt_i32_f32 distinct", k_cvtif2},
                 {"v_cvt_f64_f32 distinct", k_cvt64d},
                 {"v_mul_u32_u24 distinct", k_mu24},
                 {"v_and_b32 distinct", k_andb}};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double inst_per_simd = 4.0 * kIters * 64;
    printf("%-26s %10s %14s %8s %16s\n", "form", "us", "ns/inst/SIMD", "GHz", "cycles/inst/SIMD");
    for (auto& f : forms) {
        hipLaunchKernelGGL(f.k, dim3(blocks), dim3(256), 0, 0, out, 1.0f, clk);
        CK(hipEventRecord(e0));
        for (int r = 0; r < 5; ++r)
            hipLaunchKernelGGL(f.k, dim3(blocks), dim3(256), 0, 0, out, 1.0f, clk);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / 5;
        // the last run's loop: shader cycles and 100 MHz ticks of every
        // workgroup's wave 0 (its 4 waves per SIMD run side by side)
        CK(hipMemcpy(hclk, clk, (size_t)blocks * 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        double cyc = 0, rt = 0;
        for (int b = 0; b < blocks; ++b) {
            cyc += (double)hclk[2 * b];
            rt += (double)hclk[2 * b + 1];
        }
        const double ghz = rt > 0 ? cyc / (rt * 10.0) : 0.0;  // realtime ticks are 10 ns
        printf("%-26s %10.1f %14.3f %8.3f %16.3f\n", f.name, us, us * 1e3 / inst_per_simd, ghz,
               cyc / blocks / inst_per_simd);
    }
    return 0;
}
