// rcp_probe.hip — exhaustive check of shorter correctly-rounded reciprocal
// sequences against IEEE 1.0f / den for EVERY fp32 den in [2^-60, 2^60]
// (the projection guard).  Variants:
//   A  (production): r = rcp; r = fma(fma(-d,r,1),r,r); two proj_div_one steps  (7 ops)
//   B  one Newton step:       r = rcp; r = fma(fma(-d,r,1),r,r)                  (3 ops)
//   C  two Newton steps:      B, then r = fma(fma(-d,r,1),r,r)                   (5 ops)
//   D  B then one residual correction on the quotient form q=r: q = fma(fma(-d,q,1),r0,q) (5 ops)
// usage: rcp_probe   (prints mismatches per variant)
#include <hip/hip_runtime.h>
#include <stdio.h>

__device__ __forceinline__ float nstep(float d, float r) { return fmaf(fmaf(-d, r, 1.0f), r, r); }

__global__ void k_probe(unsigned long long* bad)
{
    unsigned long long b[4] = {0, 0, 0, 0};
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
    const unsigned long long tid = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    constexpr unsigned kLo = 0x21800000u, kHi = 0x5D800000u;  // 2^-60, 2^60
    for (unsigned long long u = kLo + tid; u <= kHi; u += stride) {
        const float d = __uint_as_float((unsigned)u);
        const unsigned ref = __float_as_uint(1.0f / d);
        const float r0 = __builtin_amdgcn_rcpf(d);
        const float r1 = nstep(d, r0);
        float q = r1;
        q = fmaf(fmaf(-d, q, 1.0f), r1, q);
        q = fmaf(fmaf(-d, q, 1.0f), r1, q);
        b[0] += __float_as_uint(q) != ref;
        b[1] += __float_as_uint(r1) != ref;
        b[2] += __float_as_uint(nstep(d, r1)) != ref;
        b[3] += __float_as_uint(fmaf(fmaf(-d, r1, 1.0f), r0, r1)) != ref;
    }
    for (int k = 0; k < 4; ++k)
        if (b[k]) atomicAdd(bad + k, b[k]);
}

int main()
{
    unsigned long long* d;
    hipMalloc(&d, 4 * sizeof(unsigned long long));
    hipMemset(d, 0, 4 * sizeof(unsigned long long));
    hipLaunchKernelGGL(k_probe, dim3(8192), dim3(256), 0, 0, d);
    unsigned long long h[4];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    const char* names[4] = {"A production (7 ops)", "B one Newton step (3 ops)",
                            "C two Newton steps (5 ops)", "D B + residual with r0 (5 ops)"};
    for (int k = 0; k < 4; ++k) printf("%-32s mismatches %llu of %u\n", names[k], h[k], 0x5D800000u - 0x21800000u + 1);
    return 0;
}
