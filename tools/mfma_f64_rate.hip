// mfma_f64_rate — can the matrix pipe take k_icp's fp64 normal-equation
// accumulation (VERDICT r01 "next" item 3)?  Measures, on gfx950, the issue
// cost per SIMD of the two fp64 MFMA forms next to the VALU fp64 FMA that
// k_icp uses today, with the chip filled (one wave per SIMD and four waves
// per SIMD, 8 independent accumulators per wave):
//
//   v_mfma_f64_16x16x4_f64   C[16x16] += A[16x4] B[4x16]   (4 doubles/lane of C)
//   v_mfma_f64_4x4x4_4b_f64  4 blocks of C[4x4] += A[4x4] B[4x4]
//   v_fma_f64                one product-accumulate per lane
//
// and converts each into SIMD cycles per ICP pixel for the 28 products a
// pixel contributes (21 J^T J + 6 J^T r + 1 r^2).  Reading: DESIGN.md §5
// "The matrix pipe" (profiles/r02/mfma_f64_rate.txt).
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_f64_rate.hip -o tools/mfma_f64_rate
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

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int kIters = 512;

__global__ __launch_bounds__(256) void k_mfma16(double* out, double seed)
{
    const double a = seed + threadIdx.x, b = seed * 0.5 + threadIdx.x;
    d4 c[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) c[k] = d4{a + k, b, a, b};
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int k = 0; k < 8; ++k) c[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[k], 0, 0, 0);
    }
    double s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += c[k].x + c[k].y + c[k].z + c[k].w;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_mfma4(double* out, double seed)
{
    const double a = seed + threadIdx.x, b = seed * 0.5 + threadIdx.x;
    double c[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) c[k] = a + k;
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int k = 0; k < 8; ++k) c[k] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c[k], 0, 0, 0);
    }
    double s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += c[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_fma64(double* out, double seed)
{
    const double a = seed + threadIdx.x, b = 1.0000001;
    double c[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) c[k] = a + k;
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int k = 0; k < 8; ++k) asm volatile("v_fma_f64 %0, %0, %1, %0" : "+v"(c[k]) : "v"(b));
    }
    double s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += c[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main()
{
    int dev = 0, n_cu = 0;
    CK(hipSetDevice(dev));
    CK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
    const int simds = n_cu * 4;
    double* out = nullptr;
    CK(hipMalloc(&out, (size_t)n_cu * 16 * 256 * sizeof(double)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    struct Form {
        const char* name;
        void (*k)(double*, double);
        double products_per_inst;  // useful per-pixel products one instruction can retire
        const char* packing;
    } forms[] = {
        {"v_mfma_f64_16x16x4_f64", k_mfma16, 8 * 28.0 / 1.0,
         "block-diagonal: 2 groups x 4 pixels along K, features [J0..J5,r,1] along M/N"},
        {"v_mfma_f64_4x4x4_4b_f64", k_mfma4, 0.0, "feature dim 8 > 4: no per-pixel outer product fits"},
        {"v_fma_f64", k_fma64, 64.0, "one product per lane (k_icp today)"},
    };
    printf("%-26s %6s %10s %14s %18s  %s\n", "form", "waves", "us", "ns/inst/SIMD",
           "SIMD cyc/px @2.1G", "packing");
    for (const Form& f : forms) {
        for (int wps : {1, 4}) {
            const dim3 grid(n_cu * wps), block(256);
            hipLaunchKernelGGL(f.k, grid, block, 0, 0, out, 1.0);  // warm
            CK(hipDeviceSynchronize());
            float best = 1e30f;
            for (int rep = 0; rep < 5; ++rep) {
                CK(hipEventRecord(e0, 0));
                hipLaunchKernelGGL(f.k, grid, block, 0, 0, out, 1.0 + rep);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (ms < best) best = ms;
            }
            // instructions per SIMD = waves per SIMD x iters x 8
            const double inst = (double)wps * kIters * 8;
            const double ns = best * 1e6 / inst;
            // cycles per pixel: one instruction retires products_per_inst useful
            // products; a pixel needs 28
            const double cyc_px = f.products_per_inst > 0 ? ns * 2.1 * 28.0 / f.products_per_inst
                                                          : -1.0;
            printf("%-26s %6d %10.1f %14.3f %18.3f  %s\n", f.name, wps, best * 1e3, ns, cyc_px,
                   f.packing);
        }
    }
    (void)simds;
    CK(hipFree(out));
    return 0;
}
