// solvebench — latency of the one-wave spec-a10 solve on ONE wave, the
// k_icp_coop critical path (tools/coopbench: LDL^T ~1.8 us of an 8.7 us
// iteration).  Each kernel runs `reps` dependent solves (the pose feeds the
// next) and reports s_memrealtime ns per solve; every variant's poses must
// equal production's bitwise.  Also checks recip_rn (the pivot reciprocal
// with hipcc's identity steps removed) against IEEE 1.0/d bitwise.
// Build: make -C tools solvebench        Run (GPU box): tools/solvebench
#include "../slam-rgbd_amd/csrc/icp_kernels.hip"

namespace {
template <int kVar>
__global__ void k_bench(const double* neq0, double* T64g, int reps, unsigned long long* ns)
{
    __shared__ double neq[kNeq], T64[12], L[36];
    __shared__ float T32[12];
    const int lane = threadIdx.x;
    if (lane < kNeq) neq[lane] = neq0[lane];
    if (lane < 12) T64[lane] = (lane % 5) == 0 ? 1.0 : 0.0;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    int st = 0;
    for (int r = 0; r < reps; ++r) {
        st |= solve_update_wave(neq, T64, T32, L, lane);
        // feed the pose back into b so every solve depends on the previous one
        if (lane == 0) neq[21] = neq0[21] + T64[3] * 1e-3;
        __syncthreads();
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (lane < 12) T64g[lane] = T64[lane];
    if (lane == 0) ns[0] = (t1 - t0) * 10;
    if (lane == 0) ns[1] = (unsigned long long)st;
}

__global__ void k_recip(unsigned long long n, unsigned long long seed, unsigned long long* bad)
{
    unsigned long long b = 0;
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
    for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += stride) {
        unsigned long long st = seed ^ (i * 0xD1B54A32D192ED03ull);
        const unsigned long long r = sm64(st);
        // exponent uniform over the guarded range [2^-900, 2^900], random mantissa;
        // every 8th case: mantissa all ones / all zeros / near those
        const int e = (int)(sm64(st) % 1801) - 900;
        unsigned long long m = r & 0xFFFFFFFFFFFFFull;
        if ((i & 7) == 0) m = (i & 8) ? 0xFFFFFFFFFFFFFull - (r & 15) : (r & 15);
        const double d = __longlong_as_double((long long)(((unsigned long long)(e + 1023) << 52) | m));
        b += __double_as_longlong(recip_rn(d)) != __double_as_longlong(1.0 / d);
    }
    if (b) atomicAdd(bad, b);
}
}  // namespace

int main()
{
    // a well-conditioned A (diagonally dominant) and b
    double h[kNeq];
    int k = 0;
    for (int a = 0; a < 6; ++a)
        for (int b = a; b < 6; ++b) h[k++] = a == b ? 1000.0 + 10 * a : 3.0 + a - b * 0.5;
    for (int i = 0; i < 6; ++i) h[21 + i] = 0.001 * (i + 1);
    h[27] = 1.0;
    h[28] = 300000.0;
    double *dn, *dT;
    unsigned long long* dns;
    (void)hipMalloc(&dn, sizeof(h));
    (void)hipMalloc(&dT, 12 * sizeof(double));
    (void)hipMalloc(&dns, 16);
    (void)hipMemcpy(dn, h, sizeof(h), hipMemcpyHostToDevice);
    const int reps = 2000;
    double T[1][12];
    for (int v = 0; v < 1; ++v) {
        unsigned long long ns[2] = {0, 0};
        for (int w = 0; w < 2; ++w) {
            hipLaunchKernelGGL(k_bench<0>, dim3(1), dim3(64), 0, 0, dn, dT, reps, dns);
            (void)hipMemcpy(ns, dns, 16, hipMemcpyDeviceToHost);
        }
        (void)hipMemcpy(T[v], dT, sizeof(T[v]), hipMemcpyDeviceToHost);
        printf("%-34s %7.0f ns per solve (one wave, %d dependent solves), status %llu\n",
               "solve_update_wave", (double)ns[0] / reps,
               reps, ns[1]);
    }
    printf("pose after the chain: t = (%.17g, %.17g, %.17g)\n", T[0][3], T[0][7], T[0][11]);
    (void)hipMemset(dns, 0, 8);
    const unsigned long long n = 1ull << 32;
    hipLaunchKernelGGL(k_recip, dim3(8192), dim3(256), 0, 0, n, 0x5EEDull, dns);
    unsigned long long bad = 0;
    (void)hipMemcpy(&bad, dns, 8, hipMemcpyDeviceToHost);
    printf("recip_rn vs IEEE 1.0/d: %llu mismatches of %llu (d in [2^-900, 2^900])\n", bad, n);
    return 0;
}
