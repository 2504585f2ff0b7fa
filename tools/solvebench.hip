// solvebench — latency of the one-wave spec-a10 solve on ONE wave, the
// k_icp_coop critical path (tools/coopbench: LDL^T ~1.8 us of an 8.7 us
// iteration).  Each kernel runs `reps` dependent solves (the pose feeds the
// next) and reports s_memrealtime ns per solve; every variant's poses must
// equal production's bitwise.
// Build: make -C tools solvebench        Run (GPU box): tools/solvebench
#include "../slam-rgbd_amd/csrc/icp_kernels.hip"
#include <cmath>
#include <cstring>
#include <vector>

namespace {

// The round-2 production solve (left-looking LDL^T, an early exit per pivot),
// kept here verbatim as the bitwise reference for the right-looking form.
__device__ __forceinline__ int solve_ref(const double* neq, double* T64, float* T32,
                                                double* Lsh, int lane)
{
    if (!(neq[28] >= 6.0)) return YOUTH_STATUS_FEW_MATCHES;
    const int i = lane < 6 ? lane : 5;
    double maxd = 0.0;
#pragma unroll
    for (int a = 0; a < 6; ++a) {
        const double da = neq[tri6(a, a)];
        if (da > maxd) maxd = da;
    }
    if (!(maxd > 0.0)) return YOUTH_STATUS_DEGENERATE;
    const double eps = 1e-12 * maxd;
    double Ar[6], Lr[6], D[6], Dinv[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        Ar[j] = neq[i <= j ? tri6(i, j) : tri6(j, i)];
        Lr[j] = 0.0;
    }
    // LDL^T, column j: lane i computes A[i][j] - sum_m (L[i][m] L[j][m]) D[m]
    // (lane j: the pivot d_j); L[i][j] = s / d_j below the diagonal
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        double sj = Ar[j];
#pragma unroll
        for (int m = 0; m < j; ++m) sj -= (Lr[m] * readlane64(Lr[m], j)) * D[m];
        const double d = readlane64(sj, j);
        if (!(d > eps)) return YOUTH_STATUS_DEGENERATE;
        D[j] = d;
        Dinv[j] = 1.0 / d;  // one divide per pivot; every use multiplies
        Lr[j] = lane > j ? sj * Dinv[j] : (lane == j ? 1.0 : 0.0);
    }
    // forward: y_i = (-b_i - sum_{m<i} L[i][m] y_m) / d_i
    double y = -neq[21 + i];
#pragma unroll
    for (int m = 0; m < 6; ++m) {
        const double ym = readlane64(y, m);
        y = lane > m ? y - Lr[m] * ym : y;
    }
    double dinv = Dinv[0];
#pragma unroll
    for (int j = 1; j < 6; ++j) dinv = i == j ? Dinv[j] : dinv;
    y = y * dinv;
    // back: x_i = y_i - sum_{m>i} L[m][i] x_m, m decreasing (column i of L via LDS)
    if (lane < 6) {
#pragma unroll
        for (int j = 0; j < 6; ++j) Lsh[lane * 6 + j] = Lr[j];
    }
    double x = y;
#pragma unroll
    for (int m = 5; m >= 0; --m) {
        const double xm = readlane64(x, m);
        const double Lmi = Lsh[m * 6 + i];
        x = lane < m ? x - Lmi * xm : x;
    }
    double xi[6];
#pragma unroll
    for (int m = 0; m < 6; ++m) xi[m] = readlane64(x, m);

    // T <- exp(xi^) T (se3_exp_left), one output entry per lane
    const double wx = xi[0], wy = xi[1], wz = xi[2];
    const double th2 = (wx * wx + wy * wy) + wz * wz;
    double a, b, c;
    if (th2 < 0x1p-7) {  // spec a10: Taylor in th2 (oracle_se3_exp: same fma chain)
        const double x2 = th2;
        a = fma(x2, fma(x2, fma(x2, fma(x2, fma(x2, -0x1.ae64567f544e4p-26, 0x1.71de3a556c734p-19),
                                          -0x1.a01a01a01a01ap-13), 0x1.1111111111111p-7),
                        -0x1.5555555555555p-3), 0x1.0000000000000p+0);
        b = fma(x2, fma(x2, fma(x2, fma(x2, fma(x2, -0x1.1eed8eff8d898p-29, 0x1.27e4fb7789f5cp-22),
                                          -0x1.a01a01a01a01ap-16), 0x1.6c16c16c16c17p-10),
                        -0x1.5555555555555p-5), 0x1.0000000000000p-1);
        c = fma(x2, fma(x2, fma(x2, fma(x2, fma(x2, -0x1.6124613a86d09p-33, 0x1.ae64567f544e4p-26),
                                          -0x1.71de3a556c734p-19), 0x1.a01a01a01a01ap-13),
                        -0x1.1111111111111p-7), 0x1.5555555555555p-3);
    } else {
        const double th = sqrt(th2);
        double sn, co;
        sincos(th, &sn, &co);
        a = sn / th;
        b = (1.0 - co) / th2;
        c = (th - sn) / (th2 * th);
    }
    const double Km[3][3] = {{0.0, -wz, wy}, {wz, 0.0, -wx}, {-wy, wx, 0.0}};
    const int l = lane < 12 ? lane : 11;
    const int r = l >> 2, col = l & 3;
    double Kr[3];  // row r of Km
#pragma unroll
    for (int k = 0; k < 3; ++k) Kr[k] = r == 0 ? Km[0][k] : (r == 1 ? Km[1][k] : Km[2][k]);
    double Er[3], Vr[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const double K2 = (Kr[0] * Km[0][k] + Kr[1] * Km[1][k]) + Kr[2] * Km[2][k];
        const double I = (r == k) ? 1.0 : 0.0;
        Er[k] = (I + a * Kr[k]) + b * K2;
        Vr[k] = (I + b * Kr[k]) + c * K2;
    }
    const double Er3 = (Vr[0] * xi[3] + Vr[1] * xi[4]) + Vr[2] * xi[5];
    double o = (Er[0] * T64[0 * 4 + col] + Er[1] * T64[1 * 4 + col]) + Er[2] * T64[2 * 4 + col];
    if (col == 3) o += Er3;
    if (lane < 12) {
        T64[lane] = o;
        T32[lane] = (float)o;
    }

    return 0;
}

// Correctly rounded 1/d without the generic division's scaling and fixup:
// v_rcp_f64, two Newton steps and a final FMA correction (Markstein), for
// positive normal d away from the exponent ends and not of significand
// 2 - 2^-52 (the known exception); anything else takes 1.0 / d.  d is
// wave-uniform in the solve (a readlane), so the test is a scalar branch.
__device__ __forceinline__ double rcp64_rn(double d)
{
    const unsigned long long bits = (unsigned long long)__double_as_longlong(d);
    const unsigned ex = (unsigned)(bits >> 52);  // sign 0 for d > 0
    const bool ok = ex >= 64u && ex <= 1983u && (bits & 0xFFFFFFFFFFFFFull) != 0xFFFFFFFFFFFFFull;
    if (!ok) return 1.0 / d;
    double r = __builtin_amdgcn_rcp(d);
    double e = fma(-d, r, 1.0);
    r = fma(r, e, r);
    e = fma(-d, r, 1.0);
    r = fma(r, e, r);
    e = fma(-d, r, 1.0);
    return fma(r, e, r);
}

__device__ __forceinline__ int solve_fast(const double* neq, double* T64, float* T32,
                                                double* Lsh, int lane)
{
    if (!(neq[28] >= 6.0)) return YOUTH_STATUS_FEW_MATCHES;
    const int i = lane < 6 ? lane : 5;
    double maxd = 0.0;
#pragma unroll
    for (int a = 0; a < 6; ++a) {
        const double da = neq[tri6(a, a)];
        if (da > maxd) maxd = da;
    }
    if (!(maxd > 0.0)) return YOUTH_STATUS_DEGENERATE;
    const double eps = 1e-12 * maxd;
    // LDL^T right-looking: lane i holds row i, S[j] = A[i][j] minus the
    // terms of the columns done so far.  Every element receives the same
    // subtractions in the same order (m increasing) as the left-looking
    // spec (solve6), so the results are bit-identical; but column m's
    // updates of the later columns and its forward-substitution step are
    // independent of column m+1's pivot divide and overlap it.  No early
    // exit inside the loop (one basic block): a failed pivot is flagged and
    // returned after it (nothing is stored before).
    double S[6], Lr[6], D[6], Dinv[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) S[j] = neq[i <= j ? tri6(i, j) : tri6(j, i)];
    // forward: y_i = (-b_i - sum_{m<i} L[i][m] y_m) / d_i, step m right after column m
    double y = -neq[21 + i];
    bool bad = false;
#pragma unroll
    for (int m = 0; m < 6; ++m) {
        const double d = readlane64(S[m], m);
        bad |= !(d > eps);
        D[m] = d;
        Dinv[m] = rcp64_rn(d);  // one divide per pivot; every use multiplies
        Lr[m] = lane > m ? S[m] * Dinv[m] : (lane == m ? 1.0 : 0.0);
#pragma unroll
        for (int j = m + 1; j < 6; ++j) S[j] -= (Lr[m] * readlane64(Lr[m], j)) * D[m];
        const double ym = readlane64(y, m);
        y = lane > m ? y - Lr[m] * ym : y;
    }
    if (bad) return YOUTH_STATUS_DEGENERATE;
    double dinv = Dinv[0];
#pragma unroll
    for (int j = 1; j < 6; ++j) dinv = i == j ? Dinv[j] : dinv;
    y = y * dinv;
    // back: x_i = y_i - sum_{m>i} L[m][i] x_m, m decreasing (column i of L via LDS)
    if (lane < 6) {
#pragma unroll
        for (int j = 0; j < 6; ++j) Lsh[lane * 6 + j] = Lr[j];
    }
    double x = y;
#pragma unroll
    for (int m = 5; m >= 0; --m) {
        const double xm = readlane64(x, m);
        const double Lmi = Lsh[m * 6 + i];
        x = lane < m ? x - Lmi * xm : x;
    }
    double xi[6];
#pragma unroll
    for (int m = 0; m < 6; ++m) xi[m] = readlane64(x, m);

    // T <- exp(xi^) T (se3_exp_left), one output entry per lane
    const double wx = xi[0], wy = xi[1], wz = xi[2];
    const double th2 = (wx * wx + wy * wy) + wz * wz;
    double a, b, c;
    if (th2 < 0x1p-7) {  // spec a10: Taylor in th2 (oracle_se3_exp: same fma chain)
        const double x2 = th2;
        a = fma(x2, fma(x2, fma(x2, fma(x2, fma(x2, -0x1.ae64567f544e4p-26, 0x1.71de3a556c734p-19),
                                          -0x1.a01a01a01a01ap-13), 0x1.1111111111111p-7),
                        -0x1.5555555555555p-3), 0x1.0000000000000p+0);
        b = fma(x2, fma(x2, fma(x2, fma(x2, fma(x2, -0x1.1eed8eff8d898p-29, 0x1.27e4fb7789f5cp-22),
                                          -0x1.a01a01a01a01ap-16), 0x1.6c16c16c16c17p-10),
                        -0x1.5555555555555p-5), 0x1.0000000000000p-1);
        c = fma(x2, fma(x2, fma(x2, fma(x2, fma(x2, -0x1.6124613a86d09p-33, 0x1.ae64567f544e4p-26),
                                          -0x1.71de3a556c734p-19), 0x1.a01a01a01a01ap-13),
                        -0x1.1111111111111p-7), 0x1.5555555555555p-3);
    } else {
        const double th = sqrt(th2);
        double sn, co;
        sincos(th, &sn, &co);
        a = sn / th;
        b = (1.0 - co) / th2;
        c = (th - sn) / (th2 * th);
    }
    const double Km[3][3] = {{0.0, -wz, wy}, {wz, 0.0, -wx}, {-wy, wx, 0.0}};
    const int l = lane < 12 ? lane : 11;
    const int r = l >> 2, col = l & 3;
    double Kr[3];  // row r of Km
#pragma unroll
    for (int k = 0; k < 3; ++k) Kr[k] = r == 0 ? Km[0][k] : (r == 1 ? Km[1][k] : Km[2][k]);
    double Er[3], Vr[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const double K2 = (Kr[0] * Km[0][k] + Kr[1] * Km[1][k]) + Kr[2] * Km[2][k];
        const double I = (r == k) ? 1.0 : 0.0;
        Er[k] = (I + a * Kr[k]) + b * K2;
        Vr[k] = (I + b * Kr[k]) + c * K2;
    }
    const double Er3 = (Vr[0] * xi[3] + Vr[1] * xi[4]) + Vr[2] * xi[5];
    double o = (Er[0] * T64[0 * 4 + col] + Er[1] * T64[1 * 4 + col]) + Er[2] * T64[2 * 4 + col];
    if (col == 3) o += Er3;
    if (lane < 12) {
        T64[lane] = o;
        T32[lane] = (float)o;
    }
    return 0;
}


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
        st |= kVar == 0   ? solve_update_wave(neq, T64, T32, L, lane)
              : kVar == 2 ? solve_fast(neq, T64, T32, L, lane)
                          : solve_ref(neq, T64, T32, L, lane);
        // feed the pose back into b so every solve depends on the previous one
        if (lane == 0) neq[21] = neq0[21] + T64[3] * 1e-3;
        __syncthreads();
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (lane < 12) T64g[lane] = T64[lane];
    if (lane == 0) ns[0] = (t1 - t0) * 10;
    if (lane == 0) ns[1] = (unsigned long long)st;
}


// Bitwise: one wave per case; case c's system is sys[c][kNeq]; both solves
// start from the same pose; mismatching poses or statuses are counted.
template <int kMode>
__global__ void k_cmp(const double* sys, int n, unsigned long long* bad)
{
    __shared__ double neq[kNeq], Ta[12], Tb[12], L[36];
    __shared__ float T32a[12], T32b[12];
    const int lane = threadIdx.x;
    for (int c = blockIdx.x; c < n; c += gridDim.x) {
        if (lane < kNeq) neq[lane] = sys[(size_t)c * kNeq + lane];
        if (lane < 12) {
            Ta[lane] = Tb[lane] = (lane % 5) == 0 ? 1.0 : 0.0;
            T32a[lane] = T32b[lane] = 0.0f;  // written only by an update
        }
        __syncthreads();
        const int sa = solve_update_wave(neq, Ta, T32a, L, lane);
        __syncthreads();
        const int sb = kMode == 0 ? solve_ref(neq, Tb, T32b, L, lane) : solve_fast(neq, Tb, T32b, L, lane);
        __syncthreads();
        const bool diff = lane < 12 && (__double_as_longlong(Ta[lane]) != __double_as_longlong(Tb[lane]) ||
                                        __float_as_uint(T32a[lane]) != __float_as_uint(T32b[lane]));
        const unsigned long long any = __ballot(diff) != 0ull || sa != sb;
        if (lane == 0 && any) atomicAdd(bad, 1ull);
        if (lane == 0 && sa) atomicAdd(bad + 1, 1ull);
        __syncthreads();
    }
}
// rcp64_rn vs 1.0 / d bitwise over n SplitMix64 doubles: random significands
// with exponents across the whole positive range, plus significands next to
// all-ones and to 1 (the hard cases).
__global__ void k_rcp_test(unsigned long long n, unsigned long long* bad)
{
    unsigned long long nb = 0;
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
    for (unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i < n; i += stride) {
        unsigned long long st = i * 0x9E3779B97F4A7C15ull + 0x1234567ull;
        const unsigned long long r1 = sm64(st), r2 = sm64(st);
        unsigned long long man = r1 & 0xFFFFFFFFFFFFFull;
        if ((i & 7) == 1) man = 0xFFFFFFFFFFFFFull - (r2 & 0xFF);   // next to all ones
        if ((i & 7) == 2) man = r2 & 0xFF;                          // next to 1.0
        const unsigned long long ex = 1 + (r2 >> 20) % 2046;        // every normal exponent
        const double d = __longlong_as_double((long long)((ex << 52) | man));
        nb += __double_as_longlong(rcp64_rn(d)) != __double_as_longlong(1.0 / d);
    }
    if (nb) atomicAdd(bad, nb);
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
    double T[3][12];
    for (int v = 0; v < 3; ++v) {
        unsigned long long ns[2] = {0, 0};
        for (int w = 0; w < 2; ++w) {
            if (v == 0) hipLaunchKernelGGL(k_bench<0>, dim3(1), dim3(64), 0, 0, dn, dT, reps, dns);
            else if (v == 1) hipLaunchKernelGGL(k_bench<1>, dim3(1), dim3(64), 0, 0, dn, dT, reps, dns);
            else hipLaunchKernelGGL(k_bench<2>, dim3(1), dim3(64), 0, 0, dn, dT, reps, dns);
            (void)hipMemcpy(ns, dns, 16, hipMemcpyDeviceToHost);
        }
        (void)hipMemcpy(T[v], dT, sizeof(T[v]), hipMemcpyDeviceToHost);
        printf("%-34s %7.0f ns per solve (one wave, %d dependent solves), status %llu\n",
               v == 0 ? "solve_update_wave (right-looking)" : v == 1 ? "left-looking reference" : "right-looking, rcp64_rn pivots", (double)ns[0] / reps,
               reps, ns[1]);
    }
    printf("pose after the chain: t = (%.17g, %.17g, %.17g), bitwise equal: %d %d\n", T[0][3], T[0][7],
           T[0][11], memcmp(T[0], T[1], sizeof(T[0])) == 0, memcmp(T[0], T[2], sizeof(T[0])) == 0);

    // random systems: A = sum of r outer products of random 6-vectors (rank r
    // = 1..8: rank < 6 is singular, its pivots fail), plus b, count, Sigma r^2
    {
        const int n = 1 << 18;
        std::vector<double> sys((size_t)n * kNeq);
        unsigned long long st = 0x5EEDull;
        auto rnd = [&] { st = st * 6364136223846793005ull + 1442695040888963407ull;
                         return ((double)(st >> 11) / 9007199254740992.0) * 2.0 - 1.0; };
        for (int c = 0; c < n; ++c) {
            double A[6][6] = {};
            const int rank = 1 + c % 8;
            const double scale = std::ldexp(1.0, (c / 8) % 40 - 20);
            for (int r = 0; r < rank * 3; ++r) {
                double v[6];
                for (int q = 0; q < 6; ++q) v[q] = rnd() * (q < 3 ? 1.0 : 0.01) * scale;
                if (r >= rank) for (int q = 0; q < 6; ++q) v[q] = 0.0;
                for (int a = 0; a < 6; ++a) for (int b2 = 0; b2 < 6; ++b2) A[a][b2] += v[a] * v[b2];
            }
            double* h = sys.data() + (size_t)c * kNeq;
            int k = 0;
            for (int a = 0; a < 6; ++a) for (int b2 = a; b2 < 6; ++b2) h[k++] = A[a][b2];
            for (int q = 0; q < 6; ++q) h[21 + q] = rnd() * 1e-3 * scale * scale;
            h[27] = 1.0;
            h[28] = (c % 97 == 0) ? 3.0 : 1000.0;  // some too-few-matches cases
        }
        double* dsys;
        (void)hipMalloc(&dsys, sys.size() * sizeof(double));
        (void)hipMemcpy(dsys, sys.data(), sys.size() * sizeof(double), hipMemcpyHostToDevice);
        (void)hipMemset(dns, 0, 16);
        for (int mode = 0; mode < 2; ++mode) {
            (void)hipMemset(dns, 0, 16);
            if (mode == 0) hipLaunchKernelGGL(k_cmp<0>, dim3(4096), dim3(64), 0, 0, dsys, n, dns);
            else hipLaunchKernelGGL(k_cmp<1>, dim3(4096), dim3(64), 0, 0, dsys, n, dns);
            unsigned long long b[2] = {0, 0};
            (void)hipMemcpy(b, dns, 16, hipMemcpyDeviceToHost);
            printf("right-looking vs %s: %llu mismatching cases of %d random systems "
                   "(%llu with a nonzero status)\n", mode == 0 ? "left-looking solve" : "rcp64_rn pivots",
                   b[0], n, b[1]);
        }
        (void)hipFree(dsys);
    }
    {
        const unsigned long long n = 1ull << 33;  // 8.6e9 reciprocals
        (void)hipMemset(dns, 0, 16);
        hipLaunchKernelGGL(k_rcp_test, dim3(16384), dim3(256), 0, 0, n, dns);
        unsigned long long b = 0;
        (void)hipMemcpy(&b, dns, 8, hipMemcpyDeviceToHost);
        printf("rcp64_rn vs 1.0 / d: %llu mismatches of %llu\n", b, n);
    }
    return 0;
}
