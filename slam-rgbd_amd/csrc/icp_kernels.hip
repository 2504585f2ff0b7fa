// icp_kernels.hip — MI355X (gfx950) kernels of the RGBD frame-to-frame ICP path.
//
// Hot path, reference boundary
// Youth.Source/AlgorithmModule/SLAM.cpp:54 (TrackRGBD, the pose maths this
// replaces) and viewerModule.c:341-345 (the back-projection formula):
//
//   k_prep    depth int16 -> XYZ planes (+ normals for target frames), one
//             64x16 tile per workgroup, the (16+2)x(64+2) back-projected
//             neighbourhood staged in LDS for the central-difference normals.
//   k_reduce  fused transform -> project -> gate -> residual -> Jacobian ->
//             29 fp64 accumulators per lane (exact fp32 products), wave
//             butterfly + LDS across waves -> one 29-double partial per
//             workgroup.  No atomics: deterministic.
//   k_solve   one wave per pair: sums the workgroup partials in fixed order,
//             LDL^T 6x6 solve, SE(3) exp, T <- exp(xi) T in fp64 on device,
//             writes the fp32 pose for the next k_reduce.  No host round trip
//             between iterations.
//
// Compiled with -ffp-contract=off: every fp32 expression rounds exactly as
// written, identical to the C oracle (oracle/icp_oracle.c) — XYZ, normals and
// association indices are bit-exact given the same fp32 pose.

#include <hip/hip_runtime.h>

#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <string>
#include <vector>

#include "youth_icp.h"

namespace {

// ----------------------------------------------------------------- layout --
// Frame f of the workspace: X plane at xyz + f*3*P, Y at +P, Z at +2P (SoA,
// fp32); normals likewise in nrm.  P = plane stride = round_up(N + 4, 256)
// floats, so float4 loads of the last pixels stay inside the (zeroed) pad.
constexpr int kTileW = 64;
constexpr int kTileH = 16;
constexpr int kPrepThreads = 256;
constexpr int kLdsW = kTileW + 2;
constexpr int kLdsH = kTileH + 2;

constexpr int kRedThreads = 256;
constexpr int kRedStep = kRedThreads * 4;  // pixels per workgroup loop step
constexpr int kNeq = YOUTH_NEQ;

struct Intr {
    float fx, fy, cx, cy, ds;
};

__device__ __forceinline__ void backproject(int d, int u, int v, const Intr& K,
                                            float& x, float& y, float& z)
{
    // viewerModule.c:341-345 with explicit intrinsics (bit-identical for
    // cx = W/2, cy = H/2, f = 570.3f, ds = 1000.0f).
    if (d > 0) {
        z = (float)d / K.ds;
        x = (((float)u - K.cx) * z) / K.fx;
        y = (((float)v - K.cy) * z) / K.fy;
    } else {
        x = 0.0f;
        y = 0.0f;
        z = 0.0f;
    }
}

// ------------------------------------------------------------------ k_prep --
// grid (ceil(W/64), ceil(H/16), n_frames); frame f reads depth from
// depth_a + f*N when f < n_a, else depth_b + (f - n_a)*N, and fills workspace
// frame out0 + f:
//   f <  xyz_end   -> SoA XYZ planes (the frame is a source);
//   f >= rec_first -> 16-byte records {z, nx, ny, nz} (the frame is a target),
//                     normals from the (16+2) x (64+2) back-projected
//                     neighbourhood staged in LDS.
__global__ __launch_bounds__(kPrepThreads) void k_prep(
    const int16_t* __restrict__ depth_a, const int16_t* __restrict__ depth_b, int n_a,
    int out0, int rec_first, int xyz_end, int W, int H, size_t P, Intr K,
    float* __restrict__ xyz, float4* __restrict__ recs)
{
    __shared__ float sX[kLdsH][kLdsW];
    __shared__ float sY[kLdsH][kLdsW];
    __shared__ float sZ[kLdsH][kLdsW];

    const int f = blockIdx.z;
    const size_t N = (size_t)W * (size_t)H;
    const int16_t* dep = (f < n_a) ? depth_a + (size_t)f * N : depth_b + (size_t)(f - n_a) * N;
    float* X = xyz + (size_t)(out0 + f) * 3 * P;
    float* Y = X + P;
    float* Z = Y + P;
    float4* R = recs + (size_t)(out0 + f) * P;
    const bool want_xyz = f < xyz_end;
    const int x0 = blockIdx.x * kTileW;
    const int y0 = blockIdx.y * kTileH;
    const int tx = threadIdx.x & 63;
    const int ty = threadIdx.x >> 6;

    if (f < rec_first) {
        // Source-only frame: XYZ planes, no neighbourhood needed.
#pragma unroll
        for (int k = 0; k < kTileH / 4; ++k) {
            const int gx = x0 + tx, gy = y0 + ty + 4 * k;
            if (gx < W && gy < H) {
                const size_t i = (size_t)gy * W + gx;
                float x, y, z;
                backproject(dep[i], gx, gy, K, x, y, z);
                X[i] = x;
                Y[i] = y;
                Z[i] = z;
            }
        }
        return;
    }

    // Target frame: stage the back-projected (kTileH+2) x (kTileW+2) halo tile.
    for (int e = threadIdx.x; e < kLdsH * kLdsW; e += kPrepThreads) {
        const int ly = e / kLdsW;
        const int lx = e - ly * kLdsW;
        const int gx = x0 - 1 + lx, gy = y0 - 1 + ly;
        float x = 0.0f, y = 0.0f, z = 0.0f;
        if (gx >= 0 && gx < W && gy >= 0 && gy < H)
            backproject(dep[(size_t)gy * W + gx], gx, gy, K, x, y, z);
        sX[ly][lx] = x;
        sY[ly][lx] = y;
        sZ[ly][lx] = z;
    }
    __syncthreads();

#pragma unroll
    for (int k = 0; k < kTileH / 4; ++k) {
        const int row = ty + 4 * k;
        const int gx = x0 + tx, gy = y0 + row;
        if (gx >= W || gy >= H) continue;
        const size_t i = (size_t)gy * W + gx;
        const int ly = row + 1, lx = tx + 1;
        const float px = sX[ly][lx], py = sY[ly][lx], pz = sZ[ly][lx];
        if (want_xyz) {
            X[i] = px;
            Y[i] = py;
            Z[i] = pz;
        }
        float nx = 0.0f, ny = 0.0f, nz = 0.0f;
        const bool inner = gx > 0 && gy > 0 && gx < W - 1 && gy < H - 1;
        if (inner) {
            const float zl = sZ[ly][lx - 1], zr = sZ[ly][lx + 1];
            const float zu = sZ[ly - 1][lx], zd = sZ[ly + 1][lx];
            if (pz > 0.0f && zl > 0.0f && zr > 0.0f && zu > 0.0f && zd > 0.0f) {
                const float ax = sX[ly][lx + 1] - sX[ly][lx - 1];
                const float ay = sY[ly][lx + 1] - sY[ly][lx - 1];
                const float az = zr - zl;
                const float bx = sX[ly + 1][lx] - sX[ly - 1][lx];
                const float by = sY[ly + 1][lx] - sY[ly - 1][lx];
                const float bz = zd - zu;
                const float cx = ay * bz - az * by;
                const float cy = az * bx - ax * bz;
                const float cz = ax * by - ay * bx;
                const float len2 = (cx * cx + cy * cy) + cz * cz;
                if (len2 > 0.0f) {
                    const float len = sqrtf(len2);  // correctly rounded (checked in .s)
                    nx = cx / len;
                    ny = cy / len;
                    nz = cz / len;
                    if (((nx * px + ny * py) + nz * pz) > 0.0f) {
                        nx = -nx;
                        ny = -ny;
                        nz = -nz;
                    }
                }
            }
        }
        R[i] = make_float4(pz, nx, ny, nz);
    }
}

// ---------------------------------------------------------------- k_reduce --
// Fused transform -> project -> gate -> residual -> Jacobian -> fp64
// normal-equation accumulation (spec a7-a9).  Data layout:
//   source  SoA XYZ planes: three dwordx4 loads per lane per 4 pixels;
//   target  one 16-byte record {z, nx, ny, nz} per pixel: ONE aligned dwordx4
//           fetch per correspondence; the target's x, y are recomputed from z
//           with k_prep's back-projection expression, so they are
//           bit-identical to the planes k_prep would have stored.
// 28 B/px per iteration instead of 36 B/px with six 4-byte gathers
// (tools/kbench: 175 -> 117 us for 64 pairs; sums bit-identical).
// Accumulators are fp64 fed with exact fp32 products: the result equals the
// oracle's row-major fp64 sum up to fp64 summation order.
struct PairMap {
    int src0, tgt0;  // pair p: source frame src0 + p, target frame tgt0 + p
};

template <typename Acc>
__device__ __forceinline__ void acc_fma(Acc& a, float x, float y);
template <>
__device__ __forceinline__ void acc_fma<double>(double& a, float x, float y)
{
    a = fma((double)x, (double)y, a);
}

template <bool kAssoc>
__device__ __forceinline__ void process4(const float xs[4], const float ys[4],
                                         const float zs[4], int i, int end,
                                         const float* __restrict__ T, const Intr& K, int W, int H,
                                         float thr2, const float4* __restrict__ rec, double* acc,
                                         int32_t* __restrict__ arow)
{
    // spec a7: P' = R P + t, fixed order, no FMA; projective association
    float qx[4], qy[4], qz[4], fu[4], fv[4];
    int j[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const float sx = xs[q], sy = ys[q], sz = (i + q) < end ? zs[q] : 0.0f;
        qx[q] = ((T[0] * sx + T[1] * sy) + T[2] * sz) + T[3];
        qy[q] = ((T[4] * sx + T[5] * sy) + T[6] * sz) + T[7];
        qz[q] = ((T[8] * sx + T[9] * sy) + T[10] * sz) + T[11];
        j[q] = -1;
        fu[q] = 0.0f;
        fv[q] = 0.0f;
        if (sz > 0.0f && qz[q] > 0.0f) {
            const float u = floorf((((K.fx * qx[q]) / qz[q]) + K.cx) + 0.5f);
            const float v = floorf((((K.fy * qy[q]) / qz[q]) + K.cy) + 0.5f);
            if (u >= 0.0f && u < (float)W && v >= 0.0f && v < (float)H) {
                j[q] = (int)v * W + (int)u;
                fu[q] = u;
                fv[q] = v;
            }
        }
    }
    // all four fetches issued back to back from clamped indices (no branch)
    float4 t[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) t[q] = rec[j[q] >= 0 ? j[q] : 0];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const float tz = t[q].x;
        const float tx = ((fu[q] - K.cx) * tz) / K.fx;  // = k_prep's X of pixel (u', v')
        const float ty = ((fv[q] - K.cy) * tz) / K.fy;
        const float nx = t[q].y, ny = t[q].z, nz = t[q].w;
        const float dx = qx[q] - tx, dy = qy[q] - ty, dz = qz[q] - tz;
        const float d2 = (dx * dx + dy * dy) + dz * dz;
        const bool nvalid = !(nx == 0.0f && ny == 0.0f && nz == 0.0f);
        const bool ok = j[q] >= 0 && tz > 0.0f && nvalid && d2 < thr2;
        if (kAssoc && (i + q) < end) arow[i + q] = ok ? j[q] : -1;
        // spec a8: r = n.(P' - P_t); J = [P' x n, n]  (zeros when unmatched)
        const float n0 = ok ? nx : 0.0f, n1 = ok ? ny : 0.0f, n2 = ok ? nz : 0.0f;
        const float r = ok ? (nx * dx + ny * dy) + nz * dz : 0.0f;
        float Jf[6];
        Jf[0] = qy[q] * n2 - qz[q] * n1;
        Jf[1] = qz[q] * n0 - qx[q] * n2;
        Jf[2] = qx[q] * n1 - qy[q] * n0;
        Jf[3] = n0;
        Jf[4] = n1;
        Jf[5] = n2;
        // spec a9: fp32 products are exact in fp64; one rounding per add
        int k = 0;
#pragma unroll
        for (int a = 0; a < 6; ++a)
#pragma unroll
            for (int b = a; b < 6; ++b) {
                acc_fma<double>(acc[k], Jf[a], Jf[b]);
                ++k;
            }
#pragma unroll
        for (int a = 0; a < 6; ++a) acc_fma<double>(acc[21 + a], Jf[a], r);
        acc_fma<double>(acc[27], r, r);
        acc[28] += ok ? 1.0 : 0.0;
    }
}

// Wave butterfly (lane-symmetric: every lane ends with the same sum), then
// waves in fixed order through LDS; one 29-double partial per workgroup.
__device__ __forceinline__ void block_reduce_store(double* acc, double (*red)[kNeq],
                                                   double* __restrict__ out)
{
#pragma unroll
    for (int k = 0; k < kNeq; ++k) {
        double v = acc[k];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        acc[k] = v;
    }
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int k = 0; k < kNeq; ++k) red[wave][k] = acc[k];
    }
    __syncthreads();
    if (threadIdx.x < kNeq) {
        const int k = threadIdx.x;
        double s = red[0][k];
#pragma unroll
        for (int w = 1; w < kRedThreads / 64; ++w) s += red[w][k];
        out[k] = s;
    }
}

// grid (nblk, n_pairs); workgroup b of pair p covers pixels
// [b*chunk, min((b+1)*chunk, N)); chunk is a multiple of kRedStep.
template <bool kAssoc>
__global__ __launch_bounds__(kRedThreads) void k_reduce(
    const float* __restrict__ xyz, const float4* __restrict__ recs, size_t P, PairMap pm,
    const float* __restrict__ T32, int W, int H, Intr K, float thr2, int chunk,
    double* __restrict__ partials, int32_t* __restrict__ assoc)
{
    __shared__ double red[kRedThreads / 64][kNeq];
    const int p = blockIdx.y;
    const int b = blockIdx.x;
    const int N = W * H;
    const float* sX = xyz + (size_t)(pm.src0 + p) * 3 * P;
    const float* sY = sX + P;
    const float* sZ = sY + P;
    const float4* rec = recs + (size_t)(pm.tgt0 + p) * P;
    float T[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) T[k] = T32[p * 12 + k];

    double acc[kNeq];
#pragma unroll
    for (int k = 0; k < kNeq; ++k) acc[k] = 0.0;

    const int start = b * chunk;
    const int end = min(start + chunk, N);
    int32_t* arow = kAssoc ? assoc + (size_t)p * N : nullptr;
    for (int i = start + threadIdx.x * 4; i < end; i += kRedStep) {
        // i % 4 == 0 and P >= N + 4: the float4 never leaves the zeroed pad
        const float4 x4 = *reinterpret_cast<const float4*>(sX + i);
        const float4 y4 = *reinterpret_cast<const float4*>(sY + i);
        const float4 z4 = *reinterpret_cast<const float4*>(sZ + i);
        const float xs[4] = {x4.x, x4.y, x4.z, x4.w};
        const float ys[4] = {y4.x, y4.y, y4.z, y4.w};
        const float zs[4] = {z4.x, z4.y, z4.z, z4.w};
        process4<kAssoc>(xs, ys, zs, i, end, T, K, W, H, thr2, rec, acc, arow);
    }
    block_reduce_store(acc, red, partials + ((size_t)p * gridDim.x + b) * kNeq);
}


// ----------------------------------------------------------------- k_solve --
// LDL^T + SE(3) exp, same algorithm and evaluation order as oracle_solve /
// oracle_se3_exp (oracle/icp_oracle.c).
__device__ int solve6(const double* neq, double xi[6])
{
    for (int i = 0; i < 6; ++i) xi[i] = 0.0;
    if (!(neq[28] >= 6.0)) return YOUTH_STATUS_FEW_MATCHES;
    double A[6][6];
    int k = 0;
    for (int a = 0; a < 6; ++a)
        for (int b = a; b < 6; ++b) {
            A[a][b] = neq[k];
            A[b][a] = neq[k];
            ++k;
        }
    double maxd = 0.0;
    for (int a = 0; a < 6; ++a)
        if (A[a][a] > maxd) maxd = A[a][a];
    if (!(maxd > 0.0)) return YOUTH_STATUS_DEGENERATE;
    const double eps = 1e-12 * maxd;
    double L[6][6], D[6];
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) L[i][j] = 0.0;
    for (int j = 0; j < 6; ++j) {
        double d = A[j][j];
        for (int m = 0; m < j; ++m) d -= (L[j][m] * L[j][m]) * D[m];
        if (!(d > eps)) return YOUTH_STATUS_DEGENERATE;
        D[j] = d;
        L[j][j] = 1.0;
        for (int i = j + 1; i < 6; ++i) {
            double s = A[i][j];
            for (int m = 0; m < j; ++m) s -= (L[i][m] * L[j][m]) * D[m];
            L[i][j] = s / d;
        }
    }
    double y[6], x[6];
    for (int i = 0; i < 6; ++i) {
        double s = -neq[21 + i];
        for (int m = 0; m < i; ++m) s -= L[i][m] * y[m];
        y[i] = s;
    }
    for (int i = 0; i < 6; ++i) y[i] = y[i] / D[i];
    for (int i = 5; i >= 0; --i) {
        double s = y[i];
        for (int m = i + 1; m < 6; ++m) s -= L[m][i] * x[m];
        x[i] = s;
    }
    for (int i = 0; i < 6; ++i) xi[i] = x[i];
    return 0;
}

__device__ void se3_exp_left(const double xi[6], double* T)
{
    const double wx = xi[0], wy = xi[1], wz = xi[2];
    const double th2 = (wx * wx + wy * wy) + wz * wz;
    double a, b, c;
    if (th2 < 1e-10) {
        a = 1.0 - th2 / 6.0;
        b = 0.5 - th2 / 24.0;
        c = 1.0 / 6.0 - th2 / 120.0;
    } else {
        const double th = sqrt(th2);
        double s, co;
        sincos(th, &s, &co);
        a = s / th;
        b = (1.0 - co) / th2;
        c = (th - s) / (th2 * th);
    }
    const double Km[3][3] = {{0.0, -wz, wy}, {wz, 0.0, -wx}, {-wy, wx, 0.0}};
    double K2[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            K2[i][j] = (Km[i][0] * Km[0][j] + Km[i][1] * Km[1][j]) + Km[i][2] * Km[2][j];
    double E[3][4];
    for (int i = 0; i < 3; ++i) {
        double V[3];
        for (int j = 0; j < 3; ++j) {
            const double I = (i == j) ? 1.0 : 0.0;
            E[i][j] = (I + a * Km[i][j]) + b * K2[i][j];
            V[j] = (I + b * Km[i][j]) + c * K2[i][j];
        }
        E[i][3] = (V[0] * xi[3] + V[1] * xi[4]) + V[2] * xi[5];
    }
    double O[12];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 4; ++j) {
            double s = (E[i][0] * T[0 * 4 + j] + E[i][1] * T[1 * 4 + j]) + E[i][2] * T[2 * 4 + j];
            if (j == 3) s += E[i][3];
            O[i * 4 + j] = s;
        }
    for (int i = 0; i < 12; ++i) T[i] = O[i];
}

// Sum the nblk partials of pair p in a fixed order: lanes 0..28 take the
// first half of the workgroups, lanes 32..60 the second, then one add.
__device__ __forceinline__ void sum_partials(const double* __restrict__ part, int nblk,
                                             double* sh)
{
    const int lane = threadIdx.x;
    const int half = (nblk + 1) >> 1;
    const int k = lane & 31;
    double s = 0.0;
    if (k < kNeq) {
        const int b0 = lane < 32 ? 0 : half;
        const int b1 = lane < 32 ? half : nblk;
        for (int bb = b0; bb < b1; ++bb) s += part[(size_t)bb * kNeq + k];
    }
    const double hi = __shfl_down(s, 32, 64);
    if (lane < kNeq) sh[lane] = s + hi;
    __syncthreads();
}

__device__ __forceinline__ void solve_update(const double* neq, double* T64, float* T32,
                                             int32_t* status)
{
    double xi[6];
    const int st = solve6(neq, xi);
    double T[16];
    for (int i = 0; i < 16; ++i) T[i] = T64[i];
    if (st == 0) se3_exp_left(xi, T);
    for (int i = 0; i < 12; ++i) {
        T64[i] = T[i];
        T32[i] = (float)T[i];
    }
    *status |= st;
}

// grid n_pairs, one wave each.
__global__ __launch_bounds__(64) void k_solve(const double* __restrict__ partials,
                                              int nblk, int it, int iters,
                                              double* __restrict__ T64,
                                              float* __restrict__ T32,
                                              int32_t* __restrict__ status,
                                              double* __restrict__ stats,
                                              double* __restrict__ neq_out)
{
    __shared__ double sh[kNeq];
    const int p = blockIdx.x;
    sum_partials(partials + (size_t)p * nblk * kNeq, nblk, sh);
    if (threadIdx.x == 0) {
        if (stats) {
            stats[((size_t)p * iters + it) * 2 + 0] = sh[28];
            stats[((size_t)p * iters + it) * 2 + 1] = sh[27];
        }
        if (neq_out) {
            for (int k = 0; k < kNeq; ++k) neq_out[(size_t)p * kNeq + k] = sh[k];
        } else {
            solve_update(sh, T64 + (size_t)p * 16, T32 + (size_t)p * 12, status + p);
        }
    }
}

// Solve from a given record (stage-level validation entry point).
__global__ void k_solve_neq(const double* __restrict__ neq, double* T64, float* T32,
                            int32_t* status)
{
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        double sh[kNeq];
        for (int k = 0; k < kNeq; ++k) sh[k] = neq[k];
        *status = 0;
        solve_update(sh, T64, T32, status);
    }
}

// T64 <- T_init (or identity), T32 <- float(T64), status <- 0.
__global__ void k_init(const double* __restrict__ T_init, int n, double* T64, float* T32,
                       int32_t* status)
{
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    for (int i = 0; i < 16; ++i) {
        const double v = T_init ? T_init[(size_t)p * 16 + i] : ((i % 5) == 0 ? 1.0 : 0.0);
        T64[(size_t)p * 16 + i] = v;
        if (i < 12) T32[(size_t)p * 12 + i] = (float)v;
    }
    status[p] = 0;
}

// [p][16] fp32 4x4 export.
__global__ void k_export(const double* __restrict__ T64, int n, float* __restrict__ out)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * 16) return;
    const int i = t & 15;
    out[t] = i < 12 ? (float)T64[(size_t)(t >> 4) * 16 + i] : (i == 15 ? 1.0f : 0.0f);
}

}  // namespace

// =============================================================== host side ==

static thread_local std::string g_last_error;

__attribute__((format(printf, 2, 3))) static int set_error(int code, const char* fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

#define HIP_TRY(expr)                                                                    \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess)                                                            \
            return set_error(YOUTH_EHIP, "%s (line %d)", hipGetErrorString(e_), __LINE__); \
    } while (0)

struct EventPair {
    hipEvent_t a, b;
    int kind;
};

struct youth_icp_ctx {
    int device = 0;
    int W = 0, H = 0, N = 0;
    size_t P = 0;
    int max_frames = 0;
    Intr K{};
    youth_icp_params prm{};
    hipStream_t stream = nullptr;

    int16_t* d_depth = nullptr;  // [max_frames][N] staging for host-side APIs
    float* d_xyz = nullptr;      // [max_frames][3][P]
    float4* d_rec = nullptr;     // [max_frames][P] target records {z, nx, ny, nz}
    double* d_T64 = nullptr;     // [max_frames][16]
    float* d_T32 = nullptr;      // [max_frames][12]
    int32_t* d_status = nullptr; // [max_frames]
    double* d_Tinit = nullptr;   // [max_frames][16]
    double* d_stats = nullptr;   // [max_frames][stats_iters][2]
    int stats_iters = 0;
    double* d_partials = nullptr;
    size_t partials_cap = 0;  // doubles
    double* d_neq = nullptr;  // [max_frames][29]
    int32_t* d_assoc = nullptr;
    float* d_Tout = nullptr;  // [max_frames][16]

    int last_pairs = 0;
    int last_iters = 0;
    hipStream_t last_stream = nullptr;

    int track_ref = -1;  // ring slot (0/1) of the tracker's reference frame

    bool timing = false;
    std::vector<EventPair> ev_live;
    std::vector<EventPair> ev_free;
    double t_ms[3] = {0, 0, 0};
    int t_n[3] = {0, 0, 0};
};

static int reduce_geometry(const youth_icp_ctx* c, int n_pairs, int* chunk_out)
{
    // ~2048 workgroups in flight over the batch, at least 8 px per lane.
    const int target_blocks = 2048;
    int nb = (target_blocks + n_pairs - 1) / n_pairs;
    const int max_nb = (c->N + 2 * kRedStep - 1) / (2 * kRedStep);
    if (nb > max_nb) nb = max_nb;
    if (nb < 1) nb = 1;
    int chunk = (c->N + nb - 1) / nb;
    chunk = (chunk + kRedStep - 1) / kRedStep * kRedStep;
    nb = (c->N + chunk - 1) / chunk;
    *chunk_out = chunk;
    return nb;
}

static int ensure_partials(youth_icp_ctx* c, size_t doubles)
{
    if (doubles <= c->partials_cap) return YOUTH_OK;
    if (c->d_partials) HIP_TRY(hipFree(c->d_partials));
    c->d_partials = nullptr;
    c->partials_cap = 0;
    HIP_TRY(hipMalloc(&c->d_partials, doubles * sizeof(double)));
    c->partials_cap = doubles;
    return YOUTH_OK;
}

static int ensure_stats(youth_icp_ctx* c, int iters)
{
    if (iters <= c->stats_iters) return YOUTH_OK;
    if (c->d_stats) HIP_TRY(hipFree(c->d_stats));
    c->d_stats = nullptr;
    HIP_TRY(hipMalloc(&c->d_stats, (size_t)c->max_frames * iters * 2 * sizeof(double)));
    c->stats_iters = iters;
    return YOUTH_OK;
}

static int ensure_assoc(youth_icp_ctx* c)
{
    if (c->d_assoc) return YOUTH_OK;
    HIP_TRY(hipMalloc(&c->d_assoc, (size_t)c->max_frames * c->N * sizeof(int32_t)));
    return YOUTH_OK;
}

static int ev_begin(youth_icp_ctx* c, hipStream_t s, EventPair* ep, int kind)
{
    if (!c->timing) return YOUTH_OK;
    if (c->ev_free.empty()) {
        EventPair e{};
        HIP_TRY(hipEventCreate(&e.a));
        HIP_TRY(hipEventCreate(&e.b));
        c->ev_free.push_back(e);
    }
    *ep = c->ev_free.back();
    c->ev_free.pop_back();
    ep->kind = kind;
    HIP_TRY(hipEventRecord(ep->a, s));
    return YOUTH_OK;
}

static int ev_end(youth_icp_ctx* c, hipStream_t s, EventPair* ep)
{
    if (!c->timing) return YOUTH_OK;
    HIP_TRY(hipEventRecord(ep->b, s));
    c->ev_live.push_back(*ep);
    return YOUTH_OK;
}

static int ev_harvest(youth_icp_ctx* c)
{
    for (auto& e : c->ev_live) {
        HIP_TRY(hipEventSynchronize(e.b));
        float ms = 0.0f;
        HIP_TRY(hipEventElapsedTime(&ms, e.a, e.b));
        c->t_ms[e.kind] += ms;
        c->t_n[e.kind] += 1;
        c->ev_free.push_back(e);
    }
    c->ev_live.clear();
    return YOUTH_OK;
}

// Launch k_prep for frames [out0, out0 + n_frames).
static int launch_prep(youth_icp_ctx* c, hipStream_t s, const int16_t* da, const int16_t* db,
                       int n_a, int out0, int n_frames, int rec_first, int xyz_end)
{
    if (n_frames <= 0) return YOUTH_OK;
    dim3 grid((c->W + kTileW - 1) / kTileW, (c->H + kTileH - 1) / kTileH, n_frames);
    EventPair ep{};
    int rc = ev_begin(c, s, &ep, 2);
    if (rc) return rc;
    hipLaunchKernelGGL(k_prep, grid, dim3(kPrepThreads), 0, s, da, db, n_a, out0, rec_first,
                       xyz_end, c->W, c->H, c->P, c->K, c->d_xyz, c->d_rec);
    HIP_TRY(hipGetLastError());
    return ev_end(c, s, &ep);
}

static int launch_reduce(youth_icp_ctx* c, hipStream_t s, PairMap pm, int n_pairs,
                         bool assoc, int* nblk_out)
{
    int chunk = 0;
    const int nb = reduce_geometry(c, n_pairs, &chunk);
    int rc = ensure_partials(c, (size_t)nb * n_pairs * kNeq);
    if (rc) return rc;
    const float thr2 = c->prm.dist_thresh * c->prm.dist_thresh;
    dim3 grid(nb, n_pairs);
    EventPair ep{};
    rc = ev_begin(c, s, &ep, 0);
    if (rc) return rc;
    if (assoc) {
        rc = ensure_assoc(c);
        if (rc) return rc;
        hipLaunchKernelGGL(k_reduce<true>, grid, dim3(kRedThreads), 0, s, c->d_xyz, c->d_rec,
                           c->P, pm, c->d_T32, c->W, c->H, c->K, thr2, chunk, c->d_partials,
                           c->d_assoc);
    } else {
        hipLaunchKernelGGL(k_reduce<false>, grid, dim3(kRedThreads), 0, s, c->d_xyz, c->d_rec,
                           c->P, pm, c->d_T32, c->W, c->H, c->K, thr2, chunk, c->d_partials,
                           (int32_t*)nullptr);
    }
    HIP_TRY(hipGetLastError());
    *nblk_out = nb;
    return ev_end(c, s, &ep);
}

static int run_iterations(youth_icp_ctx* c, hipStream_t s, PairMap pm, int n_pairs,
                          const double* T_init_host)
{
    const int iters = c->prm.iters;
    int rc = ensure_stats(c, iters > 0 ? iters : 1);
    if (rc) return rc;
    const double* dTi = nullptr;
    if (T_init_host) {
        HIP_TRY(hipMemcpyAsync(c->d_Tinit, T_init_host, (size_t)n_pairs * 16 * sizeof(double),
                               hipMemcpyHostToDevice, s));
        dTi = c->d_Tinit;
    }
    hipLaunchKernelGGL(k_init, dim3((n_pairs + 63) / 64), dim3(64), 0, s, dTi, n_pairs,
                       c->d_T64, c->d_T32, c->d_status);
    HIP_TRY(hipGetLastError());
    for (int it = 0; it < iters; ++it) {
        int nb = 0;
        rc = launch_reduce(c, s, pm, n_pairs, false, &nb);
        if (rc) return rc;
        EventPair ep{};
        rc = ev_begin(c, s, &ep, 1);
        if (rc) return rc;
        hipLaunchKernelGGL(k_solve, dim3(n_pairs), dim3(64), 0, s, c->d_partials, nb, it, iters,
                           c->d_T64, c->d_T32, c->d_status, c->d_stats, (double*)nullptr);
        HIP_TRY(hipGetLastError());
        rc = ev_end(c, s, &ep);
        if (rc) return rc;
    }
    c->last_pairs = n_pairs;
    c->last_iters = iters;
    c->last_stream = s;
    return YOUTH_OK;
}

static int export_poses(youth_icp_ctx* c, hipStream_t s, int n_pairs, float* d_T_out)
{
    if (!d_T_out) return YOUTH_OK;
    hipLaunchKernelGGL(k_export, dim3((n_pairs * 16 + 255) / 256), dim3(256), 0, s, c->d_T64,
                       n_pairs, d_T_out);
    HIP_TRY(hipGetLastError());
    return YOUTH_OK;
}

static hipStream_t pick_stream(youth_icp_ctx* c, void* stream)
{
    return stream ? (hipStream_t)stream : c->stream;
}

static int bind_device(youth_icp_ctx* c)
{
    HIP_TRY(hipSetDevice(c->device));
    return YOUTH_OK;
}

extern "C" {

youth_intrinsics youth_default_intrinsics(int width, int height)
{
    youth_intrinsics K;
    K.fx = 570.3f;  // viewerModule.c:344-345, astra_orb_slam3_rgbd.yaml:9-10
    K.fy = 570.3f;
    K.cx = (float)(width / 2);  // integer W/2 as in viewerModule.c:344
    K.cy = (float)(height / 2);
    K.depth_scale = 1000.0f;  // astra_orb_slam3_rgbd.yaml:35
    return K;
}

youth_icp_params youth_default_params(void)
{
    youth_icp_params p;
    p.iters = 10;
    p.dist_thresh = 0.10f;
    return p;
}

const char* youth_icp_last_error(void) { return g_last_error.c_str(); }

int youth_icp_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

void youth_icp_destroy(youth_icp_ctx* c)
{
    if (!c) return;
    // best-effort teardown: errors here cannot be reported to anyone useful
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (auto* v : {&c->ev_live, &c->ev_free})
        for (auto& e : *v) {
            (void)hipEventDestroy(e.a);
            (void)hipEventDestroy(e.b);
        }
    void* bufs[] = {c->d_depth, c->d_xyz,   c->d_rec,      c->d_T64, c->d_T32,   c->d_status,
                    c->d_Tinit, c->d_stats, c->d_partials, c->d_neq, c->d_assoc, c->d_Tout};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

youth_icp_ctx* youth_icp_create(int device, int W, int H, int max_frames,
                                const youth_intrinsics* K, const youth_icp_params* P)
{
    if (W < 3 || H < 3 || max_frames < 2 || (long long)W * H > (1LL << 30)) {
        set_error(YOUTH_EINVAL, "youth_icp_create: bad size %d", W);
        return nullptr;
    }
    int ndev = youth_icp_device_count();
    if (ndev <= 0 || device < 0 || device >= ndev) {
        set_error(YOUTH_ENODEV, "youth_icp_create: no HIP device %d", device);
        return nullptr;
    }
    auto* c = new youth_icp_ctx();
    c->device = device;
    c->W = W;
    c->H = H;
    c->N = W * H;
    c->P = ((size_t)c->N + 4 + 255) / 256 * 256;
    c->max_frames = max_frames;
    const youth_intrinsics Kd = K ? *K : youth_default_intrinsics(W, H);
    c->K = Intr{Kd.fx, Kd.fy, Kd.cx, Kd.cy, Kd.depth_scale};
    c->prm = P ? *P : youth_default_params();
    auto fail = [&](const char* what, hipError_t e) -> youth_icp_ctx* {
        set_error(YOUTH_EHIP, "youth_icp_create: %s (%d)", what, (int)e);
        youth_icp_destroy(c);
        return nullptr;
    };
    hipError_t e;
    if ((e = hipSetDevice(device)) != hipSuccess) return fail("hipSetDevice", e);
    if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess)
        return fail("hipStreamCreate", e);
    const size_t MF = (size_t)max_frames;
    const size_t plane_bytes = 3 * c->P * sizeof(float) * MF;
    const size_t rec_bytes = c->P * sizeof(float4) * MF;
    if ((e = hipMalloc(&c->d_depth, MF * c->N * sizeof(int16_t))) != hipSuccess)
        return fail("hipMalloc depth", e);
    if ((e = hipMalloc(&c->d_xyz, plane_bytes)) != hipSuccess) return fail("hipMalloc xyz", e);
    if ((e = hipMalloc(&c->d_rec, rec_bytes)) != hipSuccess) return fail("hipMalloc rec", e);
    // the pad beyond N of every plane must read as an invalid point (Z = 0)
    if ((e = hipMemset(c->d_xyz, 0, plane_bytes)) != hipSuccess) return fail("memset xyz", e);
    if ((e = hipMemset(c->d_rec, 0, rec_bytes)) != hipSuccess) return fail("memset rec", e);
    if ((e = hipMalloc(&c->d_T64, MF * 16 * sizeof(double))) != hipSuccess)
        return fail("hipMalloc T64", e);
    if ((e = hipMalloc(&c->d_T32, MF * 12 * sizeof(float))) != hipSuccess)
        return fail("hipMalloc T32", e);
    if ((e = hipMalloc(&c->d_status, MF * sizeof(int32_t))) != hipSuccess)
        return fail("hipMalloc status", e);
    if ((e = hipMalloc(&c->d_Tinit, MF * 16 * sizeof(double))) != hipSuccess)
        return fail("hipMalloc Tinit", e);
    if ((e = hipMalloc(&c->d_neq, MF * kNeq * sizeof(double))) != hipSuccess)
        return fail("hipMalloc neq", e);
    if ((e = hipMalloc(&c->d_Tout, MF * 16 * sizeof(float))) != hipSuccess)
        return fail("hipMalloc Tout", e);
    if ((e = hipDeviceSynchronize()) != hipSuccess) return fail("sync", e);
    if (ensure_stats(c, c->prm.iters > 0 ? c->prm.iters : 1) != YOUTH_OK) {
        youth_icp_destroy(c);
        return nullptr;
    }
    return c;
}

int youth_icp_align_pairs_device(youth_icp_ctx* c, const int16_t* d_src, const int16_t* d_dst,
                                 int n_pairs, const double* T_init, float* d_T_out,
                                 void* stream)
{
    if (!c || !d_src || !d_dst || n_pairs <= 0 || 2 * n_pairs > c->max_frames)
        return set_error(YOUTH_EINVAL, "align_pairs: bad arguments %d", n_pairs);
    int rc = bind_device(c);
    if (rc) return rc;
    hipStream_t s = pick_stream(c, stream);
    // frames [0, n): sources (XYZ only); [n, 2n): targets (XYZ + normals)
    rc = launch_prep(c, s, d_src, d_dst, n_pairs, 0, 2 * n_pairs, n_pairs, n_pairs);
    if (rc) return rc;
    rc = run_iterations(c, s, PairMap{0, n_pairs}, n_pairs, T_init);
    if (rc) return rc;
    return export_poses(c, s, n_pairs, d_T_out);
}

int youth_icp_align_sequence_device(youth_icp_ctx* c, const int16_t* d_frames, int n_frames,
                                    float* d_T_out, void* stream)
{
    if (!c || !d_frames || n_frames < 2 || n_frames > c->max_frames)
        return set_error(YOUTH_EINVAL, "align_sequence: bad arguments %d", n_frames);
    int rc = bind_device(c);
    if (rc) return rc;
    hipStream_t s = pick_stream(c, stream);
    rc = launch_prep(c, s, d_frames, d_frames, n_frames, 0, n_frames, 0, n_frames);
    if (rc) return rc;
    // pair k: source frame k+1, target frame k
    rc = run_iterations(c, s, PairMap{1, 0}, n_frames - 1, nullptr);
    if (rc) return rc;
    return export_poses(c, s, n_frames - 1, d_T_out);
}

int youth_icp_sync(youth_icp_ctx* c, void* stream)
{
    if (!c) return set_error(YOUTH_EINVAL, "sync: null context");
    int rc = bind_device(c);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(pick_stream(c, stream)));
    return YOUTH_OK;
}

int youth_icp_get_poses(youth_icp_ctx* c, int n, double* T64, float* T32, int32_t* status)
{
    if (!c || n < 0 || n > c->max_frames)
        return set_error(YOUTH_EINVAL, "get_poses: bad arguments %d", n);
    int rc = bind_device(c);
    if (rc) return rc;
    hipStream_t s = c->last_stream ? c->last_stream : c->stream;
    if (T64)
        HIP_TRY(hipMemcpyAsync(T64, c->d_T64, (size_t)n * 16 * sizeof(double),
                               hipMemcpyDeviceToHost, s));
    if (T32) {
        rc = export_poses(c, s, n, c->d_Tout);
        if (rc) return rc;
        HIP_TRY(hipMemcpyAsync(T32, c->d_Tout, (size_t)n * 16 * sizeof(float),
                               hipMemcpyDeviceToHost, s));
    }
    if (status)
        HIP_TRY(hipMemcpyAsync(status, c->d_status, (size_t)n * sizeof(int32_t),
                               hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return YOUTH_OK;
}

int youth_icp_get_stats(youth_icp_ctx* c, int n, int iters, double* count, double* sum_r2)
{
    if (!c || n < 0 || n > c->max_frames || iters != c->last_iters || iters > c->stats_iters)
        return set_error(YOUTH_EINVAL, "get_stats: bad arguments %d", iters);
    int rc = bind_device(c);
    if (rc) return rc;
    std::vector<double> st((size_t)n * iters * 2);
    hipStream_t s = c->last_stream ? c->last_stream : c->stream;
    HIP_TRY(hipMemcpyAsync(st.data(), c->d_stats, st.size() * sizeof(double),
                           hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    for (size_t i = 0; i < (size_t)n * iters; ++i) {
        if (count) count[i] = st[2 * i];
        if (sum_r2) sum_r2[i] = st[2 * i + 1];
    }
    return YOUTH_OK;
}

int youth_icp_set_timing(youth_icp_ctx* c, int enable)
{
    if (!c) return set_error(YOUTH_EINVAL, "set_timing: null context");
    int rc = bind_device(c);
    if (rc) return rc;
    rc = ev_harvest(c);
    if (rc) return rc;
    c->timing = enable != 0;
    for (int k = 0; k < 3; ++k) {
        c->t_ms[k] = 0.0;
        c->t_n[k] = 0;
    }
    return YOUTH_OK;
}

int youth_icp_get_timing(youth_icp_ctx* c, int kind, double* total_ms, int* launches)
{
    if (!c || kind < 0 || kind > 2) return set_error(YOUTH_EINVAL, "get_timing: bad kind %d", kind);
    int rc = bind_device(c);
    if (rc) return rc;
    rc = ev_harvest(c);
    if (rc) return rc;
    if (total_ms) *total_ms = c->t_ms[kind];
    if (launches) *launches = c->t_n[kind];
    return YOUTH_OK;
}

int youth_icp_prepare_host(youth_icp_ctx* c, const int16_t* depth, int n_frames,
                           int want_normals, float* X, float* Y, float* Z, float* NX,
                           float* NY, float* NZ)
{
    if (!c || !depth || n_frames <= 0 || n_frames > c->max_frames)
        return set_error(YOUTH_EINVAL, "prepare_host: bad arguments %d", n_frames);
    int rc = bind_device(c);
    if (rc) return rc;
    hipStream_t s = c->stream;
    const size_t N = c->N;
    HIP_TRY(hipMemcpyAsync(c->d_depth, depth, (size_t)n_frames * N * sizeof(int16_t),
                           hipMemcpyHostToDevice, s));
    rc = launch_prep(c, s, c->d_depth, c->d_depth, n_frames, 0, n_frames,
                     want_normals ? 0 : n_frames, n_frames);
    if (rc) return rc;
    float* outs[6] = {X, Y, Z, NX, NY, NZ};
    for (int f = 0; f < n_frames; ++f)
        for (int k = 0; k < 6; ++k) {
            if (!outs[k] || (k >= 3 && !want_normals)) continue;
            float* dst = outs[k] + (size_t)f * N;
            if (k < 3) {
                const float* base = c->d_xyz + (size_t)f * 3 * c->P + (size_t)k * c->P;
                HIP_TRY(hipMemcpyAsync(dst, base, N * sizeof(float), hipMemcpyDeviceToHost, s));
            } else {  // component k-2 of the {z, nx, ny, nz} records
                const float* base = reinterpret_cast<const float*>(c->d_rec + (size_t)f * c->P) + (k - 2);
                HIP_TRY(hipMemcpy2DAsync(dst, sizeof(float), base, sizeof(float4), sizeof(float), N,
                                         hipMemcpyDeviceToHost, s));
            }
        }
    HIP_TRY(hipStreamSynchronize(s));
    return YOUTH_OK;
}

int youth_icp_reduce_host(youth_icp_ctx* c, const int16_t* src, const int16_t* dst,
                          const float* T12, int32_t* assoc, double* neq)
{
    if (!c || !src || !dst || !T12)
        return set_error(YOUTH_EINVAL, "reduce_host: bad arguments");
    int rc = bind_device(c);
    if (rc) return rc;
    hipStream_t s = c->stream;
    const size_t N = c->N;
    HIP_TRY(hipMemcpyAsync(c->d_depth, src, N * sizeof(int16_t), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(c->d_depth + N, dst, N * sizeof(int16_t), hipMemcpyHostToDevice, s));
    rc = launch_prep(c, s, c->d_depth, c->d_depth, 2, 0, 2, 1, 1);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(c->d_T32, T12, 12 * sizeof(float), hipMemcpyHostToDevice, s));
    int nb = 0;
    rc = launch_reduce(c, s, PairMap{0, 1}, 1, assoc != nullptr, &nb);
    if (rc) return rc;
    hipLaunchKernelGGL(k_solve, dim3(1), dim3(64), 0, s, c->d_partials, nb, 0, 1, c->d_T64,
                       c->d_T32, c->d_status, (double*)nullptr, c->d_neq);
    HIP_TRY(hipGetLastError());
    if (neq)
        HIP_TRY(hipMemcpyAsync(neq, c->d_neq, kNeq * sizeof(double), hipMemcpyDeviceToHost, s));
    if (assoc)
        HIP_TRY(hipMemcpyAsync(assoc, c->d_assoc, N * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return YOUTH_OK;
}

int youth_icp_solve_host(youth_icp_ctx* c, const double* neq, double* T64)
{
    if (!c || !neq || !T64) return set_error(YOUTH_EINVAL, "solve_host: bad arguments");
    int rc = bind_device(c);
    if (rc) return rc;
    hipStream_t s = c->stream;
    HIP_TRY(hipMemcpyAsync(c->d_neq, neq, kNeq * sizeof(double), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(c->d_T64, T64, 16 * sizeof(double), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_solve_neq, dim3(1), dim3(64), 0, s, c->d_neq, c->d_T64, c->d_T32,
                       c->d_status);
    HIP_TRY(hipGetLastError());
    int32_t st = 0;
    HIP_TRY(hipMemcpyAsync(T64, c->d_T64, 12 * sizeof(double), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(&st, c->d_status, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return st;
}

// ----------------------------------------------- one-shot host batch API --
static std::mutex g_batch_mu;
static youth_icp_ctx* g_batch_ctx = nullptr;

int youth_icp_align_batch(const int16_t* src, const int16_t* dst, int n_pairs, int W, int H,
                          const youth_intrinsics* K, int iters, float* T_out,
                          int32_t* assoc_out)
{
    if (!src || !dst || n_pairs <= 0 || W < 3 || H < 3 || iters < 0 || !T_out)
        return set_error(YOUTH_EINVAL, "align_batch: bad arguments %d", n_pairs);
    std::lock_guard<std::mutex> lk(g_batch_mu);
    const youth_intrinsics Kd = K ? *K : youth_default_intrinsics(W, H);
    youth_icp_params P = youth_default_params();
    P.iters = iters;
    youth_icp_ctx* c = g_batch_ctx;
    const bool same = c && c->W == W && c->H == H && c->max_frames >= 2 * n_pairs &&
                      c->K.fx == Kd.fx && c->K.fy == Kd.fy && c->K.cx == Kd.cx &&
                      c->K.cy == Kd.cy && c->K.ds == Kd.depth_scale;
    if (!same) {
        if (c) youth_icp_destroy(c);
        g_batch_ctx = nullptr;
        c = youth_icp_create(0, W, H, 2 * n_pairs, &Kd, &P);
        if (!c) return g_last_error.find("no HIP device") != std::string::npos ? YOUTH_ENODEV : YOUTH_EHIP;
        g_batch_ctx = c;
    }
    c->prm = P;
    int rc = bind_device(c);
    if (rc) return rc;
    hipStream_t s = c->stream;
    const size_t N = c->N;
    HIP_TRY(hipMemcpyAsync(c->d_depth, src, (size_t)n_pairs * N * sizeof(int16_t),
                           hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(c->d_depth + (size_t)n_pairs * N, dst,
                           (size_t)n_pairs * N * sizeof(int16_t), hipMemcpyHostToDevice, s));
    rc = youth_icp_align_pairs_device(c, c->d_depth, c->d_depth + (size_t)n_pairs * N, n_pairs,
                                      nullptr, c->d_Tout, s);
    if (rc) return rc;
    if (assoc_out) {
        int nb = 0;
        rc = launch_reduce(c, s, PairMap{0, n_pairs}, n_pairs, true, &nb);
        if (rc) return rc;
        HIP_TRY(hipMemcpyAsync(assoc_out, c->d_assoc, (size_t)n_pairs * N * sizeof(int32_t),
                               hipMemcpyDeviceToHost, s));
    }
    HIP_TRY(hipMemcpyAsync(T_out, c->d_Tout, (size_t)n_pairs * 16 * sizeof(float),
                           hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return YOUTH_OK;
}

// ------------------------------------------------------ frame tracking --
int youth_icp_track_frame(youth_icp_ctx* c, const int16_t* depth, const double* T_init,
                          double* T_rel, int* has_ref)
{
    if (!c || !depth || !T_rel) return set_error(YOUTH_EINVAL, "track_frame: bad arguments");
    int rc = bind_device(c);
    if (rc) return rc;
    hipStream_t s = c->stream;
    const size_t N = c->N;
    const int slot = c->track_ref == 0 ? 1 : 0;
    HIP_TRY(hipMemcpyAsync(c->d_depth + (size_t)slot * N, depth, N * sizeof(int16_t),
                           hipMemcpyHostToDevice, s));
    rc = launch_prep(c, s, c->d_depth + (size_t)slot * N, nullptr, 1, slot, 1, 0, 1);
    if (rc) return rc;
    int32_t st = 0;
    const int ref = c->track_ref;
    if (has_ref) *has_ref = ref >= 0;
    if (ref >= 0) {
        rc = run_iterations(c, s, PairMap{slot, ref}, 1, T_init);
        if (rc) return rc;
        HIP_TRY(hipMemcpyAsync(T_rel, c->d_T64, 16 * sizeof(double), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(&st, c->d_status, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    }
    HIP_TRY(hipStreamSynchronize(s));
    if (ref < 0) {
        for (int i = 0; i < 16; ++i) T_rel[i] = (i % 5) == 0 ? 1.0 : 0.0;
    }
    c->track_ref = slot;
    return st;
}

void youth_icp_track_reset(youth_icp_ctx* c)
{
    if (c) c->track_ref = -1;
}

}  // extern "C"
