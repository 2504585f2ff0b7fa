/*
 * icp_oracle.c — CPU ORACLE (test infrastructure only; see icp_oracle.h).
 *
 * Every fp32 expression below is written in the exact evaluation order the
 * HIP kernels use (slam-rgbd_amd/csrc/icp_kernels.hip) and is compiled with
 * -ffp-contract=off, so back-projection, normals and association indices are
 * bit-identical between the two.  Reductions are fp64 of exact fp32
 * products (a product of two fp32 values is exact in fp64), so CPU and GPU
 * sums differ only by fp64 summation order.
 */
#include "icp_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* viewerModule.c:341-345: `if(depthValue > 0)`, `z_pos = depthValue/1000.0f`,
 * `x_pos = (x - currentWidth/2) * z_pos / 570.3f`.  With cx = (float)(W/2)
 * the subtraction ((float)u - cx) is exact, so this equals the viewer's
 * (float)(u - W/2) bit-for-bit. */
void oracle_backproject(const int16_t* depth, int W, int H,
                        const oracle_intrinsics* K, float* X, float* Y, float* Z)
{
    for (int v = 0; v < H; ++v) {
        for (int u = 0; u < W; ++u) {
            const int i = v * W + u;
            const int d = depth[i];
            if (d > 0) {
                const float z = (float)d / K->depth_scale;
                X[i] = (((float)u - K->cx) * z) / K->fx;
                Y[i] = (((float)v - K->cy) * z) / K->fy;
                Z[i] = z;
            } else {
                X[i] = 0.0f;
                Y[i] = 0.0f;
                Z[i] = 0.0f;
            }
        }
    }
}

void oracle_normals(const float* X, const float* Y, const float* Z, int W, int H,
                    float* NX, float* NY, float* NZ)
{
    for (int v = 0; v < H; ++v) {
        for (int u = 0; u < W; ++u) {
            const int i = v * W + u;
            NX[i] = 0.0f;
            NY[i] = 0.0f;
            NZ[i] = 0.0f;
            if (u == 0 || v == 0 || u == W - 1 || v == H - 1) continue;
            const int l = i - 1, r = i + 1, up = i - W, dn = i + W;
            if (!(Z[i] > 0.0f) || !(Z[l] > 0.0f) || !(Z[r] > 0.0f) ||
                !(Z[up] > 0.0f) || !(Z[dn] > 0.0f))
                continue;
            const float ax = X[r] - X[l], ay = Y[r] - Y[l], az = Z[r] - Z[l];
            const float bx = X[dn] - X[up], by = Y[dn] - Y[up], bz = Z[dn] - Z[up];
            const float cx = ay * bz - az * by;
            const float cy = az * bx - ax * bz;
            const float cz = ax * by - ay * bx;
            const float len2 = (cx * cx + cy * cy) + cz * cz;
            if (!(len2 > 0.0f)) continue;
            const float len = sqrtf(len2);
            float nx = cx / len, ny = cy / len, nz = cz / len;
            if (((nx * X[i] + ny * Y[i]) + nz * Z[i]) > 0.0f) {
                nx = -nx;
                ny = -ny;
                nz = -nz;
            }
            NX[i] = nx;
            NY[i] = ny;
            NZ[i] = nz;
        }
    }
}

/* Which restatement of spec a7/a8 the association and residual follow
 * (oracle_set_spec): ORACLE_SPEC_SURVEY, the default, is SURVEY.md §8a a7/a8
 * and §7 word for word: separately rounded products and sums in a fixed
 * order, no FMA, and the projection's quotient as an IEEE division, u' =
 * floor(fx P'x / P'z + cx + 0.5) evaluated left to right; ORACLE_SPEC_FMA is
 * the opt-in fma-chain form (one correctly rounded reciprocal).
 * Set before a run; read-only while one is in flight (OpenMP threads only
 * read it). */
static int g_spec = ORACLE_SPEC_SURVEY;

int oracle_set_spec(int spec)
{
    if (spec != ORACLE_SPEC_FMA && spec != ORACLE_SPEC_SURVEY) return -1;
    const int old = g_spec;
    g_spec = spec;
    return old;
}

int oracle_get_spec(void) { return g_spec; }

/* Spec a10 as oracle_align runs it (oracle_set_solve): the block
 * elimination (the default, what the kernels run) or the round 1-4 LDL^T,
 * kept so the fixtures' LDL^T poses stay reproducible.  Same threading rule
 * as g_spec. */
static int g_solve = ORACLE_SOLVE_BLOCK;

int oracle_set_solve(int mode)
{
    if (mode != ORACLE_SOLVE_BLOCK && mode != ORACLE_SOLVE_LDLT) return -1;
    const int old = g_solve;
    g_solve = mode;
    return old;
}

/* Spec a7 for one source point.  Returns the target index or -1 and, when
 * matched, the transformed point q. */
static inline int assoc_one(float sx, float sy, float sz, const float T[12],
                            const oracle_intrinsics* K, int W, int H,
                            const float* tX, const float* tY, const float* tZ,
                            const float* nX, const float* nY, const float* nZ,
                            float thr2, float q[3])
{
    if (!(sz > 0.0f)) return -1;
    float qx, qy, qz, fu, fv;
    if (g_spec == ORACLE_SPEC_SURVEY) {
        /* P' = R P + t, fp32, fixed op order, no FMA */
        qx = ((T[0] * sx + T[1] * sy) + T[2] * sz) + T[3];
        qy = ((T[4] * sx + T[5] * sy) + T[6] * sz) + T[7];
        qz = ((T[8] * sx + T[9] * sy) + T[10] * sz) + T[11];
        if (!(qz > 0.0f)) return -1;
        /* u' = floor(fx P'x / P'z + cx + 0.5), the division kept a division
         * (SURVEY §7 "never reciprocal-multiply"): the inverse of the viewer's
         * x = ((u - cx) z) / fx (viewerModule.c:343-345) */
        fu = floorf((((K->fx * qx) / qz) + K->cx) + 0.5f);
        fv = floorf((((K->fy * qy) / qz) + K->cy) + 0.5f);
    } else {
        /* P' = R P + t as three fma chains (one rounding per step) */
        qx = fmaf(T[2], sz, fmaf(T[1], sy, fmaf(T[0], sx, T[3])));
        qy = fmaf(T[6], sz, fmaf(T[5], sy, fmaf(T[4], sx, T[7])));
        qz = fmaf(T[10], sz, fmaf(T[9], sy, fmaf(T[8], sx, T[11])));
        if (!(qz > 0.0f)) return -1;
        /* one correctly rounded reciprocal, then fx P'x rz + (cx + 0.5) in one
         * rounding (cx + 0.5 is exact: cx is a pixel coordinate) */
        const float rz = 1.0f / qz;
        fu = floorf(fmaf(K->fx * qx, rz, K->cx + 0.5f));
        fv = floorf(fmaf(K->fy * qy, rz, K->cy + 0.5f));
    }
    if (!(fu >= 0.0f && fu < (float)W && fv >= 0.0f && fv < (float)H)) return -1;
    const int j = (int)fv * W + (int)fu;
    const float tz = tZ[j];
    if (!(tz > 0.0f)) return -1;
    if (nX[j] == 0.0f && nY[j] == 0.0f && nZ[j] == 0.0f) return -1;
    const float dx = qx - tX[j], dy = qy - tY[j], dz = qz - tz;
    const float d2 = g_spec == ORACLE_SPEC_SURVEY ? (dx * dx + dy * dy) + dz * dz
                                                  : fmaf(dz, dz, fmaf(dy, dy, dx * dx));
    if (!(d2 < thr2)) return -1;
    q[0] = qx;
    q[1] = qy;
    q[2] = qz;
    return j;
}

void oracle_associate(const float* sX, const float* sY, const float* sZ,
                      const float* tX, const float* tY, const float* tZ,
                      const float* nX, const float* nY, const float* nZ,
                      int W, int H, const oracle_intrinsics* K, const float T[12],
                      float dist_thresh, int32_t* idx)
{
    const float thr2 = dist_thresh * dist_thresh;
    const int N = W * H;
    float q[3];
    for (int i = 0; i < N; ++i)
        idx[i] = assoc_one(sX[i], sY[i], sZ[i], T, K, W, H, tX, tY, tZ, nX, nY,
                           nZ, thr2, q);
}

static int g_reduce = ORACLE_REDUCE_EXACT;
static oracle_lanes g_lanes = {ORACLE_LANES_STRIDED, 0, 0, 0};

int oracle_set_reduce(int mode, const oracle_lanes* g)
{
    if (mode == ORACLE_REDUCE_EXACT) {
        const int old = g_reduce;
        g_reduce = mode;
        return old;
    }
    if (mode != ORACLE_REDUCE_LANE32 || !g || g->threads < 64 || g->threads % 64 != 0)
        return -1;
    if (g->kind == ORACLE_LANES_STRIDED) {
        if (g->chunk < 1) return -1;
    } else if (g->kind == ORACLE_LANES_COOP || g->kind == ORACLE_LANES_COOP_TILE) {
        if (g->npx < 1 || (g->kind == ORACLE_LANES_COOP_TILE && (g->npx * g->threads) % 64 != 0))
            return -1;
    } else {
        return -1;
    }
    const int old = g_reduce;
    g_reduce = mode;
    g_lanes = *g;
    return old;
}

int oracle_get_reduce(void) { return g_reduce; }

/* Lane of source pixel i (u, v) under the partition g (icp_oracle.h), and
 * the number of lanes of a W x H frame. */
static long lane_of(const oracle_lanes* g, int W, int H, int i)
{
    const long T = g->threads;
    if (g->kind == ORACLE_LANES_STRIDED) {
        /* accumulate_chunk: i = start + 4 threadIdx + q + s (4 threads) */
        const long c = i / g->chunk, o = i - c * g->chunk;
        return c * T + (o % (4 * T)) / 4;
    }
    if (g->kind == ORACLE_LANES_COOP) {
        /* k_icp_coop source staging: i = c npx T + s T + t */
        const long C = (long)g->npx * T;
        return (i / C) * T + (i % C) % T;
    }
    /* k_icp_coop tile_src: k = s T + t, u = x0 + k % 64, v = y0 + k / 64 */
    const int th = (int)((long)g->npx * T / 64), tiles_x = (W + 63) / 64;
    const int u = i % W, v = i / W, tx = u / 64, ty = v / th;
    const long k = (long)(v - ty * th) * 64 + (u - tx * 64);
    (void)H;
    return ((long)ty * tiles_x + tx) * T + k % T;
}

static long lane_count(const oracle_lanes* g, int W, int H)
{
    const long N = (long)W * H, T = g->threads;
    if (g->kind == ORACLE_LANES_STRIDED) return (N + g->chunk - 1) / g->chunk * T;
    if (g->kind == ORACLE_LANES_COOP) return (N + (long)g->npx * T - 1) / ((long)g->npx * T) * T;
    const int th = (int)((long)g->npx * T / 64);
    return (long)((W + 63) / 64) * ((H + th - 1) / th) * T;
}

void oracle_reduce(const float* sX, const float* sY, const float* sZ,
                   const float* tX, const float* tY, const float* tZ,
                   const float* nX, const float* nY, const float* nZ,
                   int W, int H, const oracle_intrinsics* K, const float T[12],
                   float dist_thresh, double out[ORACLE_NEQ])
{
    const float thr2 = dist_thresh * dist_thresh;
    const int N = W * H;
    double acc[ORACLE_NEQ];
    memset(acc, 0, sizeof(acc));
    const int lanes32 = g_reduce == ORACLE_REDUCE_LANE32;
    const long n_lanes = lanes32 ? lane_count(&g_lanes, W, H) : 0;
    float* la = lanes32 ? (float*)calloc((size_t)n_lanes * 28, sizeof(float)) : NULL;
    if (lanes32 && !la) {
        for (int k = 0; k < ORACLE_NEQ; ++k) out[k] = NAN;
        return;
    }
    float q[3];
    for (int i = 0; i < N; ++i) {
        const int j = assoc_one(sX[i], sY[i], sZ[i], T, K, W, H, tX, tY, tZ, nX,
                                nY, nZ, thr2, q);
        if (j < 0) continue;
        const float nx = nX[j], ny = nY[j], nz = nZ[j];
        const float dx = q[0] - tX[j], dy = q[1] - tY[j], dz = q[2] - tZ[j];
        /* residual r = n . (P' - P_t) and J = [ (P' x n)^T , n^T ] for the
         * left perturbation exp(xi) T (spec a8) */
        float r, J[6];
        if (g_spec == ORACLE_SPEC_SURVEY) {
            r = (nx * dx + ny * dy) + nz * dz;
            J[0] = q[1] * nz - q[2] * ny;
            J[1] = q[2] * nx - q[0] * nz;
            J[2] = q[0] * ny - q[1] * nx;
        } else {
            r = fmaf(nz, dz, fmaf(ny, dy, nx * dx));
            J[0] = fmaf(q[1], nz, -(q[2] * ny));
            J[1] = fmaf(q[2], nx, -(q[0] * nz));
            J[2] = fmaf(q[0], ny, -(q[1] * nx));
        }
        J[3] = nx;
        J[4] = ny;
        J[5] = nz;
        acc[28] += 1.0;
        if (lanes32) {
            /* the kernels' match_accumulate with fp32 lanes: v_fma_f32 */
            float* l = la + (size_t)lane_of(&g_lanes, W, H, i) * 28;
            int k = 0;
            for (int a = 0; a < 6; ++a)
                for (int b = a; b < 6; ++b, ++k) l[k] = fmaf(J[a], J[b], l[k]);
            for (int a = 0; a < 6; ++a) l[21 + a] = fmaf(J[a], r, l[21 + a]);
            l[27] = fmaf(r, r, l[27]);
            continue;
        }
        int k = 0;
        for (int a = 0; a < 6; ++a)
            for (int b = a; b < 6; ++b)
                acc[k++] += (double)J[a] * (double)J[b];
        for (int a = 0; a < 6; ++a) acc[21 + a] += (double)J[a] * (double)r;
        acc[27] += (double)r * (double)r;
    }
    if (lanes32) {
        /* fp64 finalize: every lane's sums, converted, added in lane order */
        for (long L = 0; L < n_lanes; ++L)
            for (int k = 0; k < 28; ++k) acc[k] += (double)la[(size_t)L * 28 + k];
        free(la);
    }
    memcpy(out, acc, sizeof(acc));
}

/* Spec a10 (round 5): A x = b by block elimination with 3x3 adjugates,
 * xi = -x, ONE division on the dependent chain.  With P = A[0..2][0..2]
 * (rotation), Q = A[0..2][3..5], R = A[3..5][3..5], b = (b1, b2),
 * C = adj(P):
 *   detP = P00 C00 + P01 C01 + P02 C02, M = C Q, u = C b1
 *   S'   = detP R - Q^T M  (detP times the Schur complement)
 *   y'   = detP b2 - Q^T u
 *   x2   = adj(S') y' * (1 / det S')
 *   x1   = C (b1 - Q x2) * (1 / detP)
 * DEGENERATE (1) iff an LDL^T pivot is <= eps = 1e-12 max diag, tested on the
 * leading minors by products (pivot j = m_j / m_{j-1}; no division).  Every
 * a b - c d is fma(a, b, -(c d)); every 3-term dot is
 * fma(a2, b2, fma(a1, b1, a0 b0)).  The kernels (icp_kernels.hip
 * solve_block6) perform the same correctly rounded operations in the same
 * order: xi and the status are bit-identical. */
static double dd2(double a, double b, double c, double d) { return fma(a, b, -(c * d)); }
static double dot3(double a0, double b0, double a1, double b1, double a2, double b2)
{
    return fma(a2, b2, fma(a1, b1, a0 * b0));
}
/* symmetric 3x3 {m00, m01, m02, m11, m12, m22} */
static void adj3(const double p[6], double c[6])
{
    c[0] = dd2(p[3], p[5], p[4], p[4]);
    c[1] = dd2(p[2], p[4], p[1], p[5]);
    c[2] = dd2(p[1], p[4], p[2], p[3]);
    c[3] = dd2(p[0], p[5], p[2], p[2]);
    c[4] = dd2(p[1], p[2], p[0], p[4]);
    c[5] = dd2(p[0], p[3], p[1], p[1]);
}
static void symv3(const double c[6], const double v[3], double o[3])
{
    o[0] = dot3(c[0], v[0], c[1], v[1], c[2], v[2]);
    o[1] = dot3(c[1], v[0], c[3], v[1], c[4], v[2]);
    o[2] = dot3(c[2], v[0], c[4], v[1], c[5], v[2]);
}

int oracle_solve(const double neq[ORACLE_NEQ], double xi[6])
{
    for (int i = 0; i < 6; ++i) xi[i] = 0.0;
    if (!(neq[28] >= 6.0)) return 2;
    static const int diag[6] = {0, 6, 11, 15, 18, 20};
    double maxd = 0.0;
    for (int a = 0; a < 6; ++a)
        if (neq[diag[a]] > maxd) maxd = neq[diag[a]];
    if (!(maxd > 0.0)) return 1;
    const double eps = 1e-12 * maxd;
    const double P[6] = {neq[0], neq[1], neq[2], neq[6], neq[7], neq[11]};
    const double R[6] = {neq[15], neq[16], neq[17], neq[18], neq[19], neq[20]};
    const double Q[3][3] = {{neq[3], neq[4], neq[5]}, {neq[8], neq[9], neq[10]},
                            {neq[12], neq[13], neq[14]}};
    const double b1[3] = {neq[21], neq[22], neq[23]}, b2[3] = {neq[24], neq[25], neq[26]};
    double C[6], E[6], S[6], M[3][3], u[3], y[3], v[3], x2[3], w[3];
    adj3(P, C);
    const double detP = dot3(P[0], C[0], P[1], C[1], P[2], C[2]);
    for (int j = 0; j < 3; ++j) {  /* M = C Q, column by column */
        const double q[3] = {Q[0][j], Q[1][j], Q[2][j]};
        double o[3];
        symv3(C, q, o);
        for (int i = 0; i < 3; ++i) M[i][j] = o[i];
    }
    symv3(C, b1, u);
    static const int si[6] = {0, 0, 0, 1, 1, 2}, sj[6] = {0, 1, 2, 1, 2, 2};
    for (int e = 0; e < 6; ++e) {  /* S' upper triangle: detP R[i][j] - (Q^T M)[i][j] */
        const int i = si[e], j = sj[e];
        S[e] = fma(detP, R[e], -dot3(Q[0][i], M[0][j], Q[1][i], M[1][j], Q[2][i], M[2][j]));
    }
    for (int j = 0; j < 3; ++j)
        y[j] = fma(detP, b2[j], -dot3(Q[0][j], u[0], Q[1][j], u[1], Q[2][j], u[2]));
    adj3(S, E);
    const double detS = dot3(S[0], E[0], S[1], E[1], S[2], E[2]);
    const double epsP = eps * detP;
    /* pivots: P00, C22/P00, detP/C22, S'00/detP, E22/(detP S'00), detS/(detP E22) */
    if (!(P[0] > eps) || !(C[5] > eps * P[0]) || !(detP > eps * C[5]) || !(S[0] > epsP) ||
        !(E[5] > epsP * S[0]) || !(detS > epsP * E[5]))
        return 1;
    const double rS = 1.0 / detS, rP = 1.0 / detP;
    symv3(E, y, v);
    for (int i = 0; i < 3; ++i) x2[i] = v[i] * rS;
    for (int i = 0; i < 3; ++i) w[i] = b1[i] - dot3(Q[i][0], x2[0], Q[i][1], x2[1], Q[i][2], x2[2]);
    symv3(C, w, v);
    for (int i = 0; i < 3; ++i) {
        xi[i] = -(v[i] * rP);
        xi[3 + i] = -x2[i];
    }
    return 0;
}

/* Round 1-4 spec a10: LDL^T of A xi = -b (right-looking on the GPU, the
 * same per-element operations).  Kept for the fixtures' LDL^T poses
 * (the T64_ldlt field of the tests/golden pair fixtures) and the solve A/B. */
int oracle_solve_ldlt(const double neq[ORACLE_NEQ], double xi[6])
{
    for (int i = 0; i < 6; ++i) xi[i] = 0.0;
    if (!(neq[28] >= 6.0)) return 2;
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
    if (!(maxd > 0.0)) return 1;
    const double eps = 1e-12 * maxd;
    double L[6][6], D[6], Dinv[6];
    memset(L, 0, sizeof(L));
    for (int j = 0; j < 6; ++j) {
        double d = A[j][j];
        for (int m = 0; m < j; ++m) d -= (L[j][m] * L[j][m]) * D[m];
        if (!(d > eps)) return 1;
        D[j] = d;
        Dinv[j] = 1.0 / d;  /* one divide per pivot; every use multiplies */
        L[j][j] = 1.0;
        for (int i = j + 1; i < 6; ++i) {
            double s = A[i][j];
            for (int m = 0; m < j; ++m) s -= (L[i][m] * L[j][m]) * D[m];
            L[i][j] = s * Dinv[j];
        }
    }
    double y[6], x[6];
    for (int i = 0; i < 6; ++i) {
        double s = -neq[21 + i];
        for (int m = 0; m < i; ++m) s -= L[i][m] * y[m];
        y[i] = s;
    }
    for (int i = 0; i < 6; ++i) y[i] = y[i] * Dinv[i];
    for (int i = 5; i >= 0; --i) {
        double s = y[i];
        for (int m = 5; m > i; --m) s -= L[m][i] * x[m];  /* m decreasing */
        x[i] = s;
    }
    for (int i = 0; i < 6; ++i) xi[i] = x[i];
    return 0;
}

void oracle_se3_exp(const double xi[6], double E[16])
{
    const double wx = xi[0], wy = xi[1], wz = xi[2];
    const double th2 = (wx * wx + wy * wy) + wz * wz;
    double a, b, c;
    if (th2 < 0x1p-7) {
        /* a = sin(t)/t, b = (1 - cos t)/t^2, c = (t - sin t)/t^3 as degree-5
         * Taylor polynomials in x = t^2 (t < 5 deg, truncation < 1e-22),
         * Horner with explicit fma: the same correctly rounded operations
         * on the GPU (se3_exp_left), so both agree bit for bit */
        const double x = th2;
        a = fma(x, fma(x, fma(x, fma(x, fma(x, -0x1.ae64567f544e4p-26, 0x1.71de3a556c734p-19),
                                        -0x1.a01a01a01a01ap-13), 0x1.1111111111111p-7),
                       -0x1.5555555555555p-3), 0x1.0000000000000p+0);
        b = fma(x, fma(x, fma(x, fma(x, fma(x, -0x1.1eed8eff8d898p-29, 0x1.27e4fb7789f5cp-22),
                                        -0x1.a01a01a01a01ap-16), 0x1.6c16c16c16c17p-10),
                       -0x1.5555555555555p-5), 0x1.0000000000000p-1);
        c = fma(x, fma(x, fma(x, fma(x, fma(x, -0x1.6124613a86d09p-33, 0x1.ae64567f544e4p-26),
                                        -0x1.71de3a556c734p-19), 0x1.a01a01a01a01ap-13),
                       -0x1.1111111111111p-7), 0x1.5555555555555p-3);
    } else {
        const double th = sqrt(th2);
        const double s = sin(th), co = cos(th);
        a = s / th;
        b = (1.0 - co) / th2;
        c = (th - s) / (th2 * th);
    }
    const double Km[3][3] = {{0.0, -wz, wy}, {wz, 0.0, -wx}, {-wy, wx, 0.0}};
    double K2[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            K2[i][j] = (Km[i][0] * Km[0][j] + Km[i][1] * Km[1][j]) + Km[i][2] * Km[2][j];
    double R[3][3], V[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            const double I = (i == j) ? 1.0 : 0.0;
            R[i][j] = (I + a * Km[i][j]) + b * K2[i][j];
            V[i][j] = (I + b * Km[i][j]) + c * K2[i][j];
        }
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) E[i * 4 + j] = R[i][j];
        E[i * 4 + 3] = (V[i][0] * xi[3] + V[i][1] * xi[4]) + V[i][2] * xi[5];
    }
    E[12] = 0.0;
    E[13] = 0.0;
    E[14] = 0.0;
    E[15] = 1.0;
}

/* T <- E * T (4x4 row-major; last row of both is [0 0 0 1]). */
static void left_compose(const double E[16], double T[16])
{
    double O[16];
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 4; ++j) {
            double s = (E[i * 4 + 0] * T[0 * 4 + j] + E[i * 4 + 1] * T[1 * 4 + j]) +
                       E[i * 4 + 2] * T[2 * 4 + j];
            if (j == 3) s += E[i * 4 + 3];
            O[i * 4 + j] = s;
        }
    }
    O[12] = 0.0;
    O[13] = 0.0;
    O[14] = 0.0;
    O[15] = 1.0;
    memcpy(T, O, sizeof(O));
}

static void to_f32(const double T[16], float T32[12])
{
    for (int i = 0; i < 12; ++i) T32[i] = (float)T[i];
}

static int align_ws(const int16_t* src, const int16_t* dst, int W, int H,
                    const oracle_intrinsics* K, int iters, float dist_thresh,
                    const double* T_init, double T64[16], float T32[12],
                    double* stats, float* ws)
{
    const size_t N = (size_t)W * (size_t)H;
    float *sX = ws, *sY = ws + N, *sZ = ws + 2 * N;
    float *tX = ws + 3 * N, *tY = ws + 4 * N, *tZ = ws + 5 * N;
    float *nX = ws + 6 * N, *nY = ws + 7 * N, *nZ = ws + 8 * N;
    oracle_backproject(src, W, H, K, sX, sY, sZ);
    oracle_backproject(dst, W, H, K, tX, tY, tZ);
    oracle_normals(tX, tY, tZ, W, H, nX, nY, nZ);
    double T[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    if (T_init) memcpy(T, T_init, sizeof(T));
    int status = 0;
    for (int it = 0; it < iters; ++it) {
        float Tf[12];
        to_f32(T, Tf);
        double neq[ORACLE_NEQ], xi[6], E[16];
        oracle_reduce(sX, sY, sZ, tX, tY, tZ, nX, nY, nZ, W, H, K, Tf, dist_thresh,
                      neq);
        if (stats) {
            stats[2 * it + 0] = neq[28];
            stats[2 * it + 1] = neq[27];
        }
        const int st = g_solve == ORACLE_SOLVE_LDLT ? oracle_solve_ldlt(neq, xi) : oracle_solve(neq, xi);
        status |= st;
        if (st == 0) {
            oracle_se3_exp(xi, E);
            left_compose(E, T);
        }
    }
    memcpy(T64, T, sizeof(T));
    to_f32(T, T32);
    return status;
}

int oracle_align(const int16_t* src, const int16_t* dst, int W, int H,
                 const oracle_intrinsics* K, int iters, float dist_thresh,
                 const double* T_init, double T64[16], float T32[12],
                 double* stats)
{
    const size_t N = (size_t)W * (size_t)H;
    float* ws = (float*)malloc(9 * N * sizeof(float));
    if (!ws) return -1;
    const int st = align_ws(src, dst, W, H, K, iters, dist_thresh, T_init, T64,
                            T32, stats, ws);
    free(ws);
    return st;
}

void oracle_align_batch(const int16_t* src, const int16_t* dst, int n_pairs,
                        int W, int H, const oracle_intrinsics* K, int iters,
                        float dist_thresh, double* T64, int32_t* status,
                        double* stats, int n_threads)
{
    const size_t N = (size_t)W * (size_t)H;
#ifdef _OPENMP
    if (n_threads <= 0) n_threads = omp_get_max_threads();
#pragma omp parallel num_threads(n_threads)
#endif
    {
        float* ws = (float*)malloc(9 * N * sizeof(float));
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
        for (int p = 0; p < n_pairs; ++p) {
            float T32[12];
            status[p] = ws ? align_ws(src + (size_t)p * N, dst + (size_t)p * N, W, H,
                                      K, iters, dist_thresh, NULL,
                                      T64 + (size_t)p * 16, T32,
                                      stats ? stats + (size_t)p * 2 * iters : NULL, ws)
                           : -1;
        }
        free(ws);
    }
    (void)n_threads;
}

int oracle_max_threads(void)
{
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* viewerModule.c:336-357 (display_3d_color's loop), minus the GL calls: the
 * glColor3f / glVertex3f arguments of every valid pixel, in loop order. */
int oracle_viewer_cloud(const int16_t* depth, const uint8_t* rgb, int W, int H,
                        const oracle_intrinsics* K, float* vertices)
{
    return oracle_viewer_cloud_posed(depth, rgb, W, H, K, NULL, vertices);
}

/* youth_cloud_build_device_posed (include/youth_viewer.h): the viewer's point
 * moved by the camera -> world pose T (row-major 3x4) with the three fma
 * chains of spec a7, then the display flip; T NULL: viewerModule.c:336-357. */
int oracle_viewer_cloud_posed(const int16_t* depth, const uint8_t* rgb, int W, int H,
                              const oracle_intrinsics* K, const float* T, float* vertices)
{
    int n = 0;
    for (int y = 0; y < H; ++y) {
        for (int x = 0; x < W; ++x) {
            const int index = y * W + x;
            const int d = depth[index];
            if (d > 0) {
                const float z = (float)d / K->depth_scale;
                const float xp = (((float)x - K->cx) * z) / K->fx;
                const float yp = (((float)y - K->cy) * z) / K->fy;
                float* o = vertices + (size_t)n * 6;
                if (T) {
                    o[0] = -fmaf(T[2], z, fmaf(T[1], yp, fmaf(T[0], xp, T[3])));
                    o[1] = -fmaf(T[6], z, fmaf(T[5], yp, fmaf(T[4], xp, T[7])));
                    o[2] = -fmaf(T[10], z, fmaf(T[9], yp, fmaf(T[8], xp, T[11])));
                } else {
                    o[0] = -xp;
                    o[1] = -yp;
                    o[2] = -z;
                }
                o[3] = rgb ? (float)rgb[(size_t)index * 3 + 0] / 255.0f : 0.0f;
                o[4] = rgb ? (float)rgb[(size_t)index * 3 + 1] / 255.0f : 0.0f;
                o[5] = rgb ? (float)rgb[(size_t)index * 3 + 2] / 255.0f : 0.0f;
                ++n;
            }
        }
    }
    return n;
}
