/*
 * icp_oracle.h — CPU ORACLE for the RGBD frame-to-frame ICP path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the shipped library links, loads or
 * calls this code; only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may use it, and only as the checker / timed CPU baseline.
 *
 * What it restates (reference = SeunghwanByun/SLAM-RGBD @ 2025-08-24):
 *   - back-projection: Youth.Source/ViewerModule/viewerModule.c:341-345
 *     (valid iff d > 0; Z = d/1000.0f; X = ((u - W/2) * Z)/570.3f; Y alike),
 *     generalised to explicit intrinsics that reproduce the viewer bit-for-bit
 *     when cx = W/2, cy = H/2, fx = fy = 570.3f, depth_scale = 1000.0f;
 *   - intrinsics / depth factor: AlgorithmModule/config/astra_orb_slam3_rgbd.yaml:9-12,35;
 *   - buffer layout int16 [H][W] row-major: SLAM.h:22, frameDefinitions.h:11-20.
 * PINNED against the back-projection known-answer table of SURVEY.md §4
 * (bit patterns computed with gcc -O2 -ffp-contract=off, x86-64 SSE fp32) —
 * see tests/test_oracle.py.
 *
 * PARITY UNPINNED for everything after back-projection: the reference has no
 * ICP (its pose maths is inside un-vendored ORB-SLAM3,
 * SLAM.cpp:54, version unpinned, feature-based).  Normals, projective
 * association, point-to-plane Jacobian, 6x6 reduction, 6x6 solve and the
 * SE(3) update follow this build's own spec (SURVEY.md §8a rows a6-a10,
 * DESIGN.md §2), checked here against numpy/scipy and known-motion recovery.
 *
 * Build: gcc -O2 -ffp-contract=off (no -ffast-math, no -march=native), so
 * every fp32 expression rounds exactly as written — the GPU kernels are
 * compiled with the same contraction rule and must match bit-for-bit on XYZ,
 * normals and association indices.
 */
#ifndef YOUTH_ICP_ORACLE_H
#define YOUTH_ICP_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_intrinsics {
    float fx, fy, cx, cy, depth_scale;
} oracle_intrinsics; /* layout-identical to youth_intrinsics */

#define ORACLE_NEQ 29

/* Arithmetic of spec a7/a8 (association, residual, Jacobian):
 *   ORACLE_SPEC_SURVEY (default) SURVEY.md §8a a7/a8 + §7 literally: no FMA
 *                      (products and sums rounded separately, fixed order)
 *                      and IEEE division fx P'x / P'z — what the kernels run
 *                      by default (YOUTH_SPEC_SURVEY);
 *   ORACLE_SPEC_FMA    the opt-in fma form: fma chains and one
 *                      correctly rounded reciprocal 1/P'z (YOUTH_SPEC_FMA).
 * Back-projection, normals, reduction, solve and update are common.
 * oracle_set_spec returns the previous spec (-1: unknown spec). */
#define ORACLE_SPEC_FMA 0
#define ORACLE_SPEC_SURVEY 1
int oracle_set_spec(int spec);
int oracle_get_spec(void);

/* Reduction of spec a9 (the 28 sums of products and the count):
 *   ORACLE_REDUCE_EXACT  every product of two fp32 values is exact in fp64;
 *                        the products are summed in fp64 in pixel order;
 *   ORACLE_REDUCE_LANE32 SURVEY.md §8a a9 as worded ("fp32 lanes -> fp64
 *                        finalize"), the kernels' default: the source pixels
 *                        are partitioned into lanes exactly as one kernel
 *                        launch partitions them (oracle_lanes below); each
 *                        lane sums its matched pixels' 28 products in fp32
 *                        (fmaf, one rounding each, from +0, in increasing
 *                        pixel order); every lane's 28 sums are then
 *                        converted to fp64 and added in fp64.  The count is
 *                        an integer in both modes.
 * Lane partitions (each cites the kernel loop it restates):
 *   ORACLE_LANES_STRIDED  k_icp / k_reduce (accumulate_chunk): workgroups of
 *                        `threads` lanes own chunks of `chunk` pixels
 *                        (chunk c = [c chunk, (c+1) chunk) of the frame); in
 *                        every step of 4 threads pixels lane l takes pixels
 *                        4l .. 4l+3;
 *   ORACLE_LANES_COOP     k_icp_coop, contiguous chunks: workgroup c owns
 *                        pixels [c npx threads, (c+1) npx threads), lane t of
 *                        it the pixels c npx threads + s threads + t, s < npx;
 *   ORACLE_LANES_COOP_TILE k_icp_coop with tile-shaped chunks: workgroup c
 *                        owns target tile c (64 x tile_h pixels, tiles in
 *                        raster order, tile_h = npx threads / 64), lane t the
 *                        tile pixels k = s threads + t (k raster inside the
 *                        tile: u = x0 + k % 64, v = y0 + k / 64).
 * oracle_set_reduce returns the previous mode (-1: bad arguments; the
 * geometry is ignored in EXACT mode and may be NULL there). */
#define ORACLE_REDUCE_EXACT 0
#define ORACLE_REDUCE_LANE32 1
#define ORACLE_LANES_STRIDED 0
#define ORACLE_LANES_COOP 1
#define ORACLE_LANES_COOP_TILE 2
typedef struct oracle_lanes {
    int kind, chunk, threads, npx;
} oracle_lanes; /* layout-identical to youth_lanes */
int oracle_set_reduce(int mode, const oracle_lanes* geometry);
int oracle_get_reduce(void);

/* viewerModule.c:341-345 generalised.  Invalid pixel -> X=Y=Z=0. */
void oracle_backproject(const int16_t* depth, int W, int H,
                        const oracle_intrinsics* K, float* X, float* Y, float* Z);

/* Central-difference normals (spec a6): n = normalize((P(u+1)-P(u-1)) x
 * (P(v+1)-P(v-1))), invalid (0,0,0) on the 1-px border, if any of the 4
 * neighbours or the centre is invalid, or the cross product is zero;
 * oriented so n.P <= 0. */
void oracle_normals(const float* X, const float* Y, const float* Z, int W, int H,
                    float* NX, float* NY, float* NZ);

/* Projective association (spec a7) for every source pixel at the fp32 pose
 * T (3x4 row-major, P' = R P + t).  idx[i] = v'*W+u' or -1. */
void oracle_associate(const float* sX, const float* sY, const float* sZ,
                      const float* tX, const float* tY, const float* tZ,
                      const float* nX, const float* nY, const float* nZ,
                      int W, int H, const oracle_intrinsics* K, const float T[12],
                      float dist_thresh, int32_t* idx);

/* Point-to-plane normal equations (spec a8-a9) at pose T, summed as the
 * reduction mode says (oracle_set_reduce).  out[29] as YOUTH_NEQ. */
void oracle_reduce(const float* sX, const float* sY, const float* sZ,
                   const float* tX, const float* tY, const float* tZ,
                   const float* nX, const float* nY, const float* nZ,
                   int W, int H, const oracle_intrinsics* K, const float T[12],
                   float dist_thresh, double out[ORACLE_NEQ]);

/* Solve of A xi = -b (spec a10, round 5): block (3+3) elimination with 3x3
 * adjugates, one division on the dependent chain.  Returns 0,
 * or status bits (1 = an LDL^T pivot <= 1e-12 max diag, tested on the
 * leading minors; 2 = fewer than 6 correspondences); xi zeroed then. */
int oracle_solve(const double neq[ORACLE_NEQ], double xi[6]);
/* The round 1-4 spec a10: LDL^T, one IEEE reciprocal per pivot.  Not used by
 * oracle_align unless oracle_set_solve(ORACLE_SOLVE_LDLT); kept for the
 * fixtures' T64_ldlt poses. */
int oracle_solve_ldlt(const double neq[ORACLE_NEQ], double xi[6]);
/* Which of the two oracle_align uses (the kernels run the block form only);
 * returns the previous mode, -1 for an unknown one. */
#define ORACLE_SOLVE_BLOCK 0
#define ORACLE_SOLVE_LDLT 1
int oracle_set_solve(int mode);

/* SE(3) exponential of xi = (omega, upsilon), 4x4 row-major fp64. */
void oracle_se3_exp(const double xi[6], double E[16]);

/* Full align of one pair: back-project both, target normals, `iters` fixed
 * iterations T <- exp(xi) T.  T_init nullable (identity).  Outputs: T64
 * [16], T32 [12] (the fp32 pose used by the NEXT iteration), stats
 * nullable [iters][2] (count, sum r^2).  Returns accumulated status bits. */
int oracle_align(const int16_t* src, const int16_t* dst, int W, int H,
                 const oracle_intrinsics* K, int iters, float dist_thresh,
                 const double* T_init, double T64[16], float T32[12],
                 double* stats);

/* Batch of independent pairs, OpenMP over pairs with n_threads threads
 * (<= 0: all).  src/dst [n][H][W]; T64 [n][16]; status [n]; stats nullable
 * [n][iters][2] (count, sum r^2 per iteration, as oracle_align). */
void oracle_align_batch(const int16_t* src, const int16_t* dst, int n_pairs,
                        int W, int H, const oracle_intrinsics* K, int iters,
                        float dist_thresh, double* T64, int32_t* status,
                        double* stats, int n_threads);

/* Threads OpenMP will use for n_threads <= 0 (1 when built without OpenMP). */
int oracle_max_threads(void);

/* Viewer point list: the vertices display_3d_color emits,
 * Youth.Source/ViewerModule/viewerModule.c:336-357.  Raster order, valid
 * pixels (d > 0) only; vertex k = {-x, -y, -z, r, g, b} (6 floats) with
 * x, y, z the back-projection above (viewerModule.c:343-345, K = the viewer
 * convention reproduces it bit-for-bit) and r, g, b = rgb[3i+c] / 255.0f
 * (:349-352).  rgb may be NULL (colour 0).  Returns the vertex count. */
int oracle_viewer_cloud(const int16_t* depth, const uint8_t* rgb, int W, int H,
                        const oracle_intrinsics* K, float* vertices);
int oracle_viewer_cloud_posed(const int16_t* depth, const uint8_t* rgb, int W, int H,
                              const oracle_intrinsics* K, const float* T, float* vertices);

#ifdef __cplusplus
}
#endif

#endif
