// icp_kernels.hip — MI355X (gfx950) kernels of the RGBD frame-to-frame ICP path.
//
// Hot path.  Reference boundary:
// Youth.Source/AlgorithmModule/SLAM.cpp:54 (TrackRGBD, the pose maths this
// replaces) and viewerModule.c:341-345 (the back-projection formula).
//
//   k_prep    target frames: int16 depth -> one 16-byte record {z, nx, ny, nz}
//             per pixel.  64x16 tiles; the (16+2) x (64+2) back-projected
//             neighbourhood is staged in LDS for the central-difference
//             normals.
//   k_reduce  per ICP iteration: source pixels straight from the int16 depth
//             (back-projected in registers), transform -> project -> ONE
//             16-byte record fetch -> gate -> residual -> Jacobian -> 29 fp64
//             accumulators per lane fed with exact fp32 products; wave
//             butterfly + LDS across waves -> one 29-double partial per
//             workgroup.  No atomics: deterministic.  18 B/px/iteration.
//   k_solve   one wave per pair: sums the partials in fixed order, LDL^T 6x6
//             solve, SE(3) exp, T <- exp(xi) T in fp64 on device, fp32 pose
//             for the next k_reduce.  No host round trip between iterations.
//
// Compiled with -ffp-contract=off: every fp32 expression rounds exactly as
// written, identical to the C oracle (oracle/icp_oracle.c) — XYZ, normals and
// association indices are bit-exact given the same fp32 pose.  The
// back-projection divides use a 2-instruction sequence only after
// k_verify_fastdiv has proven it equal to IEEE division on the ENTIRE domain
// those divides can see (d in [1, 32767], u in [0, W), v in [0, H)); otherwise
// the IEEE path is compiled in.

#include <hip/hip_runtime.h>

#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <vector>

#include "host_copy.h"
#include "youth_icp.h"

namespace {

// ----------------------------------------------------------------- layout --
// Workspace frame f:
//   recs + f*P            float4 {z, nx, ny, nz} per pixel (targets);
//   xyz  + f*3*P (+P, +2P) optional X, Y, Z planes (stage-level API only).
// P = plane stride = round_up(N + 4, 256); the pad is zeroed once, so a
// clamped fetch or a float4 load past N reads an invalid point (z = 0).
// Sources are read straight from the caller's int16 depth.
constexpr int kTileW = 64;
// k_prep tiles 128 x 24 by 512-thread workgroups: four per CU fill all 32
// wave slots (LDS 40.6 KB each).  A 128-px row touches 2 lines of its own
// and 2 of its neighbours' where a 64-px row touched 1 + 2, so the depth
// over-fetch drops from 2.8x to 1.9x: k_prep's PMC traffic 1.21 -> 1.105x of
// its 18 B/px, and 586 -> 582 us per 512 frames (profiles/r04/ab_r4c.txt,
// prep128x24_pmc.txt).  Also measured: 128 x 16 650 us (1.11x), 256 x 12
// 747 us (1.07x; three per CU, LDS-limited); earlier 64 x 48 593 us, 64 x 24 by
// 256 threads 617 us, 64 x 80 / 1024 625 us (profiles/r02/ab_s44.txt,
// ab_s45.txt); fewer workgroups per CU cost more (ab_s43.txt: 7 -> 6 per CU +8 %)
constexpr int kPrepThreads = 512;
// k_prep's own tile (k_icp_coop's fused prep keeps kTileW-wide tiles, whose
// shape its lane partition and prep counters assume); -D knobs for A/B
#ifndef YOUTH_PREP_TW
#define YOUTH_PREP_TW 128
#endif
#ifndef YOUTH_PREP_TH
#define YOUTH_PREP_TH 24
#endif
constexpr int kPrepTW = YOUTH_PREP_TW;
constexpr int kPrepTH = YOUTH_PREP_TH;
// frames in flight through youth_icp_track_submit (YOUTH_TRACK_MAX_IN_FLIGHT):
// two one at a time, or two micro-batches of two, so the next submission's
// host copy and H2D overlap the launch before it
constexpr int kTrackDepth = YOUTH_TRACK_MAX_IN_FLIGHT;
constexpr int kLdsW = kTileW + 2;

constexpr int kRedThreads = 256;
constexpr int kRedStep = kRedThreads * 4;  // pixels per workgroup loop step
constexpr int kNeq = YOUTH_NEQ;
// k_icp's chunk partials: rows of 30 doubles (29 + a zero pad, 240 B) so the
// last arriver reads them as 16-byte pieces; kSumCols interleaved columns of
// chunks are summed in parallel, then the column sums in column order.
constexpr int kPartStride = 30;
constexpr int kPieces = kPartStride / 2;  // 16-byte pieces per row
constexpr int kSumCols = 16;              // kSumCols * kPieces <= kRedThreads
// Persistent-queue words (unsigned index into ctx->d_head), one 128-B line
// apart so the contended dequeue atomic shares no line with the polled flag.
// k_icp's work queues: up to kMaxQueues heads, kQHeads + 32 q (queue q holds
// the pairs p = q (mod n_queues)).
constexpr int kQHead = 0, kQError = 32, kQSpins = 64, kQWaited = 96, kQHeads = 128;
constexpr int kMaxQueues = 8, kQHeadStride = 32;
constexpr int kQWords = kQHeads + kMaxQueues * kQHeadStride;

typedef float f4v __attribute__((ext_vector_type(4)));  // a gathered {z, nx, ny, nz} record
typedef unsigned u4v __attribute__((ext_vector_type(4)));  // two doubles, raw bits

struct Intr {
    float fx, fy, cx, cy, ds;
};

// Division by the constants fx, fy, ds in two operations (Brisebarre,
// Muller & Raina, "Accelerating correctly rounded floating-point division
// when the divisor is known in advance", IEEE TC 2004): for each divisor y,
// h = RN(1/y) and l = RN((1 - y h) / y); then q = RN(n h + RN(n l)) =
// fma(n, h, n * l).  Used only where k_verify_fastdiv finds it equal to IEEE
// n / y on the whole domain the kernels divide.
struct FastK {
    float hfx, lfx, hfy, lfy, hds, lds;
};

// 64-bit lane helpers (two 32-bit halves)
__device__ __forceinline__ double join64(unsigned lo, unsigned hi)
{
    return __hiloint2double((int)hi, (int)lo);
}
__device__ __forceinline__ unsigned lo32(double x) { return (unsigned)__double2loint(x); }
__device__ __forceinline__ unsigned hi32(double x) { return (unsigned)__double2hiint(x); }

// lane `l`'s value in every lane (wave-uniform l: two v_readlane into SGPRs)
__device__ __forceinline__ double readlane64(double x, int l)
{
    return join64((unsigned)__builtin_amdgcn_readlane((int)lo32(x), l),
                  (unsigned)__builtin_amdgcn_readlane((int)hi32(x), l));
}

// fma(n, h, RN(n l)): equal to RN(n / d) wherever k_verify_fastdiv found
// no mismatch (h, l of the divisor d, FastK).
__device__ __forceinline__ float div_fast(float n, float h, float l)
{
    return fmaf(n, h, n * l);
}

template <bool kFast>
__device__ __forceinline__ float bp_div(float n, float d, float h, float l)
{
    return kFast ? div_fast(n, h, l) : n / d;
}

// Spec a7's two projection quotients nu/den and nv/den, IEEE correctly
// rounded, sharing one reciprocal.  hipcc expands an fp32 a/b (denormals on)
// to  s = div_scale(b,b,a); n = div_scale(a,b,a); r = rcp(s);
//     r = fma(fma(-s,r,1), r, r); q = n*r; q = fma(fma(-s,q,n), r, q);
//     q = div_fmas(fma(-s,q,n), r, q); result = div_fixup(q, b, a)   (`make asm`).
// For b in [2^-60, 2^60] div_scale rescales neither operand except when a is
// 0, |a/b| >= ~2^95, |a/b| < 2^-126 or |a| < 2^-103; otherwise div_fmas is a
// plain fma and div_fixup returns q unchanged, so q = RN(n r) with those two
// fma corrections equals a/b bit for bit, and its reciprocal part depends on
// b only (one correction suffices from a correctly rounded r: proj_quot).  In the excepted
// cases the results differ at most between 0 / tiny / huge / inf / NaN
// values, which the projection (+cx, +0.5, floor, range test) maps to the same
// pixel or to "outside".  Callers fall back to a/b when b is out of range.
// youth_icp_selftest_projdiv compares the two bitwise on random and edge
// cases (tests/test_gpu_parity.py).
__device__ __forceinline__ float proj_recip(float den)
{
    const float r0 = __builtin_amdgcn_rcpf(den);
    return fmaf(fmaf(-den, r0, 1.0f), r0, r0);
}
__device__ __forceinline__ bool proj_den_ok(float den)
{
    return (den >= 0x1p-60f) & (den <= 0x1p60f);
}
// Spec a7's projection reciprocal RN(1 / den): for den in [2^-60, 2^60] the
// hardware reciprocal refined by ONE Newton step, fma(fma(-den, r0, 1), r0,
// r0) (proj_recip), is already the correctly rounded 1.0f / den: measured
// for EVERY fp32 den in that range (tools/rcp_probe.hip,
// profiles/r02/rcp_probe.txt: 0 of 1,006,632,961 differ; the two further
// quotient corrections used before changed nothing), and re-checked by
// youth_icp_selftest_projdiv (tests/test_gpu_parity.py).  Outside: IEEE.
__device__ __forceinline__ float proj_rcp_rn(float den)
{
    if (proj_den_ok(den))  // always in practice (den is a depth in metres)
        return proj_recip(den);
    return 1.0f / den;
}

// Which arithmetic spec a7/a8 runs in (youth_icp_set_spec):
//   kSpecSurvey (default) SURVEY.md §8a a7/a8 + §7 literally: separately
//               rounded products and sums in a fixed order (no FMA) and the
//               projection quotient fx P'x / P'z as an IEEE division;
//   kSpecFma    opt-in: fma chains and one correctly rounded reciprocal.
// The oracle restates both (oracle_set_spec); every kernel of the iteration
// (k_icp, k_icp_coop, k_reduce) is instantiated for each.
constexpr int kSpecFma = YOUTH_SPEC_FMA;
constexpr int kSpecSurvey = YOUTH_SPEC_SURVEY;
// ... and for each reduction of spec a9 (youth_icp_set_reduce):
//   lane32 (default) SURVEY.md §8a a9 as worded, "fp32 lanes -> fp64
//          finalize": each lane sums its pixels' 28 products with v_fma_f32
//          over its whole share of a work item, then converts once;
//   exact  every product exact in fp64 (v_fmac_f64 per product).
// The kernels' template parameter kSp is the VARIANT: bit 0 the arithmetic
// (kSpecFma / kSpecSurvey), bit 1 (kRedLane32) the lane32 reduction.
constexpr int kRedLane32 = 2;
constexpr int kVariants = 4;
__host__ __device__ constexpr bool sp_survey(int v) { return (v & 1) == kSpecSurvey; }
__host__ __device__ constexpr bool sp_lane32(int v) { return (v & kRedLane32) != 0; }

// kSpecSurvey's projection quotient RN(n / den) from r = RN(1 / den)
// (proj_recip inside proj_den_ok: correctly rounded, checked exhaustively):
// q0 = RN(n r) is within one ulp of n / den, the remainder n - den q0 is
// exact in one fma, and one correction q0 + (n - den q0) r rounds to
// RN(n / den) (Markstein, IBM J. Res. Dev. 34(1), 1990, Theorem 1; barring
// under/overflow of the remainder, which only happens for quotients that
// project to the same pixel or off the frame).  hipcc's a/b applies two
// such corrections; youth_icp_selftest_projquot compares this one with
// IEEE a/b bitwise and through the projection (tests/test_gpu_parity.py).
__device__ __forceinline__ float proj_quot(float n, float den, float r)
{
    const float q0 = n * r;
    return fmaf(fmaf(-den, q0, n), r, q0);
}

// (int)floorf(x) in one instruction (v_cvt_flr_i32_f32; floorf + the int
// conversion are two 4-cycle VALU forms, profiles/r03/valu_cycles.txt).
// Equal to (int)floorf(x) for every normal or zero x with |x| < 2^30, and
// (unsigned) of it < 16384 exactly when 0 <= floorf(x) < 16384 for every
// non-NaN x but denormals (saturating conversion): youth_icp_selftest_projquot
// checks both over all 2^32 bit patterns.  kSpecSurvey's projected
// coordinate ((q + c) + 0.5) is never NaN (T finite, q finite or +-inf) and
// never denormal (it is 0 or at least 2^-25 in magnitude: s + 0.5 with s a
// float near -0.5 is exact by Sterbenz, |s| < 0.25 leaves it above 0.25).
__device__ __forceinline__ int floor_i32(float x)
{
    int r;
    asm("v_cvt_flr_i32_f32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}

// Spec a6's normalisation n = c / sqrtf(|c|^2) on its common range, bit for
// bit.  hipcc's correctly rounded sqrtf is  x' = x < 2^-96 ? x 2^32 : x;
// s = v_sqrt(x'); s -= (fma(-(s-1ulp), s, x') <= 0); s += (fma(-(s+1ulp), s,
// x') > 0); unscale; return x for +-0 / +inf (`make asm`).  For x in
// [2^-96, 2^118] the scaling and the class fix-up are identities, leaving
// the sequence below.  The three quotients then share one reciprocal
// (norm_div): len = sqrt(x) is in [2^-48, 2^59] and |c_i| <= ~len, so
// div_scale rescales no operand when |c_i| >= 2^-64; c_i = 0
// is exact through the sign: RN(c/len) = copysign(RN(|c|/len), c).  Callers
// take the IEEE expressions when norm_fast_ok is false.
// youth_icp_selftest_normalize checks both against IEEE on device.
__device__ __forceinline__ float sqrt_rn_mid(float x)
{
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sdn = __uint_as_float(__float_as_uint(s) - 1u);
    const float sup = __uint_as_float(__float_as_uint(s) + 1u);
    const float t = fmaf(-sdn, s, x) <= 0.0f ? sdn : s;
    return fmaf(-sup, s, x) > 0.0f ? sup : t;
}
__device__ __forceinline__ bool norm_comp_ok(float c)
{
    return !((fabsf(c) < 0x1p-64f) & (c != 0.0f));
}
__device__ __forceinline__ bool norm_fast_ok(float len2, float cx, float cy, float cz)
{
    return (len2 >= 0x1p-96f) && (len2 <= 0x1p118f) && norm_comp_ok(cx) && norm_comp_ok(cy) &&
           norm_comp_ok(cz);
}
// The three quotients take ONE correction from the correctly rounded
// reciprocal r = RN(1 / len) (proj_recip; len in [2^-48, 2^59]), as the
// projection's proj_quot (Markstein's theorem; youth_icp_selftest_normalize
// compares with IEEE c / sqrtf(len2) bitwise).
__device__ __forceinline__ float norm_div(float c, float len, float r)
{
    return copysignf(proj_quot(fabsf(c), len, r), c);
}
// norm_fast_ok on the bits, for k_prep: len2 (>= +0 or NaN) in [2^-96,
// 2^118] as one unsigned compare; a component c is "tiny" (0 < |c| < 2^-64)
// iff t = 2 bits(c) - 2 (sign shifted out, wrapping: +-0 -> 2^32 - 2) is
// below 2 bits(2^-64) - 2, so the three tests are one min3 and one compare.
// The self-test checks it equals norm_fast_ok on every random vector.
__device__ __forceinline__ bool norm_fast_ok_bits(float len2, float cx, float cy, float cz)
{
    constexpr unsigned kLo = 0x0F800000u, kHi = 0x7A800000u, kTiny = 2u * 0x1F800000u - 2u;
    const unsigned tx = (__float_as_uint(cx) << 1) - 2u, ty = (__float_as_uint(cy) << 1) - 2u,
                   tz = (__float_as_uint(cz) << 1) - 2u;
    return (int)((__float_as_uint(len2) - kLo) <= (kHi - kLo)) & (int)(min(min(tx, ty), tz) >= kTiny);
}

// viewerModule.c:341-345 with explicit intrinsics (bit-identical to the
// viewer for cx = W/2, cy = H/2, f = 570.3f, ds = 1000.0f):
//   valid iff d > 0;  z = d / ds;  x = ((u - cx) z) / fx;  y = ((v - cy) z) / fy
template <bool kFast>
__device__ __forceinline__ void backproject(int d, int u, int v, const Intr& K,
                                            const FastK& F, float& x, float& y, float& z)
{
    const float zz = bp_div<kFast>((float)max(d, 0), K.ds, F.hds, F.lds);  // d <= 0: 0/ds = +0
    x = bp_div<kFast>(((float)u - K.cx) * zz, K.fx, F.hfx, F.lfx);
    y = bp_div<kFast>(((float)v - K.cy) * zz, K.fy, F.hfy, F.lfy);
    z = zz;
}
// The same with the centred pixel coordinates uc = (float)u - cx and
// vc = (float)v - cy supplied (exact: integers below 2^24), so a caller
// walking a row forms them by additions.
template <bool kFast>
__device__ __forceinline__ void backproject_c(int d, float uc, float vc, const Intr& K,
                                              const FastK& F, float& x, float& y, float& z)
{
    const float zz = bp_div<kFast>((float)max(d, 0), K.ds, F.hds, F.lds);
    x = bp_div<kFast>(uc * zz, K.fx, F.hfx, F.lfx);
    y = bp_div<kFast>(vc * zz, K.fy, F.hfy, F.lfy);
    z = zz;
}

// Exhaustive check of div_fast against IEEE division over the whole
// back-projection domain: z = d/ds (d in [1, 32767]); ((u - cx) z)/fx
// (u in [0, W)); ((v - cy) z)/fy (v in [0, H)).  Also covers the target
// recompute in k_reduce (tz is some d/ds, u' in [0, W), v' in [0, H)).
__global__ void k_verify_fastdiv(Intr K, FastK F, int W, int H, unsigned* bad)
{
    const int d = blockIdx.x * blockDim.x + threadIdx.x + 1;
    if (d > 32767) return;
    const float zi = (float)d / K.ds;
    unsigned nb = (div_fast((float)d, F.hds, F.lds) != zi);
    for (int u = blockIdx.y; u < W; u += gridDim.y) {
        const float n = ((float)u - K.cx) * zi;
        nb += (div_fast(n, F.hfx, F.lfx) != n / K.fx);
    }
    for (int v = blockIdx.y; v < H; v += gridDim.y) {
        const float n = ((float)v - K.cy) * zi;
        nb += (div_fast(n, F.hfy, F.lfy) != n / K.fy);
    }
    if (nb) atomicAdd(bad, nb);
}

// Self-test of the projection reciprocal (proj_rcp_rn) against IEEE 1.0f / den:
// bad[0]: bitwise mismatches over EVERY fp32 den in [2^-60, 2^60] (the
//         guarded range: exhaustive, ~1.0e9 values; must be 0);
// bad[1]: mismatches of the projected pixel floor(fma(num, rz, c + 0.5)) and
//         its in-range test [0, 65536) between proj_rcp_rn and 1.0f / den on
//         `n` SplitMix64 cases (den any positive finite fp32 incl. outside the
//         guard, num random with exponent in [-80, 80] or next to a
//         half-integer quotient, c in [0, 4096); must be 0).
__device__ __forceinline__ unsigned long long sm64(unsigned long long& x)
{
    unsigned long long z = (x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__global__ void k_selftest_projdiv(unsigned long long n, unsigned long long seed,
                                   unsigned long long* bad)
{
    unsigned long long b0 = 0, b1 = 0;
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
    const unsigned long long tid = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    constexpr unsigned kLo = 0x21800000u, kHi = 0x5D800000u;  // 2^-60, 2^60
    for (unsigned long long b = kLo + tid; b <= kHi; b += stride) {
        const float den = __uint_as_float((unsigned)b);
        b0 += __float_as_uint(proj_rcp_rn(den)) != __float_as_uint(1.0f / den);
    }
    for (unsigned long long i = tid; i < n; i += stride) {
        unsigned long long st = seed ^ (i * 0xD1B54A32D192ED03ull);
        const unsigned long long r1 = sm64(st), r2 = sm64(st), r3 = sm64(st);
        const int ed = (i & 7) == 7 ? (int)(r1 % 254) - 126 : (int)(r1 % 121) - 60;
        const float den = __uint_as_float((unsigned)((ed + 127) << 23) | (unsigned)(r2 & 0x7FFFFF));
        float num;
        if (i & 1) {  // quotient next to a half-integer: the rounding-critical case
            const float m = (float)((int)(r3 % 8192) - 4096) + 0.5f;
            num = den * m;
            num = __uint_as_float(__float_as_uint(num) + (unsigned)((int)((r3 >> 20) & 7) - 3));
        } else {
            const int e = (int)((r3 >> 8) % 161) - 80;
            num = __uint_as_float((unsigned)((e + 127) << 23) | (unsigned)(r3 & 0x7FFFFF) |
                                  (unsigned)((r3 >> 63) << 31));
        }
        const float c = (float)(r2 >> 52);  // [0, 4096)
        const float ui = floorf(fmaf(num, 1.0f / den, c + 0.5f));
        const float uf = floorf(fmaf(num, proj_rcp_rn(den), c + 0.5f));
        const bool ii = (ui >= 0.0f) & (ui < 65536.0f), inf_ = (uf >= 0.0f) & (uf < 65536.0f);
        if (ii != inf_ || (ii && ui != uf)) ++b1;
    }
    if (b0) atomicAdd(bad + 0, b0);
    if (b1) atomicAdd(bad + 1, b1);
}

// Self-test of kSpecSurvey's projection quotient (proj_quot with
// proj_recip) against IEEE n / den:
//   bad[0]: bitwise quotient mismatches over `n` SplitMix64 cases with den
//           in the guard [2^-60, 2^60] and n of exponent in [-60, 60],
//           half of them next to a rounding midpoint of n / den (n =
//           RN(den (m + ulp(m)/2)) +- a few ulps);
//   bad[1]: mismatches of the projected pixel floor((q + c) + 0.5) and its
//           in-range test [0, 65536), den anywhere in the positive finite
//           fp32 range (outside the guard the kernels divide with IEEE),
//           c in [0, 4096): must be 0 for both;
//   bad[2]: floor_i32 against (int)floorf over ALL 2^32 bit patterns except
//           NaN and denormals: value mismatches where |x| < 2^30, and
//           in-range disagreements ((unsigned)r < 16384 vs 0 <= floorf(x) <
//           16384) anywhere: must be 0.
__device__ __forceinline__ float survey_quot(float n, float den)
{
    if (proj_den_ok(den)) return proj_quot(n, den, proj_recip(den));
    return n / den;
}
__global__ void k_selftest_projquot(unsigned long long n, unsigned long long seed,
                                    unsigned long long* bad)
{
    unsigned long long b0 = 0, b1 = 0;
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
    const unsigned long long tid = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    for (unsigned long long i = tid; i < n; i += stride) {
        unsigned long long st = seed ^ (i * 0xD1B54A32D192ED03ull);
        const unsigned long long r1 = sm64(st), r2 = sm64(st), r3 = sm64(st);
        // guard-range quotient check
        {
            const int ed = (int)(r1 % 121) - 60;
            const float den = __uint_as_float((unsigned)((ed + 127) << 23) | (unsigned)(r2 & 0x7FFFFF));
            float num;
            if (i & 1) {
                const int em = (int)((r3 >> 40) % 41) - 20;
                const float m = __uint_as_float((unsigned)((em + 127) << 23) | (unsigned)(r3 & 0x7FFFFF));
                const double mid = (double)m + 0.5 * ((double)__uint_as_float(__float_as_uint(m) + 1u) - (double)m);
                num = (float)((double)den * mid);
                num = __uint_as_float(__float_as_uint(num) + (unsigned)((int)((r3 >> 23) & 7) - 3));
            } else {
                const int e = (int)((r3 >> 8) % 121) - 60;
                num = __uint_as_float((unsigned)((e + 127) << 23) | (unsigned)(r3 & 0x7FFFFF) |
                                      (unsigned)((r3 >> 63) << 31));
            }
            b0 += __float_as_uint(survey_quot(num, den)) != __float_as_uint(num / den);
        }
        // projected pixel, den over the whole positive range
        {
            const int ed = (i & 7) == 7 ? (int)(r2 % 254) - 126 : (int)(r2 % 121) - 60;
            const float den = __uint_as_float((unsigned)((ed + 127) << 23) | (unsigned)(r1 & 0x7FFFFF));
            float num;
            if (i & 2) {
                const float m = (float)((int)(r3 % 8192) - 4096) + 0.5f;
                num = den * m;
                num = __uint_as_float(__float_as_uint(num) + (unsigned)((int)((r3 >> 20) & 7) - 3));
            } else {
                const int e = (int)((r3 >> 8) % 161) - 80;
                num = __uint_as_float((unsigned)((e + 127) << 23) | (unsigned)(r3 & 0x7FFFFF) |
                                      (unsigned)((r3 >> 63) << 31));
            }
            const float c = (float)(r1 >> 52);
            const float ui = floorf((num / den + c) + 0.5f);
            const float uf = floorf((survey_quot(num, den) + c) + 0.5f);
            const bool ii = (ui >= 0.0f) & (ui < 65536.0f), inf_ = (uf >= 0.0f) & (uf < 65536.0f);
            if (ii != inf_ || (ii && ui != uf)) ++b1;
        }
    }
    unsigned long long b2 = 0;
    for (unsigned long long b = tid; b < (1ull << 32); b += stride) {
        const float x = __uint_as_float((unsigned)b);
        if (x != x || (x != 0.0f && fabsf(x) < 0x1p-126f)) continue;  // NaN, denormal
        const float f = floorf(x);
        const int r = floor_i32(x);
        const bool in_ref = (f >= 0.0f) & (f < 16384.0f);
        const bool in_got = (unsigned)r < 16384u;
        b2 += (in_ref != in_got) || (fabsf(x) < 0x1p30f && r != (int)f);
    }
    if (b0) atomicAdd(bad + 0, b0);
    if (b1) atomicAdd(bad + 1, b1);
    if (b2) atomicAdd(bad + 2, b2);
}

// Self-test of k_prep's fast normalisation (sqrt_rn_mid, norm_div):
//   bad[0]: sqrt_rn_mid(x) != sqrtf(x) over EVERY fp32 x in [2^-96, 2^118];
//   bad[1]: bitwise differences of (nx, ny, nz) vs c / sqrtf(len2) over `n`
//           random vectors (components of mixed magnitude down to 2^-110,
//           each +-0 with probability 1/8), wherever norm_fast_ok holds,
//           plus every vector where norm_fast_ok_bits differs from it;
//   bad[2]: number of random vectors that took the fast path (coverage).
__global__ void k_selftest_normalize(unsigned long long n, unsigned long long seed,
                                     unsigned long long* bad)
{
    unsigned long long b0 = 0, b1 = 0, nf = 0;
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
    const unsigned long long tid = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    constexpr unsigned kLo = 0x0F800000u, kHi = 0x7A800000u;  // 2^-96, 2^118
    for (unsigned long long b = kLo + tid; b <= kHi; b += stride) {
        const float x = __uint_as_float((unsigned)b);
        b0 += __float_as_uint(sqrt_rn_mid(x)) != __float_as_uint(sqrtf(x));
    }
    for (unsigned long long i = tid; i < n; i += stride) {
        unsigned long long st = seed ^ (i * 0xD1B54A32D192ED03ull);
        const int e0 = (int)(sm64(st) % 131) - 70;  // leading exponent in [-70, 60]
        float c[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const unsigned long long r = sm64(st);
            const int e = max(e0 - (int)((r >> 32) % 48), -126);
            const unsigned sign = (unsigned)(r >> 63) << 31;
            c[k] = ((r >> 56) & 7) == 0
                       ? __uint_as_float(sign)
                       : __uint_as_float(sign | (unsigned)((e + 127) << 23) |
                                         (unsigned)(r & 0x7FFFFF));
        }
        const float len2 = (c[0] * c[0] + c[1] * c[1]) + c[2] * c[2];
        b1 += norm_fast_ok_bits(len2, c[0], c[1], c[2]) != norm_fast_ok(len2, c[0], c[1], c[2]);
        if (!(len2 > 0.0f) || !norm_fast_ok(len2, c[0], c[1], c[2])) continue;
        ++nf;
        const float len = sqrt_rn_mid(len2), r = proj_recip(len), ref = sqrtf(len2);
#pragma unroll
        for (int k = 0; k < 3; ++k)
            b1 += __float_as_uint(norm_div(c[k], len, r)) != __float_as_uint(c[k] / ref);
    }
    if (b0) atomicAdd(bad + 0, b0);
    if (b1) atomicAdd(bad + 1, b1);
    if (nf) atomicAdd(bad + 2, nf);
}

// ------------------------------------------------------------------ k_prep --
// grid (ceil(W/64), ceil(H/16), n_frames): frame f reads depth + f*N and
// writes the target records of workspace frame out0 + f (and, when xyz is
// non-null, its X/Y/Z planes: stage-level API only).  Normals (spec a6):
// n = normalize((P(u+1)-P(u-1)) x (P(v+1)-P(v-1))); (0,0,0) on the 1-px
// border, if the centre or any of the 4 neighbours is invalid, or if the
// cross product is zero; oriented so n.P <= 0.
// One kTileW x kTH tile of target records (and optional X/Y/Z planes) by a
// workgroup of kThreads: the (kTH+2) x (kTileW+2) back-projected
// neighbourhood is staged in the LDS planes sX/sY/sZ ([kTH+2][kLdsW]), then
// each thread forms the records of column tx = t & 63, rows ty, ty +
// kThreads/64, ...  kSc1: records are stored write-through (16-byte sc1
// buffer stores) for an in-launch hand-off (k_icp_coop).  Contains a
// workgroup barrier (every thread must call it); a caller reusing the LDS
// planes for another tile adds one more before it.
template <bool kFast, bool kWide, bool kSc1, int kThreads, int kTH, int kTW = kTileW>
__device__ __forceinline__ void prep_tile(const int16_t* __restrict__ dep, float4* __restrict__ R,
                                          int W, int H, size_t P, const Intr& K, const FastK& F,
                                          float* __restrict__ X, int x0, int y0, float* sX,
                                          float* sY, float* sZ)
{
    constexpr int kLH = kTH + 2;
    constexpr int kLW = kTW + 2;
    static_assert(kTW % 64 == 0 && kThreads % kTW == 0, "rows of whole waves");
    // the record loop below covers kTH rows in steps of kThreads / kTW: a
    // tile height that is not a multiple would leave its bottom rows unwritten
    static_assert(kTH % (kThreads / kTW) == 0, "tile rows a multiple of the rows per step");
    // the three LDS planes of the halo'd tile must fit a workgroup's 160 KB
    static_assert(3 * (kTH + 2) * (kTW + 2) * sizeof(float) <= 160 * 1024, "LDS planes fit");
    const int tx = threadIdx.x % kTW;
    const int ty = threadIdx.x / kTW;
    if (kWide) {
        // W % 4 == 0 (and an 8-byte-aligned frame): the tile's own columns
        // [x0, x0 + kTW) as kTW / 4 aligned 8-byte words per halo row (each
        // word's 4 pixels all inside or all outside the image, so no lane
        // straddles an edge and every pixel of a word is stored), then the two
        // edge columns x0 - 1 and x0 + kTW one pixel per lane.  An outside
        // pixel back-projects d = 0 at its own (u, v), as before.
        // Words load through a buffer descriptor over the frame: a row
        // outside the image or a word past the right edge takes the offset
        // W H 2 (the descriptor's size: past it, with no 32-bit wrap of
        // offset + bytes), which the range check returns as 0 (no branch, no
        // 64-bit address arithmetic).  The edge pixels are loaded first, so
        // their latency overlaps the words' instead of adding a round trip
        // before the barrier.
        static_assert(2 * kLH <= kThreads, "one edge pixel per thread");
        const bool edge = threadIdx.x < 2 * kLH;
        const int ely = threadIdx.x >> 1, eright = threadIdx.x & 1;
        const int egy = y0 - 1 + ely, egx = eright ? x0 + kTW : x0 - 1;
        const __amdgpu_buffer_rsrc_t rdep = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<int16_t*>(dep), (short)0, W * H * (int)sizeof(int16_t), 0x00020000);
        const bool ein = edge & ((unsigned)egy < (unsigned)H) & ((unsigned)egx < (unsigned)W);
        unsigned short dedge =
            __builtin_amdgcn_raw_buffer_load_b16(rdep, ein ? (egy * W + egx) * 2 : W * H * 2, 0, 0);
        // every word of the thread is requested before the first is used
        // (kIt loads in flight: 2 at 128 x 24 by 512 threads)
        constexpr int kWords = kTW / 4;  // 32 at 128: a shift, not a divide
        constexpr int kIt = (kLH * kWords + kThreads - 1) / kThreads;
        short4 wd[kIt];
#pragma unroll
        for (int it = 0; it < kIt; ++it) {
            const int e = threadIdx.x + it * kThreads;
            const int ly = e / kWords;
            const int gy = y0 - 1 + ly;
            const int c = x0 + 4 * (e - ly * kWords);
            const bool inside = (e < kLH * kWords) & ((unsigned)gy < (unsigned)H) & (c < W);
            wd[it] = __builtin_bit_cast(
                short4, __builtin_amdgcn_raw_buffer_load_b64(rdep, inside ? (gy * W + c) * 2 : W * H * 2, 0, 0));
        }
        // the loads above stay where they are: each result passes through an
        // empty asm here (the frame pointer is __restrict__, so a memory
        // clobber would not pin them), one wait for all of them
#pragma unroll
        for (int it = 0; it < kIt; ++it) {
            unsigned long long v = __builtin_bit_cast(unsigned long long, wd[it]);
            asm volatile("" : "+v"(v));
            wd[it] = __builtin_bit_cast(short4, v);
        }
        {
            unsigned v = dedge;
            asm volatile("" : "+v"(v));
            dedge = (unsigned short)v;
        }
#pragma unroll
        for (int it = 0; it < kIt; ++it) {
            const int e = threadIdx.x + it * kThreads;
            if (e >= kLH * kWords) break;
            const int ly = e / kWords;
            const int m = e - ly * kWords;
            const int gy = y0 - 1 + ly;
            const int c = x0 + 4 * m;
            const short4 d4 = wd[it];
            const int dv[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int lx = 4 * m + 1 + q;  // LDS column of pixel c + q
                float x, y, z;
                backproject<kFast>(dv[q], c + q, gy, K, F, x, y, z);
                sX[ly * kLW + lx] = x;
                sY[ly * kLW + lx] = y;
                sZ[ly * kLW + lx] = z;
            }
        }
        if (edge) {
            float x, y, z;
            backproject<kFast>((int)(short)dedge, egx, egy, K, F, x, y, z);
            const int lx = eright ? kLW - 1 : 0;
            sX[ely * kLW + lx] = x;
            sY[ely * kLW + lx] = y;
            sZ[ely * kLW + lx] = z;
        }
    } else {
        for (int e = threadIdx.x; e < kLH * kLW; e += kThreads) {
            const int ly = e / kLW;
            const int lx = e - ly * kLW;
            const int gx = x0 - 1 + lx, gy = y0 - 1 + ly;
            float x = 0.0f, y = 0.0f, z = 0.0f;
            if (gx >= 0 && gx < W && gy >= 0 && gy < H)
                backproject<kFast>(dep[(size_t)gy * W + gx], gx, gy, K, F, x, y, z);
            sX[ly * kLW + lx] = x;
            sY[ly * kLW + lx] = y;
            sZ[ly * kLW + lx] = z;
        }
    }
    __syncthreads();

    const __amdgpu_buffer_rsrc_t rrec =
        __builtin_amdgcn_make_buffer_rsrc(R, (short)0, (int)(P * sizeof(float4)), 0x00020000);
    // the row of each step is wave-uniform (ty = wave index): its tests and
    // offsets stay on the scalar unit
    const int tyw = __builtin_amdgcn_readfirstlane(ty);
#pragma unroll
    for (int k = 0; k < kTH / (kThreads / kTW); ++k) {
        const int row = tyw + (kThreads / kTW) * k;
        const int gx = x0 + tx, gy = y0 + row;
        if (gx >= W || gy >= H) continue;
        const size_t i = (size_t)gy * W + gx;
        const int ly = row + 1, lx = tx + 1;
        const int o = ly * kLW + lx;
        const float px = sX[o], py = sY[o], pz = sZ[o];
        if (X) {
            X[i] = px;
            X[P + i] = py;
            X[2 * P + i] = pz;
        }
        // branch-free: every lane forms the normal from its LDS neighbours
        // (the halo exists for every pixel of the tile) and the record is
        // selected at the end.  Every z is >= +0 (back-projection of
        // max(d, 0), 0 outside the image), so the five z > 0 tests are one
        // test of their minimum, taken on the bits (the same order for
        // non-negative floats; +0 is bits 0)
        const bool inner = (gx > 0) & (gy > 0) & (gx < W - 1) & (gy < H - 1);
        const float zl = sZ[o - 1], zr = sZ[o + 1];
        const float zu = sZ[o - kLW], zd = sZ[o + kLW];
        const unsigned zmin = min(min(min(__float_as_uint(pz), __float_as_uint(zl)),
                                      min(__float_as_uint(zr), __float_as_uint(zu))),
                                  __float_as_uint(zd));
        const float ax = sX[o + 1] - sX[o - 1];
        const float ay = sY[o + 1] - sY[o - 1];
        const float az = zr - zl;
        const float bx = sX[o + kLW] - sX[o - kLW];
        const float by = sY[o + kLW] - sY[o - kLW];
        const float bz = zd - zu;
        const float cx = ay * bz - az * by;
        const float cy = az * bx - ax * bz;
        const float cz = ax * by - ay * bx;
        const float len2 = (cx * cx + cy * cy) + cz * cz;
        const bool has_n = inner & (zmin != 0u) & (len2 > 0.0f);
        const float len = sqrt_rn_mid(len2);
        const float r = proj_recip(len);
        float nx = norm_div(cx, len, r);
        float ny = norm_div(cy, len, r);
        float nz = norm_div(cz, len, r);
        if (__builtin_expect(has_n & !norm_fast_ok_bits(len2, cx, cy, cz), 0)) {
            const float l = sqrtf(len2);  // correctly rounded (checked in .s)
            nx = cx / l;
            ny = cy / l;
            nz = cz / l;
        }
        // oriented so n.P <= 0
        if (((nx * px + ny * py) + nz * pz) > 0.0f) {
            nx = -nx;
            ny = -ny;
            nz = -nz;
        }
        if (!has_n) nx = ny = nz = 0.0f;
        // a target without a normal is stored as z = 0 ("invalid target"):
        // the spec's two tests "target valid" and "normal valid" become the
        // one tz > 0 test in the pixel loop (the Z plane keeps pz)
        const float4 rec = make_float4(has_n ? pz : 0.0f, nx, ny, nz);
        if (kSc1) {
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, rec), rrec,
                                                   (int)(i * sizeof(float4)), 0, 16);
        } else {
            // non-temporal (aux 2: nt): k_prep's 16 B/px stream of records is
            // read back by k_icp only after the whole batch is written (610 vs
            // 626 us per 512 frames, profiles/r02/ab_s30.txt, ab_s31.txt);
            // through the frame's buffer descriptor: a 32-bit byte offset
            // instead of 64-bit address arithmetic per record
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, rec), rrec,
                                                   (int)(i * sizeof(float4)), 0, 2);
        }
    }
}

// The persistent path's per-call state, set by k_prep's tile-(0,0) blocks
// (k_init's work folded in: one launch and its gap less per align): pair p's
// T64/T32 from T_init (or identity), status 0, epoch 0, arrival tickets 0;
// block (0,0,0) also zeroes the queue words.  n == 0: nothing.
struct InitArgs {
    const double* T_init;
    int n;
    double* T64;
    float* T32;
    int32_t* status;
    unsigned* epoch;
    unsigned* arrivals;  // [pair][iters]
    int iters;
    unsigned* head_err;
};

__device__ __forceinline__ void init_pairs(const InitArgs& ia, int tx, int ty, int f, int n_frames)
{
    if (tx != 0 || ty != 0) return;
    if (f == 0 && threadIdx.x < kMaxQueues && ia.head_err) {
        if (threadIdx.x == 0) {
            ia.head_err[kQHead] = 0u;
            ia.head_err[kQError] = 0u;
            ia.head_err[kQSpins] = 0u;
            ia.head_err[kQWaited] = 0u;
        }
        ia.head_err[kQHeads + kQHeadStride * threadIdx.x] = 0u;  // queue heads
    }
    const int t = threadIdx.x;
    for (int p = f; p < ia.n; p += n_frames) {
        if (t < 16) {
            const double v = ia.T_init ? ia.T_init[(size_t)p * 16 + t] : ((t % 5) == 0 ? 1.0 : 0.0);
            ia.T64[(size_t)p * 16 + t] = v;
            if (t < 12) ia.T32[(size_t)p * 12 + t] = (float)v;
        } else if (t == 16) {
            ia.status[p] = 0;
            ia.epoch[p] = 0u;
        } else {
            for (int k = t - 17; k < ia.iters; k += kPrepThreads - 17)
                ia.arrivals[(size_t)p * ia.iters + k] = 0u;
        }
    }
}

// One workgroup per 64 x 48 tile; a 1-D grid of tiles_x x tiles_y x n_frames
// workgroups.  xcd_map = 1: workgroups are dealt round-robin over the 8 XCDs
// (b and b + 8 share one; MI355X_MICROARCH.md "Workgroup dispatch"), so
// workgroup b takes tile t = (its XCD's share start) + b / 8: each XCD walks
// ONE contiguous run of tiles (frame-major, row-major within a frame), and a
// tile's horizontal and vertical halo lines belong to tiles that the same
// XCD processes at about the same time, i.e. are hits in that XCD's L2
// instead of fetches of lines that neighbouring tiles on other XCDs own.
// xcd_map = 2: each XCD takes whole rows of tiles, rows dealt round-robin
// (row R on XCD R % 8, its tiles in order), so the 8 XCDs work on 8
// adjacent tile rows of one frame at a time: a tile's horizontal halo lines
// belong to its own row (same XCD) and only the top / bottom halo rows (2 of
// 50) come from another XCD's row.  The grid is padded to a multiple of 8
// rows x tiles_x; padding workgroups return -1.
// xcd_map = 0: t = b (row-major over the frames: neighbours on other XCDs).
__device__ __forceinline__ int xcd_tile(int b, int total)
{
    const int q = total >> 3, r = total & 7, x = b & 7, j = b >> 3;
    return x < r ? x * (q + 1) + j : r * (q + 1) + (x - r) * q + j;
}
__device__ __forceinline__ int xcd_row_tile(int b, int tiles_x, int rows)
{
    const int j = b >> 3;
    const int R = (j / tiles_x) * 8 + (b & 7);
    return R < rows ? R * tiles_x + (j - (j / tiles_x) * tiles_x) : -1;
}

template <bool kFast, bool kWide>
__global__ __launch_bounds__(kPrepThreads) void k_prep(const int16_t* __restrict__ depth, int out0,
                                                      int W, int H, size_t P, Intr K, FastK F,
                                                      float4* __restrict__ recs,
                                                      float* __restrict__ xyz, InitArgs ia,
                                                      int tiles_x, int tiles_y, int n_frames,
                                                      int xcd_map)
{
    const int total = tiles_x * tiles_y * n_frames;
    const int t = xcd_map == 1   ? xcd_tile((int)blockIdx.x, total)
                  : xcd_map == 2 ? xcd_row_tile((int)blockIdx.x, tiles_x, tiles_y * n_frames)
                                 : (int)blockIdx.x;
    if (t < 0) return;  // grid padding (xcd_map 2)
    const int per = tiles_x * tiles_y;
    const int f = t / per;
    const int r = t - f * per;
    const int ty = r / tiles_x;
    const int tx = r - ty * tiles_x;
    init_pairs(ia, tx, ty, f, n_frames);
    __shared__ float sX[(kPrepTH + 2) * (kPrepTW + 2)];
    __shared__ float sY[(kPrepTH + 2) * (kPrepTW + 2)];
    __shared__ float sZ[(kPrepTH + 2) * (kPrepTW + 2)];
    const size_t N = (size_t)W * (size_t)H;
    prep_tile<kFast, kWide, false, kPrepThreads, kPrepTH, kPrepTW>(
        depth + (size_t)f * N, recs + (size_t)(out0 + f) * P, W, H, P, K, F,
        xyz ? xyz + (size_t)(out0 + f) * 3 * P : nullptr, tx * kPrepTW, ty * kPrepTH, sX, sY, sZ);
}

// ----------------------------------------------------------------- k_solve --
// Spec a10 (round 5): A x = b by block elimination with 3x3 adjugates, xi =
// -x; the same correctly rounded operations in the same order as
// oracle_solve (oracle/icp_oracle.c), so xi and the status are bit-identical.
// With P = A[0..2][0..2] (rotation), Q = A[0..2][3..5], R = A[3..5][3..5],
// b = (b1, b2), C = adj(P):
//   detP = P00 C00 + P01 C01 + P02 C02, M = C Q, u = C b1
//   S' = detP R - Q^T M (detP times the Schur complement), y' = detP b2 - Q^T u
//   x2 = adj(S') y' * (1 / det S'),  x1 = C (b1 - Q x2) * (1 / detP)
// ONE division on the dependent chain (1 / detP runs beside it) and no value
// crosses lanes, against LDL^T's six dependent reciprocals and lane
// broadcasts (tools/solvebench).  The rotation block goes first,
// as LDL^T's pivot order does: eliminating the translation block first was
// faster on paper but 2-3x more sensitive to the sums' last bits on
// ill-conditioned frames.  DEGENERATE iff an LDL^T pivot is
// <= 1e-12 max diag, tested on the leading minors by products.
__device__ __forceinline__ double dd2(double a, double b, double c, double d)
{
    return fma(a, b, -(c * d));  // a b - c d
}
__device__ __forceinline__ double dot3(double a0, double b0, double a1, double b1, double a2,
                                       double b2)
{
    return fma(a2, b2, fma(a1, b1, a0 * b0));
}
// symmetric 3x3 {m00, m01, m02, m11, m12, m22}: adjugate, matrix-vector
__device__ __forceinline__ void adj3(const double* p, double* c)
{
    c[0] = dd2(p[3], p[5], p[4], p[4]);
    c[1] = dd2(p[2], p[4], p[1], p[5]);
    c[2] = dd2(p[1], p[4], p[2], p[3]);
    c[3] = dd2(p[0], p[5], p[2], p[2]);
    c[4] = dd2(p[1], p[2], p[0], p[4]);
    c[5] = dd2(p[0], p[3], p[1], p[1]);
}
__device__ __forceinline__ void symv3(const double* c, const double* v, double* o)
{
    o[0] = dot3(c[0], v[0], c[1], v[1], c[2], v[2]);
    o[1] = dot3(c[1], v[0], c[3], v[1], c[4], v[2]);
    o[2] = dot3(c[2], v[0], c[4], v[1], c[5], v[2]);
}
// neq wave-uniform (LDS or registers); every lane computes everything, so no
// value crosses lanes.  xi is zeroed on a nonzero status.
__device__ __forceinline__ int solve_block6(const double* neq, double xi[6])
{
#pragma unroll
    for (int i = 0; i < 6; ++i) xi[i] = 0.0;
    if (!(neq[28] >= 6.0)) return YOUTH_STATUS_FEW_MATCHES;
    double maxd = 0.0;  // the diagonal, in order (a, a) = 0, 6, 11, 15, 18, 20
    maxd = neq[0] > maxd ? neq[0] : maxd;
    maxd = neq[6] > maxd ? neq[6] : maxd;
    maxd = neq[11] > maxd ? neq[11] : maxd;
    maxd = neq[15] > maxd ? neq[15] : maxd;
    maxd = neq[18] > maxd ? neq[18] : maxd;
    maxd = neq[20] > maxd ? neq[20] : maxd;
    if (!(maxd > 0.0)) return YOUTH_STATUS_DEGENERATE;
    const double eps = 1e-12 * maxd;
    const double P[6] = {neq[0], neq[1], neq[2], neq[6], neq[7], neq[11]};
    const double R[6] = {neq[15], neq[16], neq[17], neq[18], neq[19], neq[20]};
    const double Q[3][3] = {{neq[3], neq[4], neq[5]}, {neq[8], neq[9], neq[10]},
                            {neq[12], neq[13], neq[14]}};
    const double b1[3] = {neq[21], neq[22], neq[23]}, b2[3] = {neq[24], neq[25], neq[26]};
    double C[6], E[6], S[6], M[3][3], u[3], y[3], v[3], x2[3], w[3];
    adj3(P, C);
    const double detP = dot3(P[0], C[0], P[1], C[1], P[2], C[2]);
#pragma unroll
    for (int j = 0; j < 3; ++j) {  // M = C Q, column by column
        const double q[3] = {Q[0][j], Q[1][j], Q[2][j]};
        double o[3];
        symv3(C, q, o);
        M[0][j] = o[0];
        M[1][j] = o[1];
        M[2][j] = o[2];
    }
    symv3(C, b1, u);
    // S' upper triangle (i <= j): detP R[i][j] - (Q^T M)[i][j]
    S[0] = fma(detP, R[0], -dot3(Q[0][0], M[0][0], Q[1][0], M[1][0], Q[2][0], M[2][0]));
    S[1] = fma(detP, R[1], -dot3(Q[0][0], M[0][1], Q[1][0], M[1][1], Q[2][0], M[2][1]));
    S[2] = fma(detP, R[2], -dot3(Q[0][0], M[0][2], Q[1][0], M[1][2], Q[2][0], M[2][2]));
    S[3] = fma(detP, R[3], -dot3(Q[0][1], M[0][1], Q[1][1], M[1][1], Q[2][1], M[2][1]));
    S[4] = fma(detP, R[4], -dot3(Q[0][1], M[0][2], Q[1][1], M[1][2], Q[2][1], M[2][2]));
    S[5] = fma(detP, R[5], -dot3(Q[0][2], M[0][2], Q[1][2], M[1][2], Q[2][2], M[2][2]));
#pragma unroll
    for (int j = 0; j < 3; ++j)
        y[j] = fma(detP, b2[j], -dot3(Q[0][j], u[0], Q[1][j], u[1], Q[2][j], u[2]));
    adj3(S, E);
    const double detS = dot3(S[0], E[0], S[1], E[1], S[2], E[2]);
    const double epsP = eps * detP;
    // pivots P00, C22/P00, detP/C22, S'00/detP, E22/(detP S'00), detS/(detP E22)
    const bool ok = (P[0] > eps) & (C[5] > eps * P[0]) & (detP > eps * C[5]) & (S[0] > epsP) &
                    (E[5] > epsP * S[0]) & (detS > epsP * E[5]);
    if (!ok) return YOUTH_STATUS_DEGENERATE;
    const double rS = 1.0 / detS, rP = 1.0 / detP;
    symv3(E, y, v);
#pragma unroll
    for (int i = 0; i < 3; ++i) x2[i] = v[i] * rS;
#pragma unroll
    for (int i = 0; i < 3; ++i) w[i] = b1[i] - dot3(Q[i][0], x2[0], Q[i][1], x2[1], Q[i][2], x2[2]);
    symv3(C, w, v);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        xi[i] = -(v[i] * rP);
        xi[3 + i] = -x2[i];
    }
    return 0;
}

__device__ void se3_exp_left(const double xi[6], double* T)
{
    const double wx = xi[0], wy = xi[1], wz = xi[2];
    const double th2 = (wx * wx + wy * wy) + wz * wz;
    double a, b, c;
    if (th2 < 0x1p-7) {  // spec a10: Taylor in th2 (oracle_se3_exp: same fma chain)
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

// Spec a10 by ONE wave (all 64 lanes call it): solve_block6 in every lane
// (wave-uniform, no cross-lane traffic), then se3_exp_left with its
// per-element operations and order, lane l < 12 computing output entry
// (l / 4, l % 4) of exp(xi^) T.  neq (LDS, kNeq): the pair's sums; T64 (LDS,
// 12): pose in/out; T32 (LDS, 12): fp32 copy out.  Returns the status bits;
// the pose is updated only when they are 0.
__device__ __forceinline__ int solve_update_wave(const double* neq, double* T64, float* T32, int lane)
{
    double xi[6];
    const int st = solve_block6(neq, xi);
    if (st) return st;

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

// Out-of-line copy for k_icp: inlined there, the solve's loop-invariant
// constants are hoisted into the kernel prologue and spilled across the
// pixel loop (128-VGPR budget), then reloaded from scratch on the pair's
// critical path.  A call keeps its registers to itself.
__device__ __attribute__((noinline)) int solve_update_wave_call(const double* neq, double* T64,
                                                                float* T32, int lane)
{
    return solve_update_wave(neq, T64, T32, lane);
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
    const int st = solve_block6(neq, xi);
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

// T64 <- T_init (or identity), T32 <- float(T64), status <- 0; zero the
// persistent kernel's epoch/arrival words and its dequeue head + error flag
// (G16: every polled word is re-initialised on every call).
__global__ void k_init(const double* __restrict__ T_init, int n, double* T64, float* T32,
                       int32_t* status, unsigned* epoch, unsigned* arrivals, int iters,
                       unsigned* head_err)
{
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p == 0 && head_err) {  // one 128-B line each (kQ*): no false sharing
        head_err[kQHead] = 0u;     // dequeue head (contended atomic)
        head_err[kQError] = 0u;    // timeout flag (polled by waiters)
        head_err[kQSpins] = 0u;    // epoch polls (scheduler telemetry)
        head_err[kQWaited] = 0u;   // items that had to wait for their pair's pose
        for (int q = 0; q < kMaxQueues; ++q) head_err[kQHeads + kQHeadStride * q] = 0u;
    }
    if (p >= n) return;
    for (int i = 0; i < 16; ++i) {
        const double v = T_init ? T_init[(size_t)p * 16 + i] : ((i % 5) == 0 ? 1.0 : 0.0);
        T64[(size_t)p * 16 + i] = v;
        if (i < 12) T32[(size_t)p * 12 + i] = (float)v;
    }
    status[p] = 0;
    if (epoch) epoch[p] = 0u;
    if (arrivals)
        for (int k = 0; k < iters; ++k) arrivals[(size_t)p * iters + k] = 0u;
}


// ---------------------------------------------------------------- k_reduce --
// Spec a7-a9 for four consecutive source pixels per lane per step.
//   source  int16 depth (2 B/px), back-projected in registers (8-byte load
//           per lane when the frame is 8-byte aligned and W % 4 == 0);
//   target  ONE aligned 16-byte record fetch {z, nx, ny, nz} per pixel; the
//           target's x, y are recomputed from z with k_prep's expression, so
//           they are bit-identical to what k_prep would have stored.
// Branch-free: invalid lanes compute on safe values and are masked, so the
// four fetches issue back to back.  Accumulators are fp64 fed with exact
// fp32 products: the result equals the oracle's row-major fp64 sum up to
// fp64 summation order.  (tools/kbench: 205 us for the first SoA version ->
// 107 us for this one at 64 pairs, partial sums unchanged.)
struct PairMap {
    int src0, tgt0;  // pair p: source depth frame src0 + p, target record frame tgt0 + p
};

template <bool kAligned>
__device__ __forceinline__ short4 load_depth4(const int16_t* __restrict__ sD, int i, int end)
{
    // i < end always here; kAligned => i % 4 == 0 and i + 3 < end
    short4 d;
    if (kAligned) {
        d = *reinterpret_cast<const short4*>(sD + i);
    } else {
        d.x = sD[i];
        d.y = (i + 1) < end ? sD[i + 1] : (short)0;
        d.z = (i + 2) < end ? sD[i + 2] : (short)0;
        d.w = (i + 3) < end ? sD[i + 3] : (short)0;
    }
    return d;
}

// Per-iteration pose state for the fused solve (kFuse).  T32 is read by
// every workgroup of pair p at entry and rewritten only by p's LAST
// workgroup, after all of p's workgroups have arrived (so after they read it).
struct PoseState {
    double* T64;          // [pair][16]
    float* T32;           // [pair][12]
    int32_t* status;      // [pair]
    double* stats;        // [pair][iters][2] or null
    unsigned* arrivals;   // [pair], zero at launch; re-armed by the last arriver
    int it, iters;
};

// ------------------------------------------------- spec a7-a9 per pixel --
// Shared by k_reduce / k_icp (accumulate_chunk) and k_icp_coop (coop_group);
// oracle/icp_oracle.c assoc_one / oracle_reduce evaluate the same operations
// with the same roundings (fmaf = one rounding, -ffp-contract=off elsewhere).
//   a7  P' = R P + t:  P'_i = fma(R_i2, z, fma(R_i1, y, fma(R_i0, x, t_i)))
//       valid iff z > 0 and P'_z > 0;  rz = RN(1 / P'_z);
//       u' = floor(fma(fx P'_x, rz, cx + 0.5)), v' likewise; in range of the
//       target frame.  Unmatched pixels compute on safe values (branch-free)
//       and gather record 0.
//   kSpecSurvey: P'_i = ((R_i0 x + R_i1 y) + R_i2 z) + t_i and
//       u' = floor(((fx P'_x) / P'_z + cx) + 0.5), the
//       quotient IEEE (proj_quot on the shared correctly rounded reciprocal).
// Lane masks (one bit per lane of the wave, bit set only on active lanes):
// compares go straight to SGPR masks (v_cmp), combine on the scalar unit and
// feed selects through inverse_ballot, and a wave's match count is one
// s_bcnt1; a per-lane boolean would be rebuilt from a 0/1 select and a
// compare wherever it is counted (two 4-cycle VALU forms per pixel).
typedef unsigned long long LaneMask;
constexpr int kFcmpOgt = 2, kFcmpOlt = 4, kIcmpUlt = 36, kIcmpUle = 37;
__device__ __forceinline__ LaneMask mask_gt(float a, float b) { return __builtin_amdgcn_fcmpf(a, b, kFcmpOgt); }
__device__ __forceinline__ LaneMask mask_lt(float a, float b) { return __builtin_amdgcn_fcmpf(a, b, kFcmpOlt); }
__device__ __forceinline__ LaneMask mask_ult(unsigned a, unsigned b) { return __builtin_amdgcn_uicmp(a, b, kIcmpUlt); }
__device__ __forceinline__ LaneMask mask_ule(unsigned a, unsigned b) { return __builtin_amdgcn_uicmp(a, b, kIcmpUle); }
__device__ __forceinline__ bool lane_in(LaneMask m) { return __builtin_amdgcn_inverse_ballot_w64(m); }

template <int kSp>
__device__ __forceinline__ void xform_project(const float* T, float sx, float sy, float sz,
                                              const Intr& K, int W, int H, float& qx, float& qy,
                                              float& qz, float& fu, float& fv, LaneMask& inm, int& j)
{
    if (sp_survey(kSp)) {
        qx = ((T[0] * sx + T[1] * sy) + T[2] * sz) + T[3];
        qy = ((T[4] * sx + T[5] * sy) + T[6] * sz) + T[7];
        qz = ((T[8] * sx + T[9] * sy) + T[10] * sz) + T[11];
        const float nu = K.fx * qx, nv = K.fy * qy;
        // P'_z in [2^-60, 2^60] (proj_den_ok, which implies P'_z > 0) as ONE
        // unsigned compare on its bits (negative and NaN bit patterns lie
        // above 2^60's): every lane takes the fast quotient with den = P'_z;
        // a valid source whose P'_z is <= 0 or outside the range (never in
        // practice) redoes it below as the IEEE division of the spec.  The
        // other lanes' quotients may be inf / NaN; the mask drops them.
        const LaneMask sok = mask_gt(sz, 0.0f);
        const LaneMask dok = mask_ule(__float_as_uint(qz) - 0x21800000u, 0x5d800000u - 0x21800000u);
        const float r = proj_recip(qz);
        float pu = proj_quot(nu, qz, r);
        float pv = proj_quot(nv, qz, r);
        LaneMask vz = sok & dok;
        const LaneMask slow = sok & ~dok;
        if (__builtin_expect(slow != 0, 0)) {  // wave-uniform
            const LaneMask qpos = mask_gt(qz, 0.0f);
            if (lane_in(slow)) {
                const float den = lane_in(qpos) ? qz : 1.0f;
                pu = nu / den;
                pv = nv / den;
            }
            vz |= slow & qpos;
        }
        // floor, in-range test and the pixel index without selects: the
        // coordinates stay finite on every lane (saturated integers), and an
        // unmatched lane's gather is masked after it (a raw buffer load past
        // the records returns 0, any index inside them is a real record).
        // The row test is the records' own: v' outside [0, H) is clamped to
        // H, whose index lies in the frame's zeroed pad (P >= N + 4) or past
        // the buffer (returns 0), a record with z = 0, which the match gate
        // (tz > 0) rejects as it rejects a target without a normal
        const int iu = floor_i32((pu + K.cx) + 0.5f);
        const int iv = floor_i32((pv + K.cy) + 0.5f);
        const unsigned ivc = min((unsigned)iv, (unsigned)H);
        inm = vz & mask_ult((unsigned)iu, (unsigned)W);
        fu = (float)iu;
        fv = (float)iv;
        j = (int)(__umul24(ivc, (unsigned)W) + (unsigned)iu);
    } else {
        qx = fmaf(T[2], sz, fmaf(T[1], sy, fmaf(T[0], sx, T[3])));
        qy = fmaf(T[6], sz, fmaf(T[5], sy, fmaf(T[4], sx, T[7])));
        qz = fmaf(T[10], sz, fmaf(T[9], sy, fmaf(T[8], sx, T[11])));
        const LaneMask vz = mask_gt(sz, 0.0f) & mask_gt(qz, 0.0f);
        const float rz = proj_rcp_rn(lane_in(vz) ? qz : 1.0f);
        const float uu = floorf(fmaf(K.fx * qx, rz, K.cx + 0.5f));
        const float vv = floorf(fmaf(K.fy * qy, rz, K.cy + 0.5f));
        // 0 <= u' < W and 0 <= v' < H on the integer values: uu, vv are
        // finite integral floats (T finite, youth_icp.h), v_cvt_i32_f32
        // saturates outside the int range, and a negative one wraps to
        // >= 2^31 unsigned, so the unsigned compares equal the spec's four
        // float compares
        const int iu = (int)uu, iv = (int)vv;
        inm = vz & mask_ult((unsigned)iu, (unsigned)W) & mask_ult((unsigned)iv, (unsigned)H);
        const bool in = lane_in(inm);
        fu = in ? uu : 0.0f;
        fv = in ? vv : 0.0f;
        // 0 when !in; v', W <= 16384 (youth_icp_create): the 24-bit
        // multiply-add is exact and full rate
        j = in ? (int)__umul24((unsigned)iv, (unsigned)W) + iu : 0;
    }
}

//   a7  gate: target valid with a normal (k_prep stores z = 0 for a target
//       without one, so tz > 0 is both tests) and |P' - P_t|^2 < thr^2 with
//       d2 = fma(dz, dz, fma(dy, dy, dx dx));
//   a8  r = n.(P' - P_t) = fma(n2, dz, fma(n1, dy, n0 dx));
//       J = [P' x n, n], (P' x n)_0 = fma(qy, n2, -(qz n1)) etc.;
//   a9  lane32 (A = float): acc = fma(J_a, J_b, acc) in fp32, one rounding
//       per product-add; exact (A = double): the 28 products of fp32 values
//       are exact in fp64, one rounding per add.  Unmatched lanes skip the
//       update, or add J = 0 and r = +-0, which leaves every sum unchanged
//       (an accumulator is never -0: it starts at +0 and x + -x is +0).  The target's x, y are recomputed from its z with
//       k_prep's expression (bit-identical to the stored plane).
//   kSpecSurvey: d2 = (dx dx + dy dy) + dz dz, r = (n0 dx + n1 dy) + n2 dz,
//       (P' x n)_0 = qy n2 - qz n1 etc. (no FMA).
template <int kSp, bool kFast, bool kSkip, typename A>
__device__ __forceinline__ LaneMask match_accumulate(float qx, float qy, float qz, f4v t, float fu,
                                                     float fv, LaneMask inm, const Intr& K,
                                                     const FastK& F, float thr2, A* acc)
{
    const float tz = t.x;
    const float tx = bp_div<kFast>((fu - K.cx) * tz, K.fx, F.hfx, F.lfx);
    const float ty = bp_div<kFast>((fv - K.cy) * tz, K.fy, F.hfy, F.lfy);
    const float dx = qx - tx, dy = qy - ty, dz = qz - tz;
    const float d2 = sp_survey(kSp) ? (dx * dx + dy * dy) + dz * dz
                                        : fmaf(dz, dz, fmaf(dy, dy, dx * dx));
    const LaneMask okm = inm & mask_gt(tz, 0.0f) & mask_lt(d2, thr2);
    // kSkip (the throughput kernels): unmatched lanes leave the sums
    // unchanged by not running the update (exec-masked; a wave without a
    // match skips it), k_icp 2 % faster than masking the normal.  Else
    // (k_icp_coop, latency-bound: the branches cost it 5 %,
    // profiles/r03/ab_exec_mask.txt) the normal is masked to 0, so J = 0 and
    // r = +-0 add +0 exactly: the same sums either way
    const bool ok = lane_in(okm);
    if (!kSkip || ok) {
        const float n0 = kSkip || ok ? t.y : 0.0f;
        const float n1 = kSkip || ok ? t.z : 0.0f;
        const float n2 = kSkip || ok ? t.w : 0.0f;
        float r, Jf[6];
        if (sp_survey(kSp)) {
            r = (n0 * dx + n1 * dy) + n2 * dz;
            Jf[0] = qy * n2 - qz * n1;
            Jf[1] = qz * n0 - qx * n2;
            Jf[2] = qx * n1 - qy * n0;
        } else {
            r = fmaf(n2, dz, fmaf(n1, dy, n0 * dx));
            Jf[0] = fmaf(qy, n2, -(qz * n1));
            Jf[1] = fmaf(qz, n0, -(qx * n2));
            Jf[2] = fmaf(qx, n1, -(qy * n0));
        }
        Jf[3] = n0;
        Jf[4] = n1;
        Jf[5] = n2;
        int k = 0;
        if constexpr (sizeof(A) == sizeof(float)) {
#pragma unroll
            for (int a = 0; a < 6; ++a)
#pragma unroll
                for (int bb = a; bb < 6; ++bb) {
                    acc[k] = fmaf(Jf[a], Jf[bb], acc[k]);
                    ++k;
                }
#pragma unroll
            for (int a = 0; a < 6; ++a) acc[21 + a] = fmaf(Jf[a], r, acc[21 + a]);
            acc[27] = fmaf(r, r, acc[27]);
        } else {
#pragma unroll
            for (int a = 0; a < 6; ++a)
#pragma unroll
                for (int bb = a; bb < 6; ++bb) {
                    acc[k] = fma((double)Jf[a], (double)Jf[bb], acc[k]);
                    ++k;
                }
#pragma unroll
            for (int a = 0; a < 6; ++a) acc[21 + a] = fma((double)Jf[a], (double)r, acc[21 + a]);
            acc[27] = fma((double)r, (double)r, acc[27]);
        }
    }
    return okm;
}

// Accumulate source pixels [start, end) of one pair into acc (spec a7-a9).
template <int kSp, bool kAssoc, bool kFast, bool kAligned>
__device__ __forceinline__ void accumulate_chunk(const int16_t* __restrict__ sD,
                                                 const float4* __restrict__ rec, int rec_bytes,
                                                 const float* __restrict__ T, int start, int end,
                                                 int W, int H, const Intr& K, const FastK& F,
                                                 float thr2, double* acc,
                                                 int32_t* __restrict__ arow)
{
    // the pair's target records through a buffer descriptor (wave-uniform
    // base): a gather costs one 32-bit byte offset instead of 64-bit address
    // arithmetic
    const __amdgpu_buffer_rsrc_t rrec = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float4*>(rec), (short)0, rec_bytes, 0x00020000);
    // (u0, v0) of pixel i advance incrementally (no integer division per
    // step); with kAligned (W % 4 == 0, i % 4 == 0) a lane's four pixels
    // share one row.  The match conditions are lane masks (xform_project,
    // match_accumulate), so the four gathers issue back to back; an
    // unmatched pixel's gather is dropped by its mask.
    const int stepV = kRedStep / W;
    const int stepU = kRedStep - stepV * W;
    int i = start + threadIdx.x * 4;
    int v0 = i / W;
    int u0 = i - v0 * W;
    int cnt = 0;
    // lane32: this lane's fp32 sums over its whole share of the chunk,
    // converted to fp64 once at the end (acc enters zeroed)
    float facc[28];
#pragma unroll
    for (int q = 0; q < 28; ++q) facc[q] = 0.0f;
    // kAligned: the next step's depth is loaded while this step's gathers
    // and sums run (8 bytes per lane in flight), through a buffer descriptor
    // over the frame, so the load past the last step returns 0 instead of
    // faulting; its value is then never used
    const __amdgpu_buffer_rsrc_t rdep = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<int16_t*>(sD), (short)0, W * H * (int)sizeof(int16_t), 0x00020000);
    short4 dnext = kAligned && i < end ? __builtin_bit_cast(short4, __builtin_amdgcn_raw_buffer_load_b64(
                                                                       rdep, i * 2, 0, 0))
                                       : short4{};
    for (; i < end; i += kRedStep) {
        const short4 d4 = kAligned ? dnext : load_depth4<kAligned>(sD, i, end);
        const int dd[4] = {d4.x, d4.y, d4.z, d4.w};
        float qx[4], qy[4], qz[4], fu[4], fv[4];
        LaneMask in[4];
        int j[4];
        // a lane's four pixels share one row when kAligned: centred
        // coordinates by exact additions (uc0 + q == (float)(u0 + q) - cx,
        // which the host checked for these intrinsics: centred_exact)
        const float uc0 = (float)u0 - K.cx, vc0 = (float)v0 - K.cy;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float sx, sy, sz;
            if (kAligned) {
                backproject_c<kFast>(dd[q], uc0 + (float)q, vc0, K, F, sx, sy, sz);
            } else {
                int u = u0 + q, v = v0;
                const bool wrap = u >= W;
                u = wrap ? u - W : u;
                v = wrap ? v + 1 : v;
                backproject<kFast>((i + q) < end ? dd[q] : 0, u, v, K, F, sx, sy, sz);
            }
            xform_project<kSp>(T, sx, sy, sz, K, W, H, qx[q], qy[q], qz[q], fu[q], fv[q], in[q],
                               j[q]);
        }
        u0 += stepU;
        v0 += stepV;
        if (u0 >= W) {
            u0 -= W;
            ++v0;
        }
        // four 16-byte fetches back to back, then the next step's depth
        f4v t[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
            t[q] = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rrec, (int)((unsigned)j[q] * 16u),
                                                                                 0, 0));
        // (issued after the gathers: loads retire in order, so the match
        // waits for gather q, vmcnt(4 - q), never wait for the depth)
        asm volatile("" ::: "memory");
        if (kAligned)
            dnext = __builtin_bit_cast(
                short4, __builtin_amdgcn_raw_buffer_load_b64(rdep, (i + kRedStep) * 2, 0, 0));
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            LaneMask okm;
            if constexpr (sp_lane32(kSp))
                okm = match_accumulate<kSp, kFast, false>(qx[q], qy[q], qz[q], t[q], fu[q], fv[q],
                                                          in[q], K, F, thr2, facc);
            else
                okm = match_accumulate<kSp, kFast, true>(qx[q], qy[q], qz[q], t[q], fu[q], fv[q],
                                                         in[q], K, F, thr2, acc);
            if (kAssoc && (i + q) < end) arow[i + q] = lane_in(okm) ? j[q] : -1;
            // matches counted per wave on the scalar unit (s_bcnt1 of the
            // match mask) instead of a per-lane select and add
            cnt += __builtin_popcountll(okm);

        }
    }
    if constexpr (sp_lane32(kSp)) {
#pragma unroll
        for (int q = 0; q < 28; ++q) acc[q] = (double)facc[q];
    }
    // the wave's count, carried by lane 0 into the wave / workgroup sums
    acc[28] += (threadIdx.x & 63) == 0 ? (double)cnt : 0.0;
}

// Wave sum of the kNeq per-lane accumulators by recursive halving: at lane
// mask m = 32, 16, 8, 4, 2 each lane keeps one half of its remaining values
// (the upper half iff lane & m) and sends the other half to lane ^ m, so the
// fp64 exchanges number 16 + 8 + 4 + 2 + 1 + 1 = 32 instead of 29 x 6 for a
// symmetric butterfly.  On exit lane 2q and 2q+1 both hold the wave total of
// value q (q < kNeq); the summation tree is fixed, so results are
// deterministic.  Shared by k_reduce, k_icp and k_icp_coop.
//   m = 32, 16: v_permlane32_swap / v_permlane16_swap exchange the upper
//     half-wave (odd rows) of one register with the lower half (even rows) of
//     another.  With vdst = v[q] and src = v[q+h], each lane is left holding
//     the value it keeps in one register and its partner's send in the other,
//     so v[q] = D + S with no select (keep + recv, commutative: bitwise the
//     same as the shuffle form).
//   m = 8, 2, 1: DPP (row_ror:8, quad_perm) moves; m = 4: ds_swizzle xor.
// No LDS bpermute; the partners (lane ^ m) and the add order are unchanged,
// so the sums are bit-identical to the shuffle form.
template <int kM>
__device__ __forceinline__ double xchg_small(double x)
{
    int lo = (int)lo32(x), hi = (int)hi32(x);
    if (kM == 8) {
        lo = __builtin_amdgcn_update_dpp(0, lo, 0x128, 0xf, 0xf, false);  // row_ror:8
        hi = __builtin_amdgcn_update_dpp(0, hi, 0x128, 0xf, 0xf, false);
    } else if (kM == 4) {
        lo = __builtin_amdgcn_ds_swizzle(lo, 0x1F | (4 << 10));  // bit mode, xor 4
        hi = __builtin_amdgcn_ds_swizzle(hi, 0x1F | (4 << 10));
    } else if (kM == 2) {
        lo = __builtin_amdgcn_update_dpp(0, lo, 0x4E, 0xf, 0xf, false);  // quad_perm [2,3,0,1]
        hi = __builtin_amdgcn_update_dpp(0, hi, 0x4E, 0xf, 0xf, false);
    } else {
        lo = __builtin_amdgcn_update_dpp(0, lo, 0xB1, 0xf, 0xf, false);  // quad_perm [1,0,3,2]
        hi = __builtin_amdgcn_update_dpp(0, hi, 0xB1, 0xf, 0xf, false);
    }
    return join64((unsigned)lo, (unsigned)hi);
}

template <int kM>
__device__ __forceinline__ void rs_stage_small(double* v, int lane)
{
    constexpr int h = kM / 2;
    const bool up = (lane & kM) != 0;
#pragma unroll
    for (int q = 0; q < h; ++q) {
        const double send = up ? v[q] : v[q + h];
        const double keep = up ? v[q + h] : v[q];
        v[q] = keep + xchg_small<kM>(send);
    }
}

__device__ __forceinline__ void wave_reduce_scatter(const double* acc, int lane, double& total)
{
    double v[32];
#pragma unroll
    for (int q = 0; q < 32; ++q) v[q] = q < kNeq ? acc[q] : 0.0;
#pragma unroll
    for (int q = 0; q < 16; ++q) {  // m = 32
        const auto l = __builtin_amdgcn_permlane32_swap(lo32(v[q]), lo32(v[q + 16]), false, false);
        const auto h = __builtin_amdgcn_permlane32_swap(hi32(v[q]), hi32(v[q + 16]), false, false);
        v[q] = join64(l[0], h[0]) + join64(l[1], h[1]);
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {  // m = 16
        const auto l = __builtin_amdgcn_permlane16_swap(lo32(v[q]), lo32(v[q + 8]), false, false);
        const auto h = __builtin_amdgcn_permlane16_swap(hi32(v[q]), hi32(v[q + 8]), false, false);
        v[q] = join64(l[0], h[0]) + join64(l[1], h[1]);
    }
    rs_stage_small<8>(v, lane);
    rs_stage_small<4>(v, lane);
    rs_stage_small<2>(v, lane);
    total = v[0] + xchg_small<1>(v[0]);
}

template <int kSp, bool kAssoc, bool kFast, bool kAligned, bool kFuse>
__global__ __launch_bounds__(kRedThreads) void k_reduce(
    const int16_t* __restrict__ dsrc, const float4* __restrict__ recs, size_t P, PairMap pm,
    int W, int H, Intr K, FastK F, float thr2, int chunk, double* __restrict__ partials,
    int32_t* __restrict__ assoc, PoseState ps)
{
    __shared__ double red[kRedThreads / 64][kNeq];
    const int p = blockIdx.y;
    const int b = blockIdx.x;
    const int N = W * H;
    const int16_t* sD = dsrc + (size_t)(pm.src0 + p) * N;
    const float4* rec = recs + (size_t)(pm.tgt0 + p) * P;
    float T[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) T[k] = ps.T32[p * 12 + k];

    double acc[kNeq];
#pragma unroll
    for (int k = 0; k < kNeq; ++k) acc[k] = 0.0;

    const int start = b * chunk;
    const int end = min(start + chunk, N);
    int32_t* arow = kAssoc ? assoc + (size_t)p * N : nullptr;
    accumulate_chunk<kSp, kAssoc, kFast, kAligned>(sD, rec, (int)(P * sizeof(float4)), T, start, end,
                                              W, H, K, F, thr2, acc, arow);
    // wave reduce-scatter, then the four waves in fixed order through LDS
    const int wave = threadIdx.x >> 6;
    {
        const int ln = threadIdx.x & 63;
        double tot;
        wave_reduce_scatter(acc, ln, tot);
        if (!(ln & 1) && (ln >> 1) < kNeq) red[wave][ln >> 1] = tot;
    }
    __syncthreads();
    if (threadIdx.x >= 64) return;  // wave 0 publishes (and, if last, solves)
    const int lane = threadIdx.x;
    const int nblk = gridDim.x;
    double* mine = partials + ((size_t)p * nblk + b) * kNeq;
    double s = 0.0;
    if (lane < kNeq) {
#pragma unroll
        for (int w = 0; w < kRedThreads / 64; ++w) s += red[w][lane];
    }
    if (!kFuse) {
        if (lane < kNeq) mine[lane] = s;
        return;
    }
    // In-launch hand-off (cdna_hip_programming.md G16, MI355X_MICROARCH.md
    // "Valid forms" row 1): write-through (sc1) partial stores, the storing
    // wave drains them, then ONE agent-scope atomic per workgroup; the
    // workgroup whose add returns nblk-1 is last and reads every partial of
    // pair p with sc1 loads only.
    if (lane < kNeq)
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(mine) + lane,
                           (unsigned long long)__double_as_longlong(s), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned ticket = 0;
    if (lane == 0)
        ticket = __hip_atomic_fetch_add(ps.arrivals + p, 1u, __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);
    ticket = __shfl(ticket, 0, 64);
    if (ticket != (unsigned)nblk - 1) return;
    // No acquire fence: every load of the handed-off partials below is an
    // sc1 load and every store of them was an sc1 store drained before the
    // add (G16: the fence may then be dropped).  Fixed-order sum of pair p's
    // partials (same order as k_solve), loads issued in batches of 8.
    const unsigned long long* base =
        reinterpret_cast<const unsigned long long*>(partials + (size_t)p * nblk * kNeq);
    const int half = (nblk + 1) >> 1;
    const int k = lane & 31;
    double t = 0.0;
    if (k < kNeq) {
        const int b0 = lane < 32 ? 0 : half;
        const int b1 = lane < 32 ? half : nblk;
        for (int bb = b0; bb < b1; bb += 8) {
            double v[8];
#pragma unroll
            for (int q = 0; q < 8; ++q)
                v[q] = bb + q < b1 ? __longlong_as_double((long long)__hip_atomic_load(
                                         base + (size_t)(bb + q) * kNeq + k, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT))
                                   : 0.0;
#pragma unroll
            for (int q = 0; q < 8; ++q) t += v[q];
        }
    }
    t += __shfl_down(t, 32, 64);
    double neq[kNeq];
#pragma unroll
    for (int q = 0; q < kNeq; ++q) neq[q] = __shfl(t, q, 64);
    if (lane == 0) {
        ps.arrivals[p] = 0;  // re-armed for the next launch (stream order)
        if (ps.stats) {
            ps.stats[((size_t)p * ps.iters + ps.it) * 2 + 0] = neq[28];
            ps.stats[((size_t)p * ps.iters + ps.it) * 2 + 1] = neq[27];
        }
        solve_update(neq, ps.T64 + (size_t)p * 16, ps.T32 + (size_t)p * 12, ps.status + p);
    }
}

// Fixed-order sum of a pair's nblk partial rows (kPartStride doubles each,
// written with sc1 stores by other workgroups, read with sc1 loads only).
// Called by every thread of the workgroup.  Thread (column j, piece q) with
// j < kSumCols loads rows j, j + 16, ... in batches of kBatch 16-byte pieces
// and adds each batch as a pairwise tree, batches in order; then wave 0
// lane l < kNeq adds the 16 column sums of value l as a pairwise tree.  The
// tree keeps the dependent fp64 adds per value at ~8 + batches instead of the
// 16 + rows of a running sum (the solve waits on it every iteration).  Returns
// the pair total of value `lane` in wave 0's lanes < kNeq (0 elsewhere).
template <int kN>
__device__ __forceinline__ double tree_sum(const double* v)
{
    if constexpr (kN == 1) {
        return v[0];
    } else {
        return tree_sum<kN / 2>(v) + tree_sum<kN / 2>(v + kN / 2);
    }
}

template <int kBatch>
__device__ __forceinline__ double sum_pair_rows(__amdgpu_buffer_rsrc_t rpart, int nblk,
                                                double (*colsum)[kPartStride])
{
    const int t = threadIdx.x;
    const int j = t / kPieces, q = t - j * kPieces;
    if (j < kSumCols) {
        double s0 = 0.0, s1 = 0.0;
        for (int bb = j; bb < nblk; bb += kBatch * kSumCols) {
            u4v v[kBatch];
#pragma unroll
            for (int i = 0; i < kBatch; ++i) {
                const int b = bb + i * kSumCols;
                // aux 16 = sc1 (bypass this CU's L1: written by other CUs)
                v[i] = b < nblk ? __builtin_bit_cast(
                                      u4v, __builtin_amdgcn_raw_buffer_load_b128(
                                               rpart, (b * kPartStride + 2 * q) * 8, 0, 16))
                                : u4v{0u, 0u, 0u, 0u};
            }
            double a0[kBatch], a1[kBatch];
#pragma unroll
            for (int i = 0; i < kBatch; ++i) {
                a0[i] = __hiloint2double((int)v[i].y, (int)v[i].x);
                a1[i] = __hiloint2double((int)v[i].w, (int)v[i].z);
            }
            s0 += tree_sum<kBatch>(a0);
            s1 += tree_sum<kBatch>(a1);
        }
        colsum[j][2 * q] = s0;
        colsum[j][2 * q + 1] = s1;
    }
    __syncthreads();
    double tsum = 0.0;
    if (t < kNeq) {
        double c[kSumCols];
#pragma unroll
        for (int jj = 0; jj < kSumCols; ++jj) c[jj] = colsum[jj][t];
        tsum = tree_sum<kSumCols>(c);
    }
    return tsum;
}

// ------------------------------------------------------------------- k_icp --
// ONE persistent launch for all `iters` iterations of a batch.
//
// Work item = (iteration k, pair p, chunk c), ordered iteration-major:
//   item = (k * n_pairs + p) * nblk + c.
// Workgroups take items from one dynamic dequeue counter.  An item of
// iteration k >= 1 waits until epoch[p] >= k, i.e. until iteration k-1 of
// pair p has been solved.  Every item it can wait on has a SMALLER index, so
// it was dequeued earlier by a running workgroup, and the earliest
// unfinished item never waits: the scheme cannot deadlock, whatever the
// residency (no co-residency assumption; cdna_hip_programming.md §1).  Every
// spin is bounded; a timeout sets *error and the workgroup exits, and the
// host reports it as YOUTH_STATUS_TIMEOUT (the GPU never hangs).
//
// Hand-offs (G16 / MI355X_MICROARCH "Valid forms" row 1): partials, T64 and
// T32 are written with sc1 stores, the storing wave drains (vmcnt(0)), then
// ONE agent-scope atomic (arrival ticket) or flag store (epoch); every read
// of handed-off bytes is an sc1 load by the wave that saw the ticket/flag.
struct IterState {
    double* T64;          // [pair][16]
    float* T32;           // [pair][12]
    int32_t* status;      // [pair]
    double* stats;        // [pair][iters][2] or null
    unsigned* arrivals;   // [pair][iters], zeroed per call
    unsigned* epoch;      // [pair], zeroed per call
    unsigned* head;       // queue words (telemetry at kQSpins / kQWaited), zeroed per call
    unsigned* error;      // timeout flag, zeroed per call
    float* T_out;         // [pair][16] fp32 4x4 written by the final solve, or null
    int iters, n_pairs, nblk, chunk;
    int nq;               // work queues (1..kMaxQueues): heads at head[kQHeads + 32 q]
};

// One dequeue: from the workgroup's current queue q, moving on to the next
// queue when q is drained (each queue holds the pairs p = q (mod nq), items
// (iteration, pair, chunk) in that order).  Returns the item in the global
// numbering item = (k n_pairs + p) nblk + c, or `total` when every queue is
// drained.  Dependencies stay inside a queue (an item waits only on earlier
// items of its own pairs, dequeued before it by running workgroups), so
// every queue is deadlock-free on its own, as the single queue was; nq > 1
// spreads the contended returning atomics over nq words (one per 128-B line):
// MI355X_MICROARCH.md "dequeue": one head word pulled by 256+ CUs costs
// ~3 us per dequeue, 8 per-XCD heads ~1.2 us.
// Split in two so the first take's round trip can overlap other memory
// traffic: icp_dequeue_issue takes a ticket from queue q's head (the atomic),
// icp_dequeue_from decodes it, moving on to the next queues (synchronously)
// while q is drained.
__device__ __forceinline__ unsigned icp_dequeue_issue(const IterState& is, int q)
{
    return __hip_atomic_fetch_add(is.head + (kQHeads - kQHead) + q * kQHeadStride, 1u,
                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int icp_dequeue_from(const IterState& is, int& q, unsigned first,
                                                int total)
{
    unsigned t = first;
    for (int v = 0; v < is.nq; ++v) {
        const int npq = (is.n_pairs - q + is.nq - 1) / is.nq;
        if (v > 0 && npq > 0) t = icp_dequeue_issue(is, q);
        if (npq > 0) {
            const int per = npq * is.nblk;
            const int i = (int)t;
            if (i < is.iters * per) {
                const int k = i / per;
                const int rem = i - k * per;
                const int pl = rem / is.nblk;
                const int c = rem - pl * is.nblk;
                return (k * is.n_pairs + q + is.nq * pl) * is.nblk + c;
            }
        }
        q = q + 1 == is.nq ? 0 : q + 1;
    }
    return total;
}
__device__ __forceinline__ int icp_dequeue(const IterState& is, int& q, int total)
{
    return icp_dequeue_from(is, q, icp_dequeue_issue(is, q), total);
}

constexpr unsigned kSpinMax = 1u << 23;  // x s_sleep(8) ~ seconds: a bound, never reached

__device__ __forceinline__ unsigned ld_u32_sc1(const unsigned* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_u64_sc1(const void* p)
{
    return __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_u64_sc1(void* p, unsigned long long v)
{
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), v, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_u32_sc1(void* p, unsigned v)
{
    __hip_atomic_store(reinterpret_cast<unsigned*>(p), v, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// Queue side of a work item, run by thread 0 after its workgroup published
// its previous partial (so a waiting workgroup never holds work another one
// waits for): wait (bounded) until pair p's pose epoch reaches k, then copy
// the pose into LDS.  Returns the item, or `total` when the queue is drained
// or after a timeout (error flag set).
__device__ __forceinline__ int icp_claim(const IterState& is, int item, int total, int per_iter,
                                         float* sh_T)
{
    if (item >= total) return total;
    const int k = item / per_iter;
    const int p = (item - k * per_iter) / is.nblk;
    if (k > 0) {
        unsigned spins = 0;
        while (ld_u32_sc1(is.epoch + p) < (unsigned)k) {
            __builtin_amdgcn_s_sleep(8);
            if (++spins > kSpinMax || ld_u32_sc1(is.error) != 0u) {
                __hip_atomic_fetch_or(is.error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return total;
            }
        }
        if (spins) {  // scheduler telemetry (youth_icp_get_sched_stats)
            __hip_atomic_fetch_add(is.head + (kQSpins - kQHead), spins, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(is.head + (kQWaited - kQHead), 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    // the pose of (p, k): sc1 loads after the epoch matched
    unsigned long long v[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) v[q] = ld_u64_sc1(is.T32 + p * 12 + 2 * q);
#pragma unroll
    for (int q = 0; q < 6; ++q) {
        sh_T[2 * q] = __uint_as_float((unsigned)v[q]);
        sh_T[2 * q + 1] = __uint_as_float((unsigned)(v[q] >> 32));
    }
    return item;
}

// Persistent ICP: ONE launch runs every iteration of every pair.  Work items
// (k, p, c) = (iteration, pair, pixel chunk) are dequeued in that order from
// one agent-scope counter; item (k, p, c) needs pair p's pose after k
// updates, published by the LAST workgroup to finish a chunk of (p, k-1)
// (arrival ticket), which sums the pair's partials in fixed order, solves and
// bumps epoch[p].  Per item: pixel loop -> wave reduce-scatter -> barrier ->
// wave 0 publishes the partial, takes the ticket (and, if last, solves) ->
// thread 0 dequeues and claims the next item -> barrier.
// (Dequeuing ahead from wave 1 so that waves 1-3 skip the second barrier
// measured no faster: DESIGN.md §5.)
template <int kSp, bool kFast, bool kAligned>
__global__ __launch_bounds__(kRedThreads, 4) void k_icp(const int16_t* __restrict__ dsrc,
                                                    const float4* __restrict__ recs, size_t P,
                                                    PairMap pm, int W, int H, Intr K, FastK F,
                                                    float thr2, double* __restrict__ partials,
                                                    IterState is)
{
    __shared__ double red[kRedThreads / 64][kNeq];
    __shared__ double colsum[kSumCols][kPartStride];
    __shared__ double sh_neq[kNeq];
    __shared__ double sh_T64[12];
    __shared__ float sh_T32n[12];
    __shared__ int sh_item;
    __shared__ int sh_next;
    __shared__ int sh_last;
    __shared__ float sh_T[12];
    const int N = W * H;
    const int per_iter = is.n_pairs * is.nblk;
    const int total = is.iters * per_iter;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;

    // thread 0's current queue: workgroups are dealt to the queues
    // round-robin (b and b + 8 share an XCD, so with 8 queues each XCD pulls
    // from its own head)
    // (thread 1 keeps it: it dequeues the next item while wave 0 publishes)
    int myq = (int)(blockIdx.x % (unsigned)is.nq);
    if (threadIdx.x == 1) sh_next = icp_dequeue(is, myq, total);
    __syncthreads();
    if (threadIdx.x == 0) sh_item = icp_claim(is, sh_next, total, per_iter, sh_T);
    __syncthreads();
    for (;;) {
        // LDS-broadcast values are wave-uniform: readfirstlane keeps them
        // (and everything derived from them) in SGPRs
        const int item = __builtin_amdgcn_readfirstlane(sh_item);
        if (item >= total) return;
        const int k = item / per_iter;
        const int rem = item - k * per_iter;
        const int p = rem / is.nblk;
        const int c = rem - p * is.nblk;
        float T[12];
#pragma unroll
        for (int q = 0; q < 12; ++q)
            T[q] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(sh_T[q])));

        double acc[kNeq];
#pragma unroll
        for (int q = 0; q < kNeq; ++q) acc[q] = 0.0;
        const int start = c * is.chunk;
        const int end = min(start + is.chunk, N);
        accumulate_chunk<kSp, false, kFast, kAligned>(dsrc + (size_t)(pm.src0 + p) * N,
                                                 recs + (size_t)(pm.tgt0 + p) * P,
                                                 (int)(P * sizeof(float4)), T, start, end, W, H,
                                                 K, F, thr2, acc, nullptr);
        {
            double tot;
            wave_reduce_scatter(acc, lane, tot);
            if (!(lane & 1) && (lane >> 1) < kNeq) red[wave][lane >> 1] = tot;
        }
        __syncthreads();

        if (wave == 0) {
            // ---- publish this chunk's partial, take the arrival ticket; lane
            // 1 takes the next item from the queue meanwhile (its round trip
            // overlaps the stores' drain; the item is claimed, i.e. waited
            // on, only after this workgroup has published: the queue stays
            // deadlock-free)
            unsigned first = 0u;
            if (lane == 1) first = icp_dequeue_issue(is, myq);
            double sum = 0.0;
            if (lane < kPartStride) {
                if (lane < kNeq) {  // the waves' sums as a pairwise tree (2 dependent adds)
                    double r[kRedThreads / 64];
#pragma unroll
                    for (int w = 0; w < kRedThreads / 64; ++w) r[w] = red[w][lane];
                    sum = tree_sum<kRedThreads / 64>(r);
                }
                st_u64_sc1(partials + ((size_t)p * is.nblk + c) * kPartStride + lane,
                           (unsigned long long)__double_as_longlong(sum));
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane == 0) {
                const unsigned ticket = __hip_atomic_fetch_add(
                    is.arrivals + (size_t)p * is.iters + k, 1u, __ATOMIC_RELAXED,
                    __HIP_MEMORY_SCOPE_AGENT);
                sh_last = ticket == (unsigned)is.nblk - 1;
            }
            if (lane == 1) sh_next = icp_dequeue_from(is, myq, first, total);
        }
        __syncthreads();
        if (__builtin_amdgcn_readfirstlane(sh_last)) {
            // ---- last arriver of (p, k): every wave sums a share of the
            // pair's partials (sum_pair_rows: sc1 16-byte loads, one batch
            // for <= 256 chunks, fixed tree order); wave 0 solves, publishes
            // the pose, then the epoch.
            const __amdgpu_buffer_rsrc_t rpart = __builtin_amdgcn_make_buffer_rsrc(
                partials + (size_t)p * is.nblk * kPartStride, (short)0,
                is.nblk * kPartStride * (int)sizeof(double), 0x00020000);
            if (threadIdx.x >= 64 && threadIdx.x < 64 + 12)
                sh_T64[threadIdx.x - 64] = __longlong_as_double(
                    (long long)ld_u64_sc1(is.T64 + (size_t)p * 16 + (threadIdx.x - 64)));
            const double tsum = sum_pair_rows<8>(rpart, is.nblk, colsum);
            if (wave == 0) {
                if (lane < kNeq) sh_neq[lane] = tsum;
                // the fp32 pose published when the solve skips the update (status != 0)
                if (lane < 12) sh_T32n[lane] = (float)sh_T64[lane];
                if (is.stats && lane == 0) {
                    is.stats[((size_t)p * is.iters + k) * 2 + 0] = readlane64(tsum, 28);
                    is.stats[((size_t)p * is.iters + k) * 2 + 1] = readlane64(tsum, 27);
                }
                const int st = solve_update_wave_call(sh_neq, sh_T64, sh_T32n, lane);
                if (st && lane == 0)
                    __hip_atomic_fetch_or(is.status + p, st, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
                // publish: lanes < 12 store the pose (sc1), the wave drains, then the epoch
                if (lane < 12) {
                    st_u64_sc1(is.T64 + (size_t)p * 16 + lane,
                               (unsigned long long)__double_as_longlong(sh_T64[lane]));
                    st_u32_sc1(is.T32 + (size_t)p * 12 + lane, __float_as_uint(sh_T32n[lane]));
                }
                // the pair's final pose as the fp32 4x4 output (k_finish folded in)
                if (k == is.iters - 1 && is.T_out && lane < 16)
                    is.T_out[(size_t)p * 16 + lane] =
                        lane < 12 ? sh_T32n[lane] : (lane == 15 ? 1.0f : 0.0f);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (lane == 0) st_u32_sc1(is.epoch + p, (unsigned)(k + 1));
            }
        }
        // ---- next item (this workgroup has published: waiting is safe)
        if (threadIdx.x == 0) sh_item = icp_claim(is, sh_next, total, per_iter, sh_T);
        __syncthreads();
    }
}

// -------------------------------------------------------------- k_icp_coop --
// Small batches: C2's single pair and the SLAM tracker's frame-to-frame align
// (youth_icp_track_frame).  One pair cannot fill the chip, so k_icp's cost
// there is the chain of memory round trips per iteration (dequeue, pose poll,
// pose load, cold depth and record loads, ticket, last-arriver solve, pose
// publish: ~17 us).  This kernel shortens that chain:
//   * ONE cooperative launch of n_pairs x G co-resident workgroups replaces
//     k_init + k_icp + k_finish; workgroup b owns chunk c = b % G of pair
//     p = b / G for every iteration (no queue);
//   * its source pixels (npx per lane) are loaded and back-projected ONCE
//     into LDS; its record gathers hit the same lines every iteration
//     (L1/L2-warm);
//   * per iteration ONE hand-off, and no counter in it: each workgroup
//     stores its partial row (sc1, 8-byte stores) over a row that holds the
//     EMPTY pattern, and every workgroup loads ALL the pair's rows, loading
//     again every 16-byte piece that still holds EMPTY, then sums them in the
//     fixed column order of k_icp's last arriver and solves itself.
//     Identical inputs and code give every workgroup the identical fp64
//     pose, so no pose is handed off.  The wait is the data itself: one
//     memory round trip after the last row lands, where an arrival counter
//     costs three (store drain + atomic, counter poll, row loads; round 5:
//     publish + arrive 1.04, poll 0.80, row loads 1.16 us per iteration).
// EMPTY is a signalling NaN (high word kPartEmptyHi): fp64 arithmetic never
// yields one (NaN results are quiet), so a row value can never look empty;
// each value is one 8-byte store and is checked on its own, so no ordering
// between a row's values is needed.  Rows are triple-buffered by iteration
// (k % 3): once a workgroup has seen every row of iteration k, every
// workgroup of the pair has read iteration k-1's rows (it read them before it
// stored k), so it resets its OWN row of buffer (k+2) % 3 = (k-1) % 3 to
// EMPTY, drains, and only then stores iteration k+1: whoever loads
// iteration k+2's rows has seen that k+1 row first, so it sees EMPTY or the
// k+2 value, never the k-1 one.  Across calls the rows alternate between two
// arenas with the counter sets: a call resets the rows the previous call
// used in the other arena (stream order: the arena a call uses is never the
// one it resets).  Co-residency is NOT guaranteed: by default the grid is a
// plain launch sized to an idle device's capacity (coop_enqueue orders this
// process's cooperative launches per device; hipLaunchCooperativeKernel is
// opt-in, YOUTH_ICP_COOP_LAUNCH=runtime), so another process holding CUs
// can leave workgroups unscheduled.  Every spin is therefore bounded
// (timeout -> YOUTH_STATUS_TIMEOUT, no hang), every workgroup preps its
// tiles before it first waits (a timed-out launch still leaves complete
// records), and the tracker realigns a timed-out frame
// (youth_icp_track_realign: the same plan again, then the persistent k_icp).
constexpr int kCoopShardStride = 32;  // words: one 128-B line per counter
constexpr int kCoopMaxPx = 32;       // source pixels per lane (LDS: 3 x 32 KB)
constexpr int kCoopMaxPairs = 16;
constexpr int kCoopBufs = 3;         // partial-row buffers per arena (iteration k % 3)
constexpr unsigned kPartEmptyHi = 0x7FF7A5A5u;  // EMPTY = 0x7FF7A5A5'7FF7A5A5 (a signalling NaN)
constexpr unsigned long long kPartEmpty = 0x7FF7A5A57FF7A5A5ull;
// counter set layout (words): timeout word (one line) | [pair][shard][32]
// prep-done counters: workgroup c of a pair arrives on shard c % 8 (one
// 128-B line each), so no line takes more than ~G/8 of the pair's arrivals
// (MI355X_MICROARCH.md "fanin": 255 arrivals on one word take 3.2 us)
constexpr int kCoopPrepShards = 8;
constexpr int kCoopErrWord = 0;
constexpr int kCoopPrepWords = kCoopErrWord + kCoopShardStride;
constexpr int kCoopPrepPair = kCoopPrepShards * kCoopShardStride;  // words per pair
constexpr int kCoopSetWords = kCoopPrepWords + kCoopMaxPairs * kCoopPrepPair;
constexpr int kCoopTileH = 24;  // fused prep tiles: 64 x 24 pixels (one per workgroup of a 640x480 pair: 200 tiles, G = 200)
constexpr int kCoopTileHTall = 80;  // 64 x 80 (= 10 px per lane x 512: one per workgroup of a 1280x960 pair, G = 240)
// Polls before a wait gives up (~0.5-1 us each: ~35-65 ms).  A wait of a
// co-resident grid ends within microseconds; one that reaches the bound has
// a workgroup that never started (the grid is not co-resident: another
// process holds CUs), and the tracker's realign then runs after one stalled
// frame instead of a stall of seconds (round 6; 2^22 polls, ~4 s, before).
// The bound counts polls, not time: a wave that is preempted does not poll.
// (A bound chosen per iteration, short for iteration 0 only, cost C2 1.9 %:
// profiles/r06/coop_spin_bound_ab_r6j.txt.)
constexpr unsigned kCoopSpinMax = 1u << 16;
constexpr int kCoopMaxChain = YOUTH_TRACK_MAX_BATCH;  // frames per tracker micro-batch

struct CoopState {
    const double* T_init;  // [pair][16] or null (identity)
    double* T64;           // [pair][16]
    float* T32;            // [pair][12]
    int32_t* status;       // [pair]
    double* stats;         // [pair][iters][2]
    float* T_out;          // [pair][16] fp32 4x4, or null
    unsigned* set;         // this call's counters: timeout word + prep counters
    unsigned* set_next;    // the next call's: zeroed here
    unsigned* head_err;    // k_icp's queue words: error/telemetry cleared for get_poses
    int iters, n_pairs, G, npx;  // G workgroups per pair, npx source pixels per lane
    // fused target prep (null: none): pair p's workgroups turn depth frame
    // prep_src + p N into record frame prep_out0 + p; prep_wait: those are
    // the records this launch gathers (hand-off before iteration 0), else
    // they are for a later launch (the tracker's next reference frame)
    const int16_t* prep_src;
    int prep_out0, prep_wait, prep_wide;
    // pair 0's result straight into pinned host memory (the tracker): fp64
    // 4x4 pose [16], then the status word; null: none
    double* res_host;
    // 1: workgroup c's source pixels are target tile c (kTileW x kCoopTileH,
    // = npx x kThreads pixels), the tile it preps, so its iteration-0 gathers
    // (small motion) hit records it has just written; 0: a contiguous run
    int tile_src;
    // tracker micro-batch (chain = 1; youth_icp_track_submit_batch): pairs
    // (f_{p-1}, f_p) of consecutive frames.  Pair p preps its own source
    // frame f_p into record frame prep_slot[p]; its target records are record
    // frame tgt_slot[p]: pair 0 the reference, pair p >= 1 the frame pair p-1
    // preps in this launch, so pair p waits for pair p-1's prep counter.
    // Pair p's result goes to the pinned slot res_pair[p].
    int chain;
    int tgt_slot[kCoopMaxChain], prep_slot[kCoopMaxChain];
    double* res_pair[kCoopMaxChain];
    // partial rows: this call's arena [kCoopBufs][part_cap][kPartStride]
    // (row p G + c), every row EMPTY at launch; the other arena, whose first
    // part_reset rows of every buffer (the previous call's) are reset here
    double* part;
    double* part_next;
    int part_cap, part_reset;
    int poll_delay;  // x 64 clocks before the first pass over the rows
    unsigned spin_max;  // polls before a wait gives up (kCoopSpinMax; the test hook's less)
    int stall_chunk;    // test hook: this chunk of pair 0 never stores iteration stall_iter's row (-1: none)
    int stall_iter;
};

// Phase timestamps for tools/coopbench only (never in the product build):
// thread 0 of every workgroup records s_memrealtime (100 MHz) at 8 points of
// each iteration into coop_phase[block][iteration][16] (slots 8-10: solve).
#ifdef YOUTH_COOP_PHASES
__device__ unsigned long long* coop_phase;
#define COOP_MARK(k, slot)                                                           \
    do {                                                                             \
        if (threadIdx.x == 0 && coop_phase && (k) < 32)                              \
            coop_phase[((size_t)blockIdx.x * 32 + (k)) * 16 + (slot)] =              \
                __builtin_amdgcn_s_memrealtime();                                    \
    } while (0)
#define COOP_MARK_WAVE(k, slot)                                                      \
    do {                                                                             \
        if ((threadIdx.x & 63) == 0 && threadIdx.x && coop_phase && (k) < 32)       \
            coop_phase[((size_t)blockIdx.x * 32 + (k)) * 16 + (slot)] =              \
                __builtin_amdgcn_s_memrealtime();                                    \
    } while (0)
#else
#define COOP_MARK(k, slot) \
    do {                   \
    } while (0)
#define COOP_MARK_WAVE(k, slot) \
    do {                        \
    } while (0)
#endif

// sum_pair_rows for k_icp_coop's counter-free hand-off: the same loads, sums
// and order, but every 16-byte piece that still holds EMPTY (its row not
// stored yet) is loaded again until none does.  The sums are those of
// sum_pair_rows over the same rows, bit for bit.  Every spin is bounded: a
// thread that passes spin_max polls, or finds the timeout word set, sets
// it and `stop` comes back non-zero in every thread (the caller stops).
template <int kBatch>
__device__ __forceinline__ double sum_pair_rows_polled(__amdgpu_buffer_rsrc_t rpart, int nblk,
                                                       double (*colsum)[kPartStride],
                                                       unsigned* err, int* sh_stop, int delay,
                                                       unsigned spin_max, int& stop)
{
    // rows land about when this workgroup's own did: the first pass waits
    // `delay` x 64 clocks so that it finds most of them (a pass over EMPTY
    // rows is traffic every workgroup pays again)
    int d = delay;
    for (; d >= 8; d -= 8) __builtin_amdgcn_s_sleep(8);
    for (; d > 0; --d) __builtin_amdgcn_s_sleep(1);
    const int t = threadIdx.x;
    const int j = t / kPieces, q = t - j * kPieces;
    int mine = 0;
    if (j < kSumCols) {
        double s0 = 0.0, s1 = 0.0;
        for (int bb = j; bb < nblk; bb += kBatch * kSumCols) {
            u4v v[kBatch];
#pragma unroll
            for (int i = 0; i < kBatch; ++i) {
                const int b = bb + i * kSumCols;
                // aux 16 = sc1 (bypass this CU's L1: written by other CUs)
                v[i] = b < nblk ? __builtin_bit_cast(
                                      u4v, __builtin_amdgcn_raw_buffer_load_b128(
                                               rpart, (b * kPartStride + 2 * q) * 8, 0, 16))
                                : u4v{0u, 0u, 0u, 0u};
            }
            unsigned spins = 0;
            for (;;) {
                bool miss = false;
#pragma unroll
                for (int i = 0; i < kBatch; ++i) {
                    if (v[i].y == kPartEmptyHi || v[i].w == kPartEmptyHi) {  // pad rows are 0
                        miss = true;
                        // volatile (aux bit 31; emitted as sc0 sc1): the
                        // optimiser must re-issue every re-poll (a non-volatile
                        // one was once left out of a loop: DESIGN.md §9 1b)
                        v[i] = __builtin_bit_cast(
                            u4v, __builtin_amdgcn_raw_buffer_load_b128(
                                     rpart, ((bb + i * kSumCols) * kPartStride + 2 * q) * 8, 0,
                                     (int)(16u | 0x80000000u)));
                    }
                }
                if (!miss) break;
                if (++spins > spin_max || ((spins & 63u) == 0u && ld_u32_sc1(err) != 0u)) {
                    __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    mine = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            double a0[kBatch], a1[kBatch];
#pragma unroll
            for (int i = 0; i < kBatch; ++i) {
                a0[i] = __hiloint2double((int)v[i].y, (int)v[i].x);
                a1[i] = __hiloint2double((int)v[i].w, (int)v[i].z);
            }
            s0 += tree_sum<kBatch>(a0);
            s1 += tree_sum<kBatch>(a1);
        }
        colsum[j][2 * q] = s0;
        colsum[j][2 * q + 1] = s1;
    }
    // stop: sh_stop is 0 while the loop runs and is only ever set to 1 (every
    // thread then leaves the loop), so no reset is needed
    if (mine) *sh_stop = 1;
    __syncthreads();
    stop = __builtin_amdgcn_readfirstlane(*sh_stop);
    double tsum = 0.0;
    if (t < kNeq) {
        double c[kSumCols];
#pragma unroll
        for (int jj = 0; jj < kSumCols; ++jj) c[jj] = colsum[jj][t];
        tsum = tree_sum<kSumCols>(c);
    }
    return tsum;
}

// Spec a7-a9 for Q source pixels already back-projected (px = pixel slots
// s0 .. s0+Q-1 of this lane in the LDS planes X/Y/Z [slot][256]): transform,
// project, Q record gathers back to back, residual, Jacobian, exact products
// into the fp64 accumulators.  Same expressions as accumulate_chunk.
template <int kSp, bool kFast, int Q, int kThreads, typename A>
__device__ __forceinline__ void coop_group(const float* __restrict__ X, const float* __restrict__ Y,
                                           const float* __restrict__ Z, int s0, const float* T,
                                           __amdgpu_buffer_rsrc_t rrec, int W, int H,
                                           const Intr& K, const FastK& F, float thr2,
                                           A* acc, int& nmatch)
{
    const int t = threadIdx.x;
    float qx[Q], qy[Q], qz[Q], fu[Q], fv[Q];
    LaneMask in[Q];
    int j[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const float sx = X[(s0 + q) * kThreads + t];
        const float sy = Y[(s0 + q) * kThreads + t];
        const float sz = Z[(s0 + q) * kThreads + t];
        xform_project<kSp>(T, sx, sy, sz, K, W, H, qx[q], qy[q], qz[q], fu[q], fv[q], in[q], j[q]);
    }
    f4v rec[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q)
        // aux 16 = sc1: the records come from this launch's fused prep (sc1
        // stores, drained, sharded counter) and are read ONLY by sc1 loads, so
        // no agent acquire is needed after the prep wait (MI355X_MICROARCH.md
        // "Valid forms", table row 1; L1 hits were worth less than the
        // acquire: C2 15.9 -> 16.4 K, profiles/r05/c2ab_r5zc_sc1_gathers.txt)
        rec[q] = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rrec, (int)((unsigned)j[q] * 16u), 0, 16));
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        nmatch += __builtin_popcountll(match_accumulate<kSp, kFast, false>(
            qx[q], qy[q], qz[q], rec[q], fu[q], fv[q], in[q], K, F, thr2, acc));  // per wave
    }
}

// Pixels per lane cs.npx is a launch parameter: the host picks it so the
// n_pairs x G workgroups spread over every CU (the pixel phase of one wave
// is latency-bound, so it costs ~npx x the per-pixel chain: DESIGN.md §5);
// kThreads = 512 puts two waves on each SIMD to hide that latency.  Lane t
// of chunk c owns source pixels c kThreads npx + s kThreads + t, s < npx;
// their back-projected X/Y/Z live in dynamic LDS [3][npx][kThreads] for the
// whole launch.
template <int kSp, bool kFast, int kThreads, int kTH>
__global__ __launch_bounds__(kThreads, 2) void k_icp_coop(const int16_t* __restrict__ dsrc,
                                                             const float4* __restrict__ recs,
                                                             size_t P, PairMap pm, int W, int H,
                                                             Intr K, FastK F, float thr2,
                                                             CoopState cs)
{
    extern __shared__ float coop_src[];  // [3][npx][kThreads]
    __shared__ float sPX[(kTH + 2) * kLdsW];  // fused prep neighbourhood
    __shared__ float sPY[(kTH + 2) * kLdsW];
    __shared__ float sPZ[(kTH + 2) * kLdsW];
    __shared__ double red[kThreads / 64][kNeq];
    __shared__ double colsum[kSumCols][kPartStride];
    __shared__ double sh_neq[kNeq];
    __shared__ double sh_T64[12];
    __shared__ float sh_T[12];
    __shared__ int sh_stop;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int G = cs.G;
    const int npx = cs.npx;
    const int p = blockIdx.x / G;
    const int c = blockIdx.x - p * G;
    const int N = W * H;
    unsigned* err = cs.set + kCoopErrWord;
    unsigned* prep_cnt = cs.set + kCoopPrepWords + (size_t)p * kCoopPrepPair;
    // the prep counter this pair waits on: its own (prep_wait), or in a
    // tracker chain the previous pair's (whose prep is this pair's target)
    const bool prep_wait = cs.chain ? p > 0 : cs.prep_wait != 0;
    unsigned* wait_cnt = cs.chain ? prep_cnt - kCoopPrepPair : prep_cnt;
    const int tgt_frame = cs.chain ? cs.tgt_slot[p] : pm.tgt0 + p;
    float* X = coop_src;
    float* Y = coop_src + npx * kThreads;
    float* Z = coop_src + 2 * npx * kThreads;

    COOP_MARK(3, 15);  // prologue stamps: kernel entry (slot 15 of iterations 3, 0, 1, 2)
    if (blockIdx.x == 0) {
        // the next call's words: the timeout word and every prep shard word
        // (word 0 of each 128-B line; the rest of a line is never used)
        for (int i = threadIdx.x; i < 1 + kCoopMaxPairs * kCoopPrepShards; i += kThreads)
            st_u32_sc1(cs.set_next + (i == 0 ? kCoopErrWord
                                             : kCoopPrepWords + (i - 1) * kCoopShardStride),
                       0u);
        if (threadIdx.x == 0) {
            st_u32_sc1(cs.head_err + kQError, 0u);
            st_u32_sc1(cs.head_err + kQSpins, 0u);
            st_u32_sc1(cs.head_err + kQWaited, 0u);
        }
    }
    // the previous call's partial rows (the other arena) back to EMPTY, for
    // the next call; spread over the whole grid
    if (cs.part_reset > 0) {
        const unsigned per = (unsigned)cs.part_reset * kPartStride;  // doubles per buffer
        const unsigned stride = gridDim.x * kThreads;
        for (unsigned i = blockIdx.x * kThreads + threadIdx.x; i < kCoopBufs * per; i += stride) {
            const unsigned b = i / per;
            st_u64_sc1(cs.part_next + (size_t)b * cs.part_cap * kPartStride + (i - b * per),
                       kPartEmpty);
        }
    }
    if (threadIdx.x < 12) {
        const double v = cs.T_init ? cs.T_init[(size_t)p * 16 + threadIdx.x]
                                   : ((threadIdx.x % 5) == 0 ? 1.0 : 0.0);
        sh_T64[threadIdx.x] = v;
        sh_T[threadIdx.x] = (float)v;
    }
    // ---- fused target prep: tiles c, c + G, ... of pair p's target frame,
    // records stored write-through (sc1); every storing wave drains, then
    // one arrival on the pair's prep counter (R1 hand-off)
    if (cs.prep_src) {
        const int tiles_x = (W + kTileW - 1) / kTileW;
        const int tiles = tiles_x * ((H + kTH - 1) / kTH);
        const int16_t* tdep = cs.prep_src + (size_t)p * N;
        float4* R = const_cast<float4*>(recs) +
                    (size_t)(cs.chain ? cs.prep_slot[p] : cs.prep_out0 + p) * P;
        for (int t = c; t < tiles; t += G) {  // uniform per workgroup
            const int ty = t / tiles_x;
            const int x0 = (t - ty * tiles_x) * kTileW, y0 = ty * kTH;
            if (cs.prep_wide)
                prep_tile<kFast, true, true, kThreads, kTH>(tdep, R, W, H, P, K, F, nullptr,
                                                                   x0, y0, sPX, sPY, sPZ);
            else
                prep_tile<kFast, false, true, kThreads, kTH>(tdep, R, W, H, P, K, F,
                                                                    nullptr, x0, y0, sPX, sPY, sPZ);
            __syncthreads();  // LDS planes reused by the next tile
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave
        __syncthreads();
        if ((cs.prep_wait || cs.chain) && threadIdx.x == 0)
            __hip_atomic_fetch_add(prep_cnt + (c & (kCoopPrepShards - 1)) * kCoopShardStride, 1u,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    COOP_MARK(0, 15);  // prep published
    // ---- this workgroup's source pixels, back-projected once (spec a2)
    {
        const int16_t* sD = dsrc + (size_t)(pm.src0 + p) * N;
        const int base = c * npx * kThreads + threadIdx.x;
        const int tiles_x = (W + kTileW - 1) / kTileW;
        const int tyc = c / tiles_x;
        const int tx0 = (c - tyc * tiles_x) * kTileW, ty0 = tyc * kTH;
        for (int s = 0; s < npx; ++s) {
            int u, v;
            bool inr;
            if (cs.tile_src) {
                const int k = s * kThreads + threadIdx.x;
                u = tx0 + (k & (kTileW - 1));
                v = ty0 + k / kTileW;
                inr = u < W && v < H;
            } else {
                const int i = base + s * kThreads;
                inr = i < N;
                v = inr ? i / W : 0;
                u = inr ? i - v * W : 0;
            }
            const int d = inr ? (int)sD[(size_t)v * W + u] : 0;
            float x, y, z;
            backproject<kFast>(d, inr ? u : 0, inr ? v : 0, K, F, x, y, z);
            X[s * kThreads + threadIdx.x] = x;
            Y[s * kThreads + threadIdx.x] = y;
            Z[s * kThreads + threadIdx.x] = z;
        }
    }
    const __amdgpu_buffer_rsrc_t rrec = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float4*>(recs + (size_t)tgt_frame * P), (short)0,
        (int)(P * sizeof(float4)), 0x00020000);
    const size_t buf_stride = (size_t)cs.part_cap * kPartStride;  // doubles per buffer
    double* const part0 = cs.part + (size_t)p * G * kPartStride;  // pair p's rows, buffer 0
    int32_t st_acc = 0;
    bool timeout = false;
    COOP_MARK(1, 15);  // source pixels staged
    if (cs.prep_src && prep_wait) {
        // every workgroup of pair p prepped its tiles: ONE relaxed poll (lane
        // s of wave 0 polls shard s, which counts the chunks c = s mod 8);
        // the other waves load after the barrier below, and every gather of
        // the records is an sc1 load (coop_group), so no acquire follows
        if (wave == 0) {
            const unsigned want = lane < kCoopPrepShards
                                      ? (unsigned)((G - lane + kCoopPrepShards - 1) / kCoopPrepShards)
                                      : 0u;
            unsigned spins = 0;
            int stop = 0;
            for (;;) {
                const unsigned have =
                    lane < kCoopPrepShards ? ld_u32_sc1(wait_cnt + lane * kCoopShardStride) : 0u;
                if (__ballot(have < want) == 0ull) break;
                __builtin_amdgcn_s_sleep(1);
                if (++spins > cs.spin_max || ld_u32_sc1(err) != 0u) {
                    if (lane == 0)
                        __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    stop = 1;
                    break;
                }
            }
            if (lane == 0) sh_stop = stop;
        }
        __syncthreads();
        timeout = __builtin_amdgcn_readfirstlane(sh_stop) != 0;
    } else {
        if (threadIdx.x == 0) sh_stop = 0;
        __syncthreads();
    }

    COOP_MARK(2, 15);  // every record of the pair visible
    for (int k = 0; k < cs.iters && !timeout; ++k) {
        COOP_MARK(k, 0);
        float T[12];
#pragma unroll
        for (int q = 0; q < 12; ++q)
            T[q] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(sh_T[q])));
        double acc[kNeq];
        // lane32: the lane's fp32 sums over its npx pixels, converted once
        typedef std::conditional_t<sp_lane32(kSp), float, double> A;
        A la[28];
#pragma unroll
        for (int q = 0; q < 28; ++q) la[q] = A(0);
        int nmatch = 0;
        int s0 = 0;
        for (; s0 + 4 <= npx; s0 += 4)
            coop_group<kSp, kFast, 4, kThreads>(X, Y, Z, s0, T, rrec, W, H, K, F, thr2, la, nmatch);
        switch (npx - s0) {  // wave-uniform tail
        case 3: coop_group<kSp, kFast, 3, kThreads>(X, Y, Z, s0, T, rrec, W, H, K, F, thr2, la, nmatch); break;
        case 2: coop_group<kSp, kFast, 2, kThreads>(X, Y, Z, s0, T, rrec, W, H, K, F, thr2, la, nmatch); break;
        case 1: coop_group<kSp, kFast, 1, kThreads>(X, Y, Z, s0, T, rrec, W, H, K, F, thr2, la, nmatch); break;
        default: break;
        }
#pragma unroll
        for (int q = 0; q < 28; ++q) acc[q] = (double)la[q];
        acc[28] = lane == 0 ? (double)nmatch : 0.0;  // the wave's count, lane 0
        COOP_MARK(k, 1);
        if (wave < 4) COOP_MARK_WAVE(k, 11 + wave);  // slots 12-14: waves 1-3 pixel loop done
        {
            double tot;
            wave_reduce_scatter(acc, lane, tot);
            COOP_MARK(k, 11);
            if (!(lane & 1) && (lane >> 1) < kNeq) red[wave][lane >> 1] = tot;
        }
        __syncthreads();
        double* part = part0 + (size_t)(k % kCoopBufs) * buf_stride;
        COOP_MARK(k, 2);
        if (wave == 0) {
            // ---- store this chunk's partial row (sc1) over its EMPTY row.
            // The drain first: this wave's reset of its row of buffer
            // (k+1) % 3 (stored at iteration k-1) must be visible before any
            // value of iteration k is (see the hand-off above)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            double sum = 0.0;
            if (lane < kPartStride && !(k == cs.stall_iter && p == 0 && c == cs.stall_chunk)) {
                if (lane < kNeq) {  // the waves' sums as a pairwise tree (3 dependent adds)
                    double r[kThreads / 64];
#pragma unroll
                    for (int w = 0; w < kThreads / 64; ++w) r[w] = red[w][lane];
                    sum = tree_sum<kThreads / 64>(r);
                }
                st_u64_sc1(part + (size_t)c * kPartStride + lane,
                           (unsigned long long)__double_as_longlong(sum));
            }
            COOP_MARK(k, 3);
            COOP_MARK(k, 4);
        }
        COOP_MARK(k, 5);
        // ---- every workgroup sums the pair's partials in the same fixed
        // order, as soon as each row has landed (no counter, no barrier)
        const __amdgpu_buffer_rsrc_t rpart = __builtin_amdgcn_make_buffer_rsrc(
            part, (short)0, G * kPartStride * (int)sizeof(double), 0x00020000);
        int stop = 0;
        const double tsum = sum_pair_rows_polled<16>(rpart, G, colsum, err, &sh_stop,
                                                      cs.poll_delay, cs.spin_max, stop);
        COOP_MARK(k, 6);
        if (stop) {
            timeout = true;
            break;
        }
        if (wave == 0) {
            if (lane < kNeq) sh_neq[lane] = tsum;
            if (c == 0 && cs.stats && lane == 0) {
                cs.stats[((size_t)p * cs.iters + k) * 2 + 0] = readlane64(tsum, 28);
                cs.stats[((size_t)p * cs.iters + k) * 2 + 1] = readlane64(tsum, 27);
            }
            COOP_MARK(k, 8);
            st_acc |= solve_update_wave(sh_neq, sh_T64, sh_T, lane);
            COOP_MARK(k, 9);
            // every row of iteration k seen: every workgroup of the pair has
            // read iteration k-1's, so this row of that buffer ((k+2) % 3,
            // written next at iteration k+2) goes back to EMPTY now
            if (k + 2 < cs.iters && lane < kPartStride)
                st_u64_sc1(part0 + (size_t)((k + 2) % kCoopBufs) * buf_stride +
                               (size_t)c * kPartStride + lane,
                           kPartEmpty);
            COOP_MARK(k, 10);
        }
        __syncthreads();
        COOP_MARK(k, 7);
    }

    // ---- pair p's results, from its chunk-0 workgroup (replaces k_finish)
    if (c == 0 && threadIdx.x < 16) {
        const int i = threadIdx.x;
        const double v = i < 12 ? sh_T64[i]
                                : (cs.T_init ? cs.T_init[(size_t)p * 16 + i] : (i == 15 ? 1.0 : 0.0));
        cs.T64[(size_t)p * 16 + i] = v;
        if (i < 12) cs.T32[(size_t)p * 12 + i] = (float)v;
        if (cs.T_out) cs.T_out[(size_t)p * 16 + i] = i < 12 ? (float)v : (i == 15 ? 1.0f : 0.0f);
        const int32_t st = st_acc | (timeout ? YOUTH_STATUS_TIMEOUT : 0);
        if (i == 0) cs.status[p] = st;
        double* res = cs.chain ? cs.res_pair[p] : (p == 0 ? cs.res_host : nullptr);
        if (res) {
            // fine-grained pinned slot: system-scope stores go to host memory
            // past the L2, and the wave waits for them before it ends, so the
            // tracker's completion event needs no system-scope L2 writeback
            __hip_atomic_store(res + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if (i == 0)
                __hip_atomic_store(reinterpret_cast<int32_t*>(res + 16), st,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __builtin_amdgcn_s_waitcnt(0);
        }
    }
}

// Copy out fp32 4x4 poses (optional) and fold a persistent-kernel timeout
// into every pair's status.
__global__ void k_finish(const double* __restrict__ T64, int n, float* __restrict__ out,
                         int32_t* __restrict__ status, const unsigned* __restrict__ error)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * 16) return;
    const int i = t & 15;
    if (out) out[t] = i < 12 ? (float)T64[(size_t)(t >> 4) * 16 + i] : (i == 15 ? 1.0f : 0.0f);
    if (i == 0 && error && *error) status[t >> 4] |= YOUTH_STATUS_TIMEOUT;
}

// The tracker's H2D of m page-locked host frames, pulled by the GPU itself
// (the default; YOUTH_ICP_TRACK_COPY=sdma uses hipMemcpyAsync on the copy
// engine instead).  On the shared GPU hosts the SDMA path ran at 36-41 K
// frames/s in quiet passes but stalled the submitting thread inside
// hipMemcpyAsync for 8-18 ms about once in ten backlogged passes and fell to
// ~9 K frames/s while the host was loaded; this kernel's passes stayed within
// a few per cent of each other under the same conditions (DESIGN.md §6,
// profiles/r05/).  Few 64-lane workgroups (a total of ~32 per launch), four
// 16-byte loads in flight per lane, so its waves sit beside the resident
// cooperative grid of the launch before it without slowing it much.
struct FramePtrs {
    const int16_t* src[kCoopMaxChain];
};
__global__ __launch_bounds__(64) void k_pull_frames(FramePtrs fp, int16_t* __restrict__ dst, int N,
                                                    int m)
{
    const int f = blockIdx.y;
    if (f >= m) return;
    const int16_t* __restrict__ s16 = fp.src[f];
    int16_t* __restrict__ d16 = dst + (size_t)f * N;
    const int stride = gridDim.x * 64;
    const int t0 = blockIdx.x * 64 + threadIdx.x;
    // 16-byte body when both ends are 16-byte aligned (page-locked buffers
    // and W*H % 8 == 0 frames), else element by element
    const bool vec = (((uintptr_t)s16 | (uintptr_t)d16) & 15) == 0;
    int done = 0;
    if (vec) {
        typedef int v4i __attribute__((ext_vector_type(4)));
        const v4i* __restrict__ s = reinterpret_cast<const v4i*>(s16);
        v4i* __restrict__ d = reinterpret_cast<v4i*>(d16);
        const int nv = N / 8;
        int i = t0;
        for (; i + 3 * stride < nv; i += 4 * stride) {
            const v4i a = __builtin_nontemporal_load(s + i);
            const v4i b = __builtin_nontemporal_load(s + i + stride);
            const v4i c = __builtin_nontemporal_load(s + i + 2 * stride);
            const v4i e = __builtin_nontemporal_load(s + i + 3 * stride);
            d[i] = a;
            d[i + stride] = b;
            d[i + 2 * stride] = c;
            d[i + 3 * stride] = e;
        }
        for (; i < nv; i += stride) d[i] = __builtin_nontemporal_load(s + i);
        done = nv * 8;
    }
    for (int i = done + t0; i < N; i += stride) d16[i] = s16[i];
}

// Per-pair status of one chunk of the host batch API, the launch's timeout
// flag folded in (as youth_icp_get_poses does).
__global__ void k_status_out(const int32_t* __restrict__ status, int n,
                             const unsigned* __restrict__ error, int32_t* __restrict__ out)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) out[t] = status[t] | (*error ? YOUTH_STATUS_TIMEOUT : 0);
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
    FastK F{};
    bool fast = false;  // verified 2-op back-projection division
    bool centred_exact = true;  // aligned loop's centred columns exact (centred_exact)
    int spec = kSpecSurvey;  // spec a7/a8 arithmetic (youth_icp_set_spec, YOUTH_ICP_SPEC)
    youth_icp_params prm{};
    hipStream_t stream = nullptr;

    int16_t* d_depth = nullptr;  // [max_frames][N] staging for host-side APIs
    float4* d_rec = nullptr;     // [max_frames][P] target records {z, nx, ny, nz}
    float* d_xyz = nullptr;      // [max_frames][3][P] (lazy: stage-level API only)
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
    unsigned* d_flag = nullptr;
    unsigned* d_arrivals = nullptr;  // [max_frames] fused-solve arrival counters
    unsigned* d_arr_it = nullptr;    // [max_frames][stats_iters] persistent arrival tickets
    unsigned* d_epoch = nullptr;     // [max_frames] persistent pose epochs
    unsigned* d_head = nullptr;      // queue words kQHead / kQError / kQSpins / kQWaited
    bool persistent = true;          // one k_icp launch per align (else per-iteration k_reduce)
    int reduce = YOUTH_REDUCE_EXACT; // spec a9 (youth_icp_set_reduce, YOUTH_ICP_REDUCE)
    youth_lanes lanes{};             // lane partition of the last align's iterations
    bool has_lanes = false;
    bool lanes_mixed = false;        // the last host batch call ran more than one partition
    int icp_blocks_per_cu[4 * kVariants] = {};  // occupancy of k_icp<variant, fast, aligned> [variant 4 + fast 2 + aligned]
    int n_cu = 0;
    // small batches: k_icp_coop (youth_icp_create reads the knobs)
    bool coop = true;                // YOUTH_ICP_NO_COOP=1 disables
    int coop_px = 0;                 // YOUTH_ICP_COOP_PX: force pixels per lane (0: plan)
    int coop_px_env = 0;             // coop_px outside the tracker's batch mode
    int coop_threads = 512;          // YOUTH_ICP_COOP_THREADS=256: one wave per SIMD
    int coop_max_pairs = kCoopMaxPairs;  // YOUTH_ICP_COOP_MAX_PAIRS (<= kCoopMaxPairs)
    int coop_launch = 0;             // YOUTH_ICP_COOP_LAUNCH: 0 serial (default), 1 runtime, 2 plain
    bool trk_copy_compute = false;   // YOUTH_ICP_TRACK_COPY=compute: tracker H2D on the launch stream
    bool trk_copy_sdma = false;      // YOUTH_ICP_TRACK_COPY=sdma: hipMemcpyAsync, not k_pull_frames
    int trk_pull_wg = 0;             // YOUTH_ICP_PULL_WG: k_pull_frames workgroups per frame (0: auto)
    int trk_pull_lds = 48 << 10;     // YOUTH_ICP_PULL_LDS: LDS bytes a k_pull_frames workgroup reserves
    int trk_pull_reserve = 32;       // YOUTH_ICP_PULL_RESERVE_CU: CUs a micro-batch plan leaves free
    // staging copies of host frames (track_submit_batch / track_host_sequence):
    // split over the submitting thread and trk_copy_helpers persistent threads
    // once a submission holds trk_copy_min bytes (host_copy.h); the pool starts
    // with the first such submission
    int trk_copy_helpers = 3;        // YOUTH_ICP_COPY_THREADS: helper threads (0: one thread copies)
    size_t trk_copy_min = 1u << 20;  // bytes per submission from which the copy is split
    std::unique_ptr<youth::HostCopyPool> copy_pool;
    bool coop_refuse = false;       // YOUTH_ICP_TEST_REFUSE_COOP=1 (test hook)
    // occupancy of k_icp_coop<variant, fast, threads> [threads 256?][variant 2 + fast] at npx (LDS)
    int coop_bpc[2][2 * kVariants][kCoopMaxPx + 1] = {};
    int coop_bpc_tall[2 * kVariants] = {};  // the 64 x 80 prep-tile kernel at 10 px per lane
    unsigned* d_coop = nullptr;      // 2 counter sets of kCoopSetWords
    int32_t* d_status_out = nullptr; // [max_frames] host batch API: status per pair of the call
    int coop_par = 0;                // set (and partial-row arena) used by the next coop call
    double* d_coop_part = nullptr;   // 2 arenas x kCoopBufs x coop_part_cap rows (EMPTY when idle)
    int coop_part_cap = 0;           // rows per buffer
    int coop_part_rows[2] = {0, 0};  // rows per buffer the last call on each arena used
    int coop_poll_delay = -1;        // YOUTH_ICP_COOP_POLL_DELAY (x 64 clocks); -1: G / 8
    int coop_stall_once = -1;        // YOUTH_ICP_TEST_COOP_STALL (test hook): chunk that stalls
    int coop_stall_left = 0;         // coop launches the hook still stalls
    int coop_stall_iter = 1;         // YOUTH_ICP_TEST_COOP_STALL_ITER: the iteration whose row is lost
    bool realign_stall = false;      // YOUTH_ICP_TEST_REALIGN_STALL=1 (test hook): realigns' coop launches stall
    int last_coop_G = 0, last_coop_px = 0;
    bool last_coop = false;          // the last align ran k_icp_coop

    int last_pairs = 0;
    int last_iters = 0;
    hipStream_t last_stream = nullptr;

    int track_ref = -1;  // ring slot (0/1) of the tracker's reference frame
    double* coop_res_host = nullptr;  // set around a tracker align: k_icp_coop writes its result there
    bool coop_tile_src = true;        // YOUTH_ICP_COOP_TILE_SRC=0: contiguous source chunks
    int trk_batch = 1;                // frames per submission in youth_icp_track_host_sequence
    long long trk_chained = 0;        // micro-batch launches so far (youth_icp_track_chained)
    long long trk_chained_frames = 0; // frames those launches aligned (youth_icp_track_chained_frames)
    long long trk_realigned[3] = {};  // youth_icp_track_realign: coop / persistent / still failed
    long long batch_realigned = 0;    // host batch API chunks realigned after a coop timeout
    int queues = 0;                  // k_icp work queues (YOUTH_ICP_QUEUES=1..8; 0: by batch size)
    int share = 1;                   // contexts launching k_icp concurrently (set_concurrency)
    int prep_xcd_map = 0;             // YOUTH_ICP_PREP_XCD_MAP=1: k_prep tiles contiguous per XCD (slower)
    // pipelined tracking (youth_icp_track_submit / _collect): up to
    // kTrackDepth frames in flight, each with a pinned staging buffer, pinned
    // results and events
    struct TrackSlot {
        int16_t* pinned = nullptr;     // host depth copy, H2D source
        double* res = nullptr;         // pinned: T64 [16], then the status word
        hipEvent_t h2d = nullptr;      // staging -> device depth done (xfer)
        hipEvent_t done = nullptr;     // align + result D2H done (stream)
        hipEvent_t done_nf = nullptr;  // the same without the system-scope fence (the
                                       // kernel stored the result to host memory itself)
        hipEvent_t ev = nullptr;       // the one of the two recorded for this submission
        int has_ref = 0;
    } trk[kTrackDepth];
    int trk_dslot_last[2 * YOUTH_TRACK_MAX_BATCH];  // trk[] entry of the last launch that read depth slot d (-1: none)
    int trk_prev_d0 = -1;                       // first depth slot of the last launch
    int trk_head = 0, trk_n = 0;       // oldest in-flight submission, count in flight
    int trk_cap = 2;                   // ring entries in use (grows to kTrackDepth on demand)

    // host-buffer batch API: H2D of chunk k+1 on xfer overlaps the align of chunk k
    hipStream_t xfer = nullptr;
    std::vector<hipEvent_t> xfer_ev;

    bool timing = false;
    bool timing_iter_only = false;  // set_timing(2): events around the iteration kernel only
    std::vector<EventPair> ev_live;
    std::vector<EventPair> ev_free;
    double t_ms[3] = {0, 0, 0};
    int t_n[3] = {0, 0, 0};
};

// The kernels' template variant of a context: spec a7/a8 arithmetic in bit
// 0, the lane32 reduction of spec a9 in bit 1.
static int variant(const youth_icp_ctx* c)
{
    return c->spec | (c->reduce == YOUTH_REDUCE_LANE32 ? kRedLane32 : 0);
}

static int reduce_geometry(const youth_icp_ctx* c, int n_pairs, int* chunk_out)
{
    // work chunks per iteration: fewer chunks make items wait for their
    // pair's pose, more pay the per-item hand-off.  Measured
    // best (tools/chunk_sweep.sh, profiles/r02/chunk_sweep.txt): ~2048 up to
    // 256 pairs per launch (64 pairs: +2.4 %, 128: +3.4 % over 3072), ~3072
    // above.  At least 8 pixels per lane.
    static const int knob = [] {
        const char* e = getenv("YOUTH_ICP_TARGET_CHUNKS");  // tuning knob
        const int v = e ? atoi(e) : 0;
        return v > 0 ? v : 0;
    }();
    // a context that shares the device with share - 1 concurrent ones runs on
    // 1/share of the workgroup slots, so it takes 1/share of the chunks: the
    // same items per workgroup and iteration (youth_icp_set_concurrency).
    // Shared, <= 96 pairs: 1536 / share (64 pairs, share 2: 768 chunks 81.6 K
    // aligns/s, 1024 81.1 K, 1280 79.9 K; profiles/r03/ab_share.txt)
    const int base = c->share > 1 && n_pairs <= 96 ? 1536 : (n_pairs <= 256 ? 2048 : 3072);
    const int target_blocks = (knob ? knob : base) / c->share;
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

// k_icp_coop's partial-row arenas, every row EMPTY (k_icp_coop comment).  A
// call needing more rows than there are reallocates (hipFree waits for the
// device, so no launch still uses the old rows).  The EMPTY fill is enqueued
// on the launch's stream ahead of the launch; any later coop launch of this
// context is ordered after this one (coop_enqueue), so after the fill too.
static int ensure_coop_part(youth_icp_ctx* c, hipStream_t s, int rows)
{
    if (rows <= c->coop_part_cap) return YOUTH_OK;
    const int cap = std::max(rows, c->n_cu * 2);
    if (c->d_coop_part) HIP_TRY(hipFree(c->d_coop_part));
    c->d_coop_part = nullptr;
    c->coop_part_cap = 0;
    const size_t doubles = (size_t)2 * kCoopBufs * cap * kPartStride;
    HIP_TRY(hipMalloc(&c->d_coop_part, doubles * sizeof(double)));
    static_assert((unsigned)(kPartEmpty >> 32) == (unsigned)kPartEmpty, "EMPTY fills by words");
    HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)c->d_coop_part, (int)kPartEmptyHi, doubles * 2, s));
    c->coop_part_cap = cap;
    c->coop_part_rows[0] = c->coop_part_rows[1] = 0;
    return YOUTH_OK;
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
    if (c->d_arr_it) HIP_TRY(hipFree(c->d_arr_it));
    c->d_stats = nullptr;
    c->d_arr_it = nullptr;
    HIP_TRY(hipMalloc(&c->d_stats, (size_t)c->max_frames * iters * 2 * sizeof(double)));
    HIP_TRY(hipMalloc(&c->d_arr_it, (size_t)c->max_frames * iters * sizeof(unsigned)));
    c->stats_iters = iters;
    return YOUTH_OK;
}

static int ensure_assoc(youth_icp_ctx* c)
{
    if (c->d_assoc) return YOUTH_OK;
    HIP_TRY(hipMalloc(&c->d_assoc, (size_t)c->max_frames * c->N * sizeof(int32_t)));
    return YOUTH_OK;
}

static int ensure_xyz(youth_icp_ctx* c)
{
    if (c->d_xyz) return YOUTH_OK;
    const size_t bytes = 3 * c->P * sizeof(float) * (size_t)c->max_frames;
    HIP_TRY(hipMalloc(&c->d_xyz, bytes));
    HIP_TRY(hipMemset(c->d_xyz, 0, bytes));
    return YOUTH_OK;
}

static int ev_begin(youth_icp_ctx* c, hipStream_t s, EventPair* ep, int kind)
{
    ep->a = nullptr;
    if (!c->timing || (c->timing_iter_only && kind != 0)) return YOUTH_OK;
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
    if (!c->timing || !ep->a) return YOUTH_OK;
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

// Target records (and optionally XYZ planes) for n_frames depth frames at
// `depth`, into workspace frames [out0, out0 + n_frames).
static int launch_prep(youth_icp_ctx* c, hipStream_t s, const int16_t* depth, int n_frames,
                       int out0, bool want_xyz, const InitArgs* init = nullptr)
{
    if (n_frames <= 0) return YOUTH_OK;
    if (want_xyz) {
        int rc = ensure_xyz(c);
        if (rc) return rc;
    }
    const int tiles_x = (c->W + kPrepTW - 1) / kPrepTW, tiles_y = (c->H + kPrepTH - 1) / kPrepTH;
    const long long rows = (long long)tiles_y * n_frames;
    const long long blocks = (long long)tiles_x * (c->prep_xcd_map == 2 ? (rows + 7) / 8 * 8 : rows);
    if (blocks > 0x7fffffffLL) return set_error(YOUTH_EINVAL, "launch_prep: %lld tiles", blocks);
    EventPair ep{};
    int rc = ev_begin(c, s, &ep, 2);
    if (rc) return rc;
    float* xyz = want_xyz ? c->d_xyz : nullptr;
    const bool wide = (c->W % 4 == 0) && (reinterpret_cast<uintptr_t>(depth) % 8 == 0);
    auto kern = c->fast ? (wide ? k_prep<true, true> : k_prep<true, false>)
                        : (wide ? k_prep<false, true> : k_prep<false, false>);
    const InitArgs ia = init ? *init : InitArgs{};
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kPrepThreads), 0, s, depth, out0, c->W,
                       c->H, c->P, c->K, c->F, c->d_rec, xyz, ia, tiles_x, tiles_y, n_frames,
                       c->prep_xcd_map);
    HIP_TRY(hipGetLastError());
    return ev_end(c, s, &ep);
}

template <int kSp, bool kAssoc, bool kFast, bool kAligned, bool kFuse>
static void launch_reduce_t(youth_icp_ctx* c, hipStream_t s, dim3 grid, const int16_t* dsrc,
                            PairMap pm, float thr2, int chunk, const PoseState& ps)
{
    hipLaunchKernelGGL((k_reduce<kSp, kAssoc, kFast, kAligned, kFuse>), grid, dim3(kRedThreads), 0,
                       s, dsrc, c->d_rec, c->P, pm, c->W, c->H, c->K, c->F, thr2, chunk,
                       c->d_partials, kAssoc ? c->d_assoc : (int32_t*)nullptr, ps);
}

// sel = assoc 8 | fuse 4 | fast 2 | aligned 1 (assoc with fuse excluded)
template <int kSp>
static void launch_reduce_sel(youth_icp_ctx* c, hipStream_t s, dim3 grid, const int16_t* dsrc,
                              PairMap pm, float thr2, int chunk, const PoseState& ps, int sel)
{
    switch (sel) {
    case 0: launch_reduce_t<kSp, false, false, false, false>(c, s, grid, dsrc, pm, thr2, chunk, ps); break;
    case 1: launch_reduce_t<kSp, false, false, true, false>(c, s, grid, dsrc, pm, thr2, chunk, ps); break;
    case 2: launch_reduce_t<kSp, false, true, false, false>(c, s, grid, dsrc, pm, thr2, chunk, ps); break;
    case 3: launch_reduce_t<kSp, false, true, true, false>(c, s, grid, dsrc, pm, thr2, chunk, ps); break;
    case 4: launch_reduce_t<kSp, false, false, false, true>(c, s, grid, dsrc, pm, thr2, chunk, ps); break;
    case 5: launch_reduce_t<kSp, false, false, true, true>(c, s, grid, dsrc, pm, thr2, chunk, ps); break;
    case 6: launch_reduce_t<kSp, false, true, false, true>(c, s, grid, dsrc, pm, thr2, chunk, ps); break;
    case 7: launch_reduce_t<kSp, false, true, true, true>(c, s, grid, dsrc, pm, thr2, chunk, ps); break;
    case 8: launch_reduce_t<kSp, true, false, false, false>(c, s, grid, dsrc, pm, thr2, chunk, ps); break;
    case 9: launch_reduce_t<kSp, true, false, true, false>(c, s, grid, dsrc, pm, thr2, chunk, ps); break;
    case 10: launch_reduce_t<kSp, true, true, false, false>(c, s, grid, dsrc, pm, thr2, chunk, ps); break;
    default: launch_reduce_t<kSp, true, true, true, false>(c, s, grid, dsrc, pm, thr2, chunk, ps); break;
    }
}

// fuse_it >= 0: fused solve of iteration fuse_it (k_reduce's last workgroup
// per pair updates the pose); fuse_it < 0: partials only (k_solve follows).
static int launch_reduce(youth_icp_ctx* c, hipStream_t s, const int16_t* dsrc, PairMap pm,
                         int n_pairs, bool assoc, int* nblk_out, int fuse_it = -1)
{
    int chunk = 0;
    const int nb = reduce_geometry(c, n_pairs, &chunk);
    int rc = ensure_partials(c, (size_t)nb * n_pairs * kNeq);
    if (rc) return rc;
    if (assoc) {
        rc = ensure_assoc(c);
        if (rc) return rc;
    }
    const float thr2 = c->prm.dist_thresh * c->prm.dist_thresh;
    const bool aligned = (reinterpret_cast<uintptr_t>(dsrc) % 8 == 0) && (c->W % 4 == 0) &&
                           c->centred_exact;
    dim3 grid(nb, n_pairs);
    EventPair ep{};
    rc = ev_begin(c, s, &ep, 0);
    if (rc) return rc;
    const PoseState ps{c->d_T64, c->d_T32, c->d_status, c->d_stats, c->d_arrivals,
                       fuse_it < 0 ? 0 : fuse_it, c->prm.iters};
    const bool fuse = fuse_it >= 0;
    if (assoc && fuse) return set_error(YOUTH_EINVAL, "launch_reduce: assoc with fused solve");
    const int sel = (assoc ? 8 : 0) | (fuse ? 4 : 0) | (c->fast ? 2 : 0) | (aligned ? 1 : 0);
    switch (variant(c)) {
    case 0: launch_reduce_sel<0>(c, s, grid, dsrc, pm, thr2, chunk, ps, sel); break;
    case 1: launch_reduce_sel<1>(c, s, grid, dsrc, pm, thr2, chunk, ps, sel); break;
    case 2: launch_reduce_sel<2>(c, s, grid, dsrc, pm, thr2, chunk, ps, sel); break;
    default: launch_reduce_sel<3>(c, s, grid, dsrc, pm, thr2, chunk, ps, sel); break;
    }
    HIP_TRY(hipGetLastError());
    c->lanes = youth_lanes{YOUTH_LANES_STRIDED, chunk, kRedThreads, 0};
    c->has_lanes = true;
    c->lanes_mixed = false;
    *nblk_out = nb;
    return ev_end(c, s, &ep);
}

// Small-batch plan.  One wave per SIMD issues a wave64 instruction in >= 4
// cycles, so a pair's pixel phase costs ~ npx x (workgroups per CU): pick
// the npx (source pixels per lane) minimising npx x ceil(n_pairs G / CUs)
// among those whose n_pairs x G workgroups fit the co-resident capacity with
// one block per CU to spare (cooperative launch admission,
// MI355X_MICROARCH.md); ties go to the larger npx (fewer partials to sum).
static size_t coop_lds(int npx, int threads) { return (size_t)3 * npx * threads * sizeof(float); }

static bool coop_plan(const youth_icp_ctx* c, int n_pairs, int* npx_out, int* G_out)
{
    if (!c->coop || n_pairs > c->coop_max_pairs || n_pairs > kCoopMaxPairs) return false;
    const int v = variant(c) * 2 + (c->fast ? 1 : 0);
    long long best = -1;
    for (int npx = 1; npx <= kCoopMaxPx; ++npx) {
        if (c->coop_px && npx != c->coop_px) continue;
        const int chunk = npx * c->coop_threads;
        const int G = (c->N + chunk - 1) / chunk;
        const long long wgs = (long long)G * n_pairs;
        // VGPR-limited occupancy: k_icp_coop's SGPR count (106) admits 6
        // 256-thread blocks per CU (MI355X_MICROARCH.md residency formula),
        // more than the API's VGPR answer, so the API count is exact here
        const int bpc = c->coop_bpc[c->coop_threads == 256][v][npx];
        if (bpc < 1 || wgs > (long long)c->n_cu * bpc) continue;
        const long long cost = (long long)npx * ((wgs + c->n_cu - 1) / c->n_cu);
        if (best < 0 || cost <= best) {
            best = cost;
            *npx_out = npx;
            *G_out = G;
        }
    }
    return best >= 0;
}

template <int kSp>
static const void* coop_kernel_t(bool fast, int threads, bool tall)
{
    if (threads == 256)
        return fast ? (const void*)k_icp_coop<kSp, true, 256, kCoopTileH>
                    : (const void*)k_icp_coop<kSp, false, 256, kCoopTileH>;
    if (tall)
        return fast ? (const void*)k_icp_coop<kSp, true, 512, kCoopTileHTall>
                    : (const void*)k_icp_coop<kSp, false, 512, kCoopTileHTall>;
    return fast ? (const void*)k_icp_coop<kSp, true, 512, kCoopTileH>
                : (const void*)k_icp_coop<kSp, false, 512, kCoopTileH>;
}

static const void* coop_kernel(int var, bool fast, int threads, bool tall = false)
{
    switch (var) {
    case 0: return coop_kernel_t<0>(fast, threads, tall);
    case 1: return coop_kernel_t<1>(fast, threads, tall);
    case 2: return coop_kernel_t<2>(fast, threads, tall);
    default: return coop_kernel_t<3>(fast, threads, tall);
    }
}

// Target frames to turn into records before (or, for the tracker, beside)
// the iterations: depth frames [depth, depth + n N) -> record frames
// [out0, out0 + n); wait: the iterations gather exactly these records.
struct PrepJob {
    const int16_t* depth;
    int n, out0;
    bool wait;
    // tracker micro-batch (k_icp_coop only; CoopState.chain): pair p preps
    // its source frame into record frame prep_slot[p] and gathers record
    // frame tgt_slot[p]; results to the pinned slots res[p]
    bool chain = false;
    int tgt_slot[kCoopMaxChain] = {}, prep_slot[kCoopMaxChain] = {};
    double* res[kCoopMaxChain] = {};
};

// k_icp_coop's workgroups poll each other, so all n_pairs x G of them must be
// resident together.  The planner sizes the grid to the co-resident capacity
// of an idle device; what remains is another spin-waiting grid occupying the
// CUs at the same time.  In this library that can only be another
// k_icp_coop (k_icp never waits on a workgroup that is not running), so the
// cooperative launches of a device are totally ordered instead, and launched
// as plain kernels: hipLaunchCooperativeKernel's runtime path costs ~20 us
// per launch on ROCm 7 (single-pair aligns/s 9.2 K against 11.3 K,
// profiles/r02/stream_probe.txt).
//   * While every coop launch of the device has come from ONE stream, stream
//     order is the total order: no extra packet.
//   * The first launch from a second stream switches the device to ordered
//     mode for good: the host waits once for the device to drain (the
//     previous stream's last coop grid included; that stream's handle is not
//     touched, the caller may have destroyed it), and from then on every
//     coop launch records the device's
//     completion event and waits on it when its stream differs from the
//     previous launch's (an event record costs ~2.7 us per launch: 10.9 K).
// YOUTH_ICP_COOP_LAUNCH=runtime restores hipLaunchCooperativeKernel.
struct CoopOrder {
    std::mutex mu;
    std::condition_variable cv;  // launches wait while the one-time drain runs
    hipStream_t last = nullptr;
    hipEvent_t done = nullptr;
    bool any = false;
    bool multi = false;     // launches seen from more than one stream
    bool draining = false;  // the first switch's device drain is in progress (mu released)
};
static CoopOrder g_coop_order[64];

static int coop_enqueue(youth_icp_ctx* c, hipStream_t s, void** args, int blocks, int npx,
                        bool tall)
{
    const void* kern = coop_kernel(variant(c), c->fast, c->coop_threads, tall);
    const dim3 grid((unsigned)blocks), block(c->coop_threads);
    const unsigned lds = (unsigned)coop_lds(npx, c->coop_threads);
    if (c->coop_refuse)  // test hook: the runtime's refusal, nothing enqueued
        return set_error(YOUTH_EHIP, "coop_enqueue: cooperative launch refused (test hook)");
    if (c->coop_launch == 1) {
        HIP_TRY(hipLaunchCooperativeKernel(kern, grid, block, args, lds, s));
        return YOUTH_OK;
    }
    if (c->coop_launch == 2 || c->device < 0 || c->device >= 64) {  // unordered (probe only)
        HIP_TRY(hipLaunchKernel(kern, grid, block, args, lds, s));
        return YOUTH_OK;
    }
    CoopOrder& o = g_coop_order[c->device];
    std::unique_lock<std::mutex> lk(o.mu);
    o.cv.wait(lk, [&o] { return !o.draining; });
    if (o.any && o.last != s) {
        if (!o.done) HIP_TRY(hipEventCreateWithFlags(&o.done, hipEventDisableTiming));
        if (!o.multi) {
            // first switch: the previous stream may be a caller's stream that
            // has been destroyed since, so its handle is not used again
            // (ADVICE r3); the host waits once for the device to drain, which
            // covers that stream's last coop grid.  The drain runs without
            // holding mu: other threads' coop launches on this
            // device wait on cv meanwhile (none may start before it ends),
            // nothing else is blocked.  From now on every launch records
            // `done` on its own stream right after it
            o.draining = true;
            lk.unlock();
            const hipError_t e = hipDeviceSynchronize();
            lk.lock();
            o.draining = false;
            o.cv.notify_all();
            if (e != hipSuccess)
                return set_error(YOUTH_EHIP, "coop launch: device drain on the first stream "
                                             "switch: %s", hipGetErrorString(e));
            o.multi = true;
        } else {
            HIP_TRY(hipStreamWaitEvent(s, o.done, 0));
        }
    }
    HIP_TRY(hipLaunchKernel(kern, grid, block, args, lds, s));
    if (o.multi) HIP_TRY(hipEventRecord(o.done, s));
    o.last = s;
    o.any = true;
    return YOUTH_OK;
}

static int launch_coop(youth_icp_ctx* c, hipStream_t s, const int16_t* dsrc, PairMap pm,
                       int n_pairs, const double* dTi, float* d_T_out, int npx, int G,
                       const PrepJob* job)
{
    const int iters = c->prm.iters;
    int rc = ensure_coop_part(c, s, n_pairs * G);
    if (rc) return rc;
    const int par = c->coop_par;
    unsigned* set = c->d_coop + (size_t)par * kCoopSetWords;
    unsigned* set_next = c->d_coop + (size_t)(par ^ 1) * kCoopSetWords;
    c->coop_par ^= 1;
    const bool wide = job && (c->W % 4 == 0) && (reinterpret_cast<uintptr_t>(job->depth) % 8 == 0);
    // tile-shaped source chunks when one target tile is exactly one
    // workgroup's pixels and the pair has one workgroup per tile: 64 x 24
    // tiles at 3 px per lane (640x480), 64 x 80 at 10 (1280x960; that
    // kernel's larger prep LDS must still admit the planned grid)
    auto tiles_of = [&](int th) {
        return ((c->W + kTileW - 1) / kTileW) * ((c->H + th - 1) / th);
    };
    const bool tall = c->coop_tile_src && c->coop_threads == 512 &&
                      npx * 512 == kTileW * kCoopTileHTall && G == tiles_of(kCoopTileHTall) &&
                      (long long)n_pairs * G <= (long long)c->n_cu * c->coop_bpc_tall[variant(c) * 2 + (c->fast ? 1 : 0)];
    const bool tile_src = tall || (c->coop_tile_src && npx * c->coop_threads == kTileW * kCoopTileH &&
                                   G == tiles_of(kCoopTileH));
    CoopState cs{dTi,      c->d_T64, c->d_T32, c->d_status,          c->d_stats,
                 d_T_out,  set,      set_next, c->d_head,            iters,
                 n_pairs,  G,        npx,      job ? job->depth : nullptr,
                 job ? job->out0 : 0, job && job->wait ? 1 : 0, wide ? 1 : 0,
                 c->coop_res_host, tile_src ? 1 : 0};
    if (job && job->chain) {
        cs.chain = 1;
        for (int i = 0; i < kCoopMaxChain; ++i) {
            cs.tgt_slot[i] = job->tgt_slot[i];
            cs.prep_slot[i] = job->prep_slot[i];
            cs.res_pair[i] = job->res[i];
        }
    }
    const size_t arena = (size_t)kCoopBufs * c->coop_part_cap * kPartStride;
    cs.part = c->d_coop_part + (size_t)par * arena;
    cs.part_next = c->d_coop_part + (size_t)(par ^ 1) * arena;
    cs.part_cap = c->coop_part_cap;
    cs.part_reset = c->coop_part_rows[par ^ 1];  // the previous call's rows
    // the first pass over the rows waits G / 8 x 64 clocks by default: the
    // rows' landing spread grows with the rows every workgroup loads
    // (profiles/r05/delay_sweep_r5s.txt, _r5t.txt: 640x480 (G 200) best at
    // 20-24, 1280x960 (G 240) at 28-32; no wait 13.7 K / 4.93 K aligns/s,
    // 24: 15.7 K / 5.32 K, 32: 15.3 K / 5.41 K; the tracker within noise)
    cs.poll_delay = c->coop_poll_delay >= 0 ? c->coop_poll_delay : G / 8;
    // test hook (YOUTH_ICP_TEST_COOP_STALL=<chunk>[:<launches>]): the
    // context's first coop launches lose one row, so their waits time out
    // after ~20 ms
    cs.stall_chunk = c->coop_stall_once;
    cs.stall_iter = c->coop_stall_iter;
    // a lost iteration-0 row is ended by the product's bound itself (the
    // test of it); a later one by the hook's shorter bound
    cs.spin_max = c->coop_stall_once >= 0 && c->coop_stall_iter != 0 ? 20000u : kCoopSpinMax;
    if (c->coop_stall_once >= 0 && --c->coop_stall_left <= 0) c->coop_stall_once = -1;
    const float4* recs = c->d_rec;
    size_t P = c->P;
    int W = c->W, H = c->H;
    Intr K = c->K;
    FastK F = c->F;
    float thr2 = c->prm.dist_thresh * c->prm.dist_thresh;
    void* args[] = {(void*)&dsrc, (void*)&recs, (void*)&P, (void*)&pm, (void*)&W, (void*)&H,
                    (void*)&K, (void*)&F, (void*)&thr2, (void*)&cs};
    EventPair ep{};
    rc = ev_begin(c, s, &ep, 0);
    if (rc) return rc;
    rc = coop_enqueue(c, s, args, n_pairs * G, npx, tall);
    if (rc) {
        c->coop_par = par;  // nothing ran: the sets and arenas stay as they were
        return rc;
    }
    c->coop_part_rows[par ^ 1] = 0;          // reset by this launch
    c->coop_part_rows[par] = n_pairs * G;    // dirtied by it
    c->last_coop_G = G;
    c->last_coop_px = npx;
    c->lanes = youth_lanes{tile_src ? YOUTH_LANES_COOP_TILE : YOUTH_LANES_COOP, npx * c->coop_threads,
                           c->coop_threads, npx};
    c->has_lanes = true;
    c->lanes_mixed = false;
    return ev_end(c, s, &ep);
}

// k_icp<variant, fast, aligned> by index variant 4 + fast 2 + aligned
typedef void (*IcpKernel)(const int16_t*, const float4*, size_t, PairMap, int, int, Intr, FastK,
                          float, double*, IterState);
static IcpKernel icp_kernel(int var)
{
    static const IcpKernel tab[4 * kVariants] = {
        k_icp<0, false, false>, k_icp<0, false, true>, k_icp<0, true, false>, k_icp<0, true, true>,
        k_icp<1, false, false>, k_icp<1, false, true>, k_icp<1, true, false>, k_icp<1, true, true>,
        k_icp<2, false, false>, k_icp<2, false, true>, k_icp<2, true, false>, k_icp<2, true, true>,
        k_icp<3, false, false>, k_icp<3, false, true>, k_icp<3, true, false>, k_icp<3, true, true>};
    return tab[var & (4 * kVariants - 1)];
}

// All ICP iterations of n_pairs pairs.  *exported is set when the kernel
// also wrote the fp32 4x4 poses to d_T_out (k_icp_coop); otherwise the
// caller runs export_poses.
static int run_iterations(youth_icp_ctx* c, hipStream_t s, const int16_t* dsrc, PairMap pm,
                          int n_pairs, const double* T_init_host, float* d_T_out = nullptr,
                          bool* exported = nullptr, const PrepJob* job = nullptr)
{
    const int iters = c->prm.iters;
    if (exported) *exported = false;
    // k_icp_coop fuses the prep job (one pair of workgroups per target);
    // every other path runs k_prep first
    int npx = 0, G = 0;
    bool coop;
    if (job && job->chain) {
        // a tracker micro-batch runs every pair on the single-pair plan, so
        // each pair's summation tree (and pose) is the one track_frame gives;
        // refused (EINVAL, nothing enqueued) when that grid is not co-resident
        if (iters <= 0 || job->n != n_pairs || n_pairs > kCoopMaxChain ||
            !coop_plan(c, 1, &npx, &G) ||
            (long long)n_pairs * G >
                (long long)c->n_cu *
                    c->coop_bpc[c->coop_threads == 256][variant(c) * 2 + (c->fast ? 1 : 0)][npx])
            return set_error(YOUTH_EINVAL, "track batch: %d pairs do not fit one cooperative grid",
                             n_pairs);
        coop = true;
    } else {
        coop = iters > 0 && (!job || job->n == n_pairs || (!job->wait && job->n == 1)) &&
               coop_plan(c, n_pairs, &npx, &G);
    }
    c->last_coop = coop;
    int rc = ensure_stats(c, iters > 0 ? iters : 1);
    if (rc) return rc;
    const double* dTi = nullptr;
    if (T_init_host) {
        // finite initial poses keep every projected coordinate finite, which
        // the kernels' integer in-range test relies on (xform_project)
        for (size_t i = 0; i < (size_t)n_pairs * 16; ++i)
            if (!std::isfinite(T_init_host[i]))
                return set_error(YOUTH_EINVAL, "T_init: non-finite entry in pair %d",
                                 (int)(i / 16));
        HIP_TRY(hipMemcpyAsync(c->d_Tinit, T_init_host, (size_t)n_pairs * 16 * sizeof(double),
                               hipMemcpyHostToDevice, s));
        dTi = c->d_Tinit;
    }
    if (coop) {
        rc = launch_coop(c, s, dsrc, pm, n_pairs, dTi, d_T_out, npx, G, job);
        if (rc == YOUTH_OK) {
            if (exported) *exported = d_T_out != nullptr;
            c->last_pairs = n_pairs;
            c->last_iters = iters;
            c->last_stream = s;
            return YOUTH_OK;
        }
        if (job && job->chain) return rc;  // a micro-batch has no other kernel path
        // the runtime refused the cooperative launch (nothing was enqueued): this
        // context takes the persistent path from now on
        fprintf(stderr, "youth_icp: cooperative launch refused (%s); using the persistent path\n",
                youth_icp_last_error());
        (void)hipGetLastError();
        c->coop = false;
        c->last_coop = false;
    }
    const bool persistent = c->persistent && iters > 0;
    if (persistent && job) {
        // k_prep also sets the per-call state (k_init folded in)
        const InitArgs ia{dTi,         n_pairs,    c->d_T64, c->d_T32, c->d_status,
                          c->d_epoch,  c->d_arr_it, iters,   c->d_head};
        rc = launch_prep(c, s, job->depth, job->n, job->out0, false, &ia);
        if (rc) return rc;
    } else {
        if (job) {
            rc = launch_prep(c, s, job->depth, job->n, job->out0, false);
            if (rc) return rc;
        }
        hipLaunchKernelGGL(k_init, dim3((n_pairs + 63) / 64), dim3(64), 0, s, dTi, n_pairs,
                           c->d_T64, c->d_T32, c->d_status,
                           persistent ? c->d_epoch : (unsigned*)nullptr,
                           persistent ? c->d_arr_it : (unsigned*)nullptr, iters, c->d_head);
        HIP_TRY(hipGetLastError());
    }
    if (persistent) {
        int chunk = 0;
        const int nb = reduce_geometry(c, n_pairs, &chunk);
        rc = ensure_partials(c, (size_t)nb * n_pairs * kPartStride);
        if (rc) return rc;
        const bool aligned = (reinterpret_cast<uintptr_t>(dsrc) % 8 == 0) && (c->W % 4 == 0) &&
                           c->centred_exact;
        const int var = variant(c) * 4 + (c->fast ? 2 : 0) + (aligned ? 1 : 0);
        const long long items = (long long)iters * n_pairs * nb;
        long long grid = (long long)c->n_cu * c->icp_blocks_per_cu[var] / c->share;
        if (grid > items) grid = items;
        if (grid < 1) grid = 1;
        const IterState is{c->d_T64,  c->d_T32,  c->d_status, c->d_stats,
                           c->d_arr_it, c->d_epoch, c->d_head + kQHead, c->d_head + kQError,
                           d_T_out,   iters,      n_pairs,    nb,
                           chunk,
                           // 8 per-XCD heads from 128 pairs (+0.7 % there), one below (64
                           // pairs: -0.8 % with 8; profiles/r03/ab_queues.txt)
                           c->queues ? c->queues : (n_pairs >= 128 ? kMaxQueues : 1)};
        if (exported) *exported = d_T_out != nullptr;  // k_icp's final solves write d_T_out
        const float thr2 = c->prm.dist_thresh * c->prm.dist_thresh;
        EventPair ep{};
        rc = ev_begin(c, s, &ep, 0);
        if (rc) return rc;
        auto kern = icp_kernel(var);
        hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(kRedThreads), 0, s, dsrc, c->d_rec,
                           c->P, pm, c->W, c->H, c->K, c->F, thr2, c->d_partials, is);
        HIP_TRY(hipGetLastError());
        c->lanes = youth_lanes{YOUTH_LANES_STRIDED, chunk, kRedThreads, 0};
        c->has_lanes = true;
        c->lanes_mixed = false;
        rc = ev_end(c, s, &ep);
        if (rc) return rc;
    } else {
        // arrival counters of the per-iteration fused kernel, re-armed in-kernel
        HIP_TRY(hipMemsetAsync(c->d_arrivals, 0, (size_t)c->max_frames * sizeof(unsigned), s));
        for (int it = 0; it < iters; ++it) {
            int nb = 0;
            rc = launch_reduce(c, s, dsrc, pm, n_pairs, false, &nb, it);  // + fused solve
            if (rc) return rc;
        }
    }
    c->last_pairs = n_pairs;
    c->last_iters = iters;
    c->last_stream = s;
    return YOUTH_OK;
}

static int export_poses(youth_icp_ctx* c, hipStream_t s, int n_pairs, float* d_T_out)
{
    hipLaunchKernelGGL(k_finish, dim3((n_pairs * 16 + 255) / 256), dim3(256), 0, s, c->d_T64,
                       n_pairs, d_T_out, c->d_status, (const unsigned*)(c->d_head + kQError));
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

// FastK of the intrinsics: h = RN(1/y), l = RN((1 - y h) / y) with the
// residual 1 - y h exact (fma) and the quotient rounded once from fp64 (any
// l is safe: k_verify_fastdiv decides whether the pair is used).
static FastK fast_consts(const youth_intrinsics& K)
{
    auto hl = [](float y, float& h, float& l) {
        h = 1.0f / y;
        l = (float)((double)std::fma(-y, h, 1.0f) / (double)y);
    };
    FastK F;
    hl(K.fx, F.hfx, F.lfx);
    hl(K.fy, F.hfy, F.lfy);
    hl(K.depth_scale, F.hds, F.lds);
    return F;
}

// Whether k_icp's aligned pixel loop may form a lane's centred column
// coordinates by additions: ((float)(u & ~3) - cx) + (u & 3) must equal the
// spec's (float)u - cx for every column.  It does when cx is near the frame's
// centre (the difference then keeps cx's ulp); a principal point far to one
// side (e.g. cx = 20.9316 at W = 640: 9 columns) can make the difference
// round, and such intrinsics take the unaligned loop, which converts every
// column (tests/test_gpu_reduce.py::test_off_centre_principal_point).
static bool centred_exact(float cx, int W)
{
    for (int u = 0; u < W; ++u) {
        volatile float a = (float)u - cx;
        volatile float b0 = (float)(u & ~3) - cx;
        volatile float b = b0 + (float)(u & 3);
        if (a != b) return false;
    }
    return true;
}

// Decide the division path for these intrinsics (k_verify_fastdiv).
static int verify_fastdiv(youth_icp_ctx* c)
{
    c->fast = false;
    const char* off = getenv("YOUTH_ICP_NO_FASTDIV");
    if (off && *off && *off != '0') return YOUTH_OK;
    HIP_TRY(hipMemsetAsync(c->d_flag, 0, sizeof(unsigned), c->stream));
    hipLaunchKernelGGL(k_verify_fastdiv, dim3(128, 64), dim3(256), 0, c->stream, c->K, c->F, c->W,
                       c->H, c->d_flag);
    HIP_TRY(hipGetLastError());
    unsigned bad = 1;
    HIP_TRY(hipMemcpyAsync(&bad, c->d_flag, sizeof(unsigned), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->fast = bad == 0;
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

int youth_icp_fastdiv_enabled(youth_icp_ctx* c) { return c && c->fast ? 1 : 0; }

int youth_icp_set_spec(youth_icp_ctx* c, int spec)
{
    if (!c || (spec != YOUTH_SPEC_FMA && spec != YOUTH_SPEC_SURVEY))
        return set_error(YOUTH_EINVAL, "set_spec: bad arguments (%d)", spec);
    const int old = c->spec;
    c->spec = spec;
    return old;
}

int youth_icp_set_reduce(youth_icp_ctx* c, int mode)
{
    if (!c || (mode != YOUTH_REDUCE_EXACT && mode != YOUTH_REDUCE_LANE32))
        return set_error(YOUTH_EINVAL, "set_reduce: bad arguments (%d)", mode);
    const int old = c->reduce;
    c->reduce = mode;
    return old;
}

int youth_icp_get_reduce(const youth_icp_ctx* c)
{
    return c ? c->reduce : set_error(YOUTH_EINVAL, "get_reduce: null context");
}

int youth_icp_get_lanes(const youth_icp_ctx* c, youth_lanes* out)
{
    if (!c || !out) return set_error(YOUTH_EINVAL, "get_lanes: bad arguments");
    if (!c->has_lanes) return set_error(YOUTH_EINVAL, "get_lanes: no align has run");
    if (c->lanes_mixed)
        return set_error(YOUTH_EINVAL, "get_lanes: the last call ran launches of more than one "
                                       "lane partition");
    *out = c->lanes;
    return YOUTH_OK;
}

int youth_icp_set_concurrency(youth_icp_ctx* c, int contexts)
{
    if (!c || contexts < 1 || contexts > YOUTH_ICP_MAX_CONCURRENCY)
        return set_error(YOUTH_EINVAL, "set_concurrency: bad arguments (%d)", contexts);
    const int old = c->share;
    c->share = contexts;
    return old;
}

int youth_icp_get_spec(const youth_icp_ctx* c)
{
    return c ? c->spec : set_error(YOUTH_EINVAL, "get_spec: null context");
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
    if (c->xfer) (void)hipStreamSynchronize(c->xfer);
    for (hipEvent_t e : c->xfer_ev) (void)hipEventDestroy(e);
    for (auto& q : c->trk) {
        if (q.pinned) (void)hipHostFree(q.pinned);
        if (q.res) (void)hipHostFree(q.res);
        if (q.h2d) (void)hipEventDestroy(q.h2d);
        if (q.done) (void)hipEventDestroy(q.done);
        if (q.done_nf) (void)hipEventDestroy(q.done_nf);
    }
    void* bufs[] = {c->d_depth, c->d_rec,   c->d_xyz,      c->d_T64, c->d_T32,   c->d_status,
                    c->d_Tinit, c->d_stats, c->d_partials, c->d_neq, c->d_assoc, c->d_Tout,
                    c->d_flag,  c->d_arrivals, c->d_arr_it, c->d_epoch, c->d_head,
                    c->d_coop,  c->d_status_out, c->d_coop_part};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    if (c->device >= 0 && c->device < 64) {
        // the device's coop ordering must not take a later stream that reuses
        // this handle for the same stream (its work is complete: synchronised
        // above, and every earlier coop launch ran before it)
        CoopOrder& o = g_coop_order[c->device];
        std::lock_guard<std::mutex> lk(o.mu);
        if (o.any && o.last == c->stream) {
            o.any = false;
            o.last = nullptr;
        }
    }
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->xfer) (void)hipStreamDestroy(c->xfer);
    delete c;
}

youth_icp_ctx* youth_icp_create(int device, int W, int H, int max_frames,
                                const youth_intrinsics* K, const youth_icp_params* P)
{
    // W, H <= 16384 and W*H <= 2^26: pixel indices fit the pixel loop's 24-bit
    // multiply and a target frame's records (16 B/px) its 32-bit buffer offsets
    if (W < 3 || H < 3 || W > 16384 || H > 16384 || max_frames < 2 ||
        (long long)W * H > (1LL << 26)) {
        set_error(YOUTH_EINVAL,
                  "youth_icp_create: bad size %dx%d / max_frames %d (need 3 <= W, H <= 16384, "
                  "W*H <= 2^26, max_frames >= 2)",
                  W, H, max_frames);
        return nullptr;
    }
    const int ndev = youth_icp_device_count();
    if (ndev <= 0 || device < 0 || device >= ndev) {
        set_error(YOUTH_ENODEV, "youth_icp_create: no HIP device %d", device);
        return nullptr;
    }
    auto* c = new youth_icp_ctx();
    for (int& d : c->trk_dslot_last) d = -1;
    c->device = device;
    c->W = W;
    c->H = H;
    c->N = W * H;
    c->P = ((size_t)c->N + 4 + 255) / 256 * 256;
    c->max_frames = max_frames;
    const youth_intrinsics Kd = K ? *K : youth_default_intrinsics(W, H);
    c->K = Intr{Kd.fx, Kd.fy, Kd.cx, Kd.cy, Kd.depth_scale};
    c->F = fast_consts(Kd);
    c->centred_exact = centred_exact(Kd.cx, W);
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
    const size_t rec_bytes = c->P * sizeof(float4) * MF;
    if ((e = hipMalloc(&c->d_depth, MF * c->N * sizeof(int16_t))) != hipSuccess)
        return fail("hipMalloc depth", e);
    if ((e = hipMalloc(&c->d_rec, rec_bytes)) != hipSuccess) return fail("hipMalloc rec", e);
    // the pad beyond N of every frame must read as an invalid point (z = 0)
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
    if ((e = hipMalloc(&c->d_flag, 16)) != hipSuccess) return fail("hipMalloc flag", e);
    if ((e = hipMalloc(&c->d_epoch, MF * sizeof(unsigned))) != hipSuccess)
        return fail("hipMalloc epoch", e);
    if ((e = hipMalloc(&c->d_head, kQWords * 4)) != hipSuccess) return fail("hipMalloc head", e);
    if ((e = hipMemset(c->d_head, 0, kQWords * 4)) != hipSuccess) return fail("memset head", e);
    {
        hipDeviceProp_t prop;
        if ((e = hipGetDeviceProperties(&prop, device)) != hipSuccess)
            return fail("hipGetDeviceProperties", e);
        c->n_cu = prop.multiProcessorCount;
        for (int v = 0; v < 4 * kVariants; ++v) {
            int nb = 0;
            if ((e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
                     &nb, (const void*)icp_kernel(v), kRedThreads, 0)) != hipSuccess)
                return fail("occupancy", e);
            c->icp_blocks_per_cu[v] = nb > 0 ? nb : 1;
        }
        const char* np = getenv("YOUTH_ICP_NO_PERSISTENT");
        c->persistent = !(np && *np && *np != '0');
        const char* cth = getenv("YOUTH_ICP_COOP_THREADS");
        if (cth && atoi(cth) == 256) c->coop_threads = 256;
        for (int ti = 0; ti < 2; ++ti)
            for (int v = 0; v < 2 * kVariants; ++v)
                for (int npx = 1; npx <= kCoopMaxPx; ++npx) {
                    const int th = ti ? 256 : 512;
                    int nb = 0;
                    if ((e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
                             &nb, coop_kernel(v >> 1, (v & 1) != 0, th), th, coop_lds(npx, th))) !=
                        hipSuccess)
                        return fail("occupancy coop", e);
                    c->coop_bpc[ti][v][npx] = nb;
                }
        for (int v = 0; v < 2 * kVariants; ++v) {
            int nb = 0;
            const int npx = kTileW * kCoopTileHTall / 512;
            if ((e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
                     &nb, coop_kernel(v >> 1, (v & 1) != 0, 512, true), 512,
                     coop_lds(npx, 512))) != hipSuccess)
                return fail("occupancy coop tall", e);
            c->coop_bpc_tall[v] = nb;
        }
        const char* nc = getenv("YOUTH_ICP_NO_COOP");
        c->coop = !(nc && *nc && *nc != '0');
        const char* cpd = getenv("YOUTH_ICP_COOP_POLL_DELAY");  // tuning knob
        if (cpd && atoi(cpd) >= 0) c->coop_poll_delay = atoi(cpd);
        const char* cpx = getenv("YOUTH_ICP_COOP_PX");
        if (cpx && atoi(cpx) >= 1 && atoi(cpx) <= kCoopMaxPx) c->coop_px = atoi(cpx);
        c->coop_px_env = c->coop_px;
        const char* cl = getenv("YOUTH_ICP_COOP_LAUNCH");
        c->coop_launch = !cl ? 0 : strcmp(cl, "runtime") == 0 ? 1 : strcmp(cl, "plain") == 0 ? 2 : 0;
        const char* tcp = getenv("YOUTH_ICP_TRACK_COPY");
        c->trk_copy_compute = tcp && strcmp(tcp, "compute") == 0;
        c->trk_copy_sdma = tcp && (strcmp(tcp, "sdma") == 0 || c->trk_copy_compute);
        const char* pwg = getenv("YOUTH_ICP_PULL_WG");
        c->trk_pull_wg = pwg && atoi(pwg) > 0 ? std::min(atoi(pwg), 1024) : 0;
        const char* plds = getenv("YOUTH_ICP_PULL_LDS");
        if (plds && atoi(plds) >= 0) c->trk_pull_lds = std::min(atoi(plds), 64 << 10);
        const char* pres = getenv("YOUTH_ICP_PULL_RESERVE_CU");
        if (pres && atoi(pres) >= 0) c->trk_pull_reserve = atoi(pres);
        const char* cpt = getenv("YOUTH_ICP_COPY_THREADS");
        if (cpt && atoi(cpt) >= 0) c->trk_copy_helpers = std::min(atoi(cpt), 15);
        // test hooks (tests/): YOUTH_ICP_TEST_COOP_STALL=<chunk>[:<launches>]
        // makes the context's first <launches> (default 1) cooperative
        // launches lose chunk <chunk>'s iteration-1 row of pair 0, so they
        // time out (the tracker's realign path); YOUTH_ICP_TEST_REFUSE_COOP=1
        // refuses every cooperative launch as the runtime would (the
        // persistent fallback of run_iterations).  Either one is announced on
        // stderr: a stray variable must not pass for a device fault
        const char* cst = getenv("YOUTH_ICP_TEST_COOP_STALL");
        if (cst && atoi(cst) >= 0) {
            c->coop_stall_once = atoi(cst);
            const char* colon = strchr(cst, ':');
            c->coop_stall_left = colon && atoi(colon + 1) > 0 ? atoi(colon + 1) : 1;
            fprintf(stderr, "youth_icp: TEST HOOK YOUTH_ICP_TEST_COOP_STALL=%s active: the first %d "
                            "cooperative launch(es) of this context time out\n",
                    cst, c->coop_stall_left);
        }
        const char* sit = getenv("YOUTH_ICP_TEST_COOP_STALL_ITER");
        if (sit && atoi(sit) >= 0) c->coop_stall_iter = atoi(sit);
        const char* rst = getenv("YOUTH_ICP_TEST_REALIGN_STALL");
        c->realign_stall = rst && *rst && *rst != '0';
        if (c->realign_stall)
            fprintf(stderr, "youth_icp: TEST HOOK YOUTH_ICP_TEST_REALIGN_STALL active: the "
                            "cooperative launch of every youth_icp_track_realign times out\n");
        const char* crf = getenv("YOUTH_ICP_TEST_REFUSE_COOP");
        c->coop_refuse = crf && *crf && *crf != '0';
        if (c->coop_refuse)
            fprintf(stderr, "youth_icp: TEST HOOK YOUTH_ICP_TEST_REFUSE_COOP active: cooperative "
                            "launches of this context are refused\n");
        const char* nqs = getenv("YOUTH_ICP_QUEUES");
        if (nqs && atoi(nqs) >= 1 && atoi(nqs) <= kMaxQueues) c->queues = atoi(nqs);
        const char* pxm = getenv("YOUTH_ICP_PREP_XCD_MAP");
        if (pxm && (*pxm == '1' || *pxm == '2')) c->prep_xcd_map = *pxm - '0';
        const char* cts = getenv("YOUTH_ICP_COOP_TILE_SRC");
        if (cts && *cts == '0') c->coop_tile_src = false;
        const char* cmp = getenv("YOUTH_ICP_COOP_MAX_PAIRS");
        if (cmp && atoi(cmp) >= 0) c->coop_max_pairs = atoi(cmp);
        // spec a7/a8 arithmetic: "survey" (SURVEY §8a literally) or "fma"
        const char* sp = getenv("YOUTH_ICP_SPEC");
        if (sp && strcmp(sp, "survey") == 0) c->spec = kSpecSurvey;
        if (sp && strcmp(sp, "fma") == 0) c->spec = kSpecFma;
        // spec a9 reduction: "lane32" (SURVEY §8a a9 as worded) or "exact"
        const char* rd = getenv("YOUTH_ICP_REDUCE");
        if (rd && strcmp(rd, "lane32") == 0) c->reduce = YOUTH_REDUCE_LANE32;
        if (rd && strcmp(rd, "exact") == 0) c->reduce = YOUTH_REDUCE_EXACT;
    }
    if ((e = hipMalloc(&c->d_coop, 2 * kCoopSetWords * sizeof(unsigned))) != hipSuccess)
        return fail("hipMalloc coop", e);
    if ((e = hipMemset(c->d_coop, 0, 2 * kCoopSetWords * sizeof(unsigned))) != hipSuccess)
        return fail("memset coop", e);
    const size_t arr_bytes = (MF * sizeof(unsigned) + 15) / 16 * 16;
    if ((e = hipMalloc(&c->d_arrivals, arr_bytes)) != hipSuccess)
        return fail("hipMalloc arrivals", e);
    if ((e = hipMemset(c->d_arrivals, 0, arr_bytes)) != hipSuccess)
        return fail("memset arrivals", e);
    if ((e = hipDeviceSynchronize()) != hipSuccess) return fail("sync", e);
    if (ensure_stats(c, c->prm.iters > 0 ? c->prm.iters : 1) != YOUTH_OK ||
        verify_fastdiv(c) != YOUTH_OK) {
        youth_icp_destroy(c);
        return nullptr;
    }
    return c;
}

int youth_icp_align_pairs_device(youth_icp_ctx* c, const int16_t* d_src, const int16_t* d_dst,
                                 int n_pairs, const double* T_init, float* d_T_out,
                                 void* stream)
{
    if (!c || !d_src || !d_dst || n_pairs <= 0 || n_pairs > c->max_frames)
        return set_error(YOUTH_EINVAL, "align_pairs: bad arguments %d", n_pairs);
    int rc = bind_device(c);
    if (rc) return rc;
    hipStream_t s = pick_stream(c, stream);
    // targets -> records [0, n); sources are read straight from d_src
    const PrepJob job{d_dst, n_pairs, 0, true};
    bool exported = false;
    rc = run_iterations(c, s, d_src, PairMap{0, 0}, n_pairs, T_init, d_T_out, &exported, &job);
    if (rc) return rc;
    return exported ? YOUTH_OK : export_poses(c, s, n_pairs, d_T_out);
}

int youth_icp_align_sequence_device(youth_icp_ctx* c, const int16_t* d_frames, int n_frames,
                                    float* d_T_out, void* stream)
{
    if (!c || !d_frames || n_frames < 2 || n_frames - 1 > c->max_frames)
        return set_error(YOUTH_EINVAL, "align_sequence: bad arguments %d", n_frames);
    int rc = bind_device(c);
    if (rc) return rc;
    hipStream_t s = pick_stream(c, stream);
    // every frame but the last is a target: one record set per frame, reused;
    // pair k: source depth frame k+1, target record frame k
    const PrepJob job{d_frames, n_frames - 1, 0, true};
    bool exported = false;
    rc = run_iterations(c, s, d_frames, PairMap{1, 0}, n_frames - 1, nullptr, d_T_out, &exported,
                        &job);
    if (rc) return rc;
    return exported ? YOUTH_OK : export_poses(c, s, n_frames - 1, d_T_out);
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
    unsigned err = 0;
    if (status) {
        HIP_TRY(hipMemcpyAsync(status, c->d_status, (size_t)n * sizeof(int32_t),
                               hipMemcpyDeviceToHost, s));
        // a timed-out launch (either kernel path) marks every pair
        HIP_TRY(hipMemcpyAsync(&err, c->d_head + kQError, sizeof(unsigned),
                               hipMemcpyDeviceToHost, s));
    }
    HIP_TRY(hipStreamSynchronize(s));
    if (status && err)
        for (int i = 0; i < n; ++i) status[i] |= YOUTH_STATUS_TIMEOUT;
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
    c->timing_iter_only = enable == 2;
    for (int k = 0; k < 3; ++k) {
        c->t_ms[k] = 0.0;
        c->t_n[k] = 0;
    }
    return YOUTH_OK;
}

int youth_icp_selftest_projdiv(int device, long long n, unsigned long long seed,
                               long long* bit_mismatches, long long* proj_mismatches)
{
    if (n < 0) return set_error(YOUTH_EINVAL, "selftest_projdiv: n < 0");
    const int ndev = youth_icp_device_count();
    if (ndev <= 0 || device < 0 || device >= ndev)
        return set_error(YOUTH_ENODEV, "selftest_projdiv: no HIP device %d", device);
    HIP_TRY(hipSetDevice(device));
    unsigned long long* d_bad = nullptr;
    HIP_TRY(hipMalloc(&d_bad, 2 * sizeof(unsigned long long)));
    unsigned long long h[2] = {0, 0};
    hipError_t e = hipMemset(d_bad, 0, sizeof(h));
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_selftest_projdiv, dim3(4096), dim3(256), 0, 0,
                           (unsigned long long)n, seed, d_bad);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(h, d_bad, sizeof(h), hipMemcpyDeviceToHost);
    (void)hipFree(d_bad);
    if (e != hipSuccess) return set_error(YOUTH_EHIP, "selftest_projdiv: %s", hipGetErrorString(e));
    if (bit_mismatches) *bit_mismatches = (long long)h[0];
    if (proj_mismatches) *proj_mismatches = (long long)h[1];
    return YOUTH_OK;
}

int youth_icp_selftest_projquot(int device, long long n, unsigned long long seed,
                                long long* quot_mismatches, long long* proj_mismatches,
                                long long* floor_mismatches)
{
    if (n < 0) return set_error(YOUTH_EINVAL, "selftest_projquot: n < 0");
    const int ndev = youth_icp_device_count();
    if (ndev <= 0 || device < 0 || device >= ndev)
        return set_error(YOUTH_ENODEV, "selftest_projquot: no HIP device %d", device);
    HIP_TRY(hipSetDevice(device));
    unsigned long long* d_bad = nullptr;
    HIP_TRY(hipMalloc(&d_bad, 3 * sizeof(unsigned long long)));
    unsigned long long h[3] = {0, 0, 0};
    hipError_t e = hipMemset(d_bad, 0, sizeof(h));
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_selftest_projquot, dim3(4096), dim3(256), 0, 0,
                           (unsigned long long)n, seed, d_bad);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(h, d_bad, sizeof(h), hipMemcpyDeviceToHost);
    (void)hipFree(d_bad);
    if (e != hipSuccess) return set_error(YOUTH_EHIP, "selftest_projquot: %s", hipGetErrorString(e));
    if (quot_mismatches) *quot_mismatches = (long long)h[0];
    if (proj_mismatches) *proj_mismatches = (long long)h[1];
    if (floor_mismatches) *floor_mismatches = (long long)h[2];
    return YOUTH_OK;
}

int youth_icp_selftest_normalize(int device, long long n, unsigned long long seed,
                                 long long* sqrt_mismatches, long long* quot_mismatches,
                                 long long* fast_cases)
{
    if (n < 0) return set_error(YOUTH_EINVAL, "selftest_normalize: n < 0");
    const int ndev = youth_icp_device_count();
    if (ndev <= 0 || device < 0 || device >= ndev)
        return set_error(YOUTH_ENODEV, "selftest_normalize: no HIP device %d", device);
    HIP_TRY(hipSetDevice(device));
    unsigned long long* d_bad = nullptr;
    HIP_TRY(hipMalloc(&d_bad, 3 * sizeof(unsigned long long)));
    unsigned long long h[3] = {0, 0, 0};
    hipError_t e = hipMemset(d_bad, 0, sizeof(h));
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_selftest_normalize, dim3(8192), dim3(256), 0, 0,
                           (unsigned long long)n, seed, d_bad);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(h, d_bad, sizeof(h), hipMemcpyDeviceToHost);
    (void)hipFree(d_bad);
    if (e != hipSuccess)
        return set_error(YOUTH_EHIP, "selftest_normalize: %s", hipGetErrorString(e));
    if (sqrt_mismatches) *sqrt_mismatches = (long long)h[0];
    if (quot_mismatches) *quot_mismatches = (long long)h[1];
    if (fast_cases) *fast_cases = (long long)h[2];
    return YOUTH_OK;
}

int youth_icp_get_sched_stats(youth_icp_ctx* c, unsigned* spins, unsigned* waited_items)
{
    if (!c) return set_error(YOUTH_EINVAL, "get_sched_stats: null context");
    int rc = bind_device(c);
    if (rc) return rc;
    unsigned h[kQWords];
    HIP_TRY(hipMemcpyAsync(h, c->d_head, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (spins) *spins = h[kQSpins];
    if (waited_items) *waited_items = h[kQWaited];
    return YOUTH_OK;
}

int youth_icp_get_plan(youth_icp_ctx* c, int* workgroups_per_pair, int* px_per_lane)
{
    if (!c) return set_error(YOUTH_EINVAL, "get_plan: null context");
    if (workgroups_per_pair) *workgroups_per_pair = c->last_coop ? c->last_coop_G : 0;
    if (px_per_lane) *px_per_lane = c->last_coop ? c->last_coop_px : 0;
    return c->last_coop ? 1 : c->persistent ? 0 : 2;
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
    // no X/Y/Z wanted: the align path's record kernel (k_prep without planes)
    rc = launch_prep(c, s, c->d_depth, n_frames, 0, X || Y || Z);
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
                const float* base = reinterpret_cast<const float*>(c->d_rec + (size_t)f * c->P) +
                                    (k - 2);
                HIP_TRY(hipMemcpy2DAsync(dst, sizeof(float), base, sizeof(float4), sizeof(float),
                                         N, hipMemcpyDeviceToHost, s));
            }
        }
    HIP_TRY(hipStreamSynchronize(s));
    return YOUTH_OK;
}

int youth_icp_reduce_host(youth_icp_ctx* c, const int16_t* src, const int16_t* dst,
                          const float* T12, int32_t* assoc, double* neq)
{
    if (!c || !src || !dst || !T12) return set_error(YOUTH_EINVAL, "reduce_host: bad arguments");
    int rc = bind_device(c);
    if (rc) return rc;
    hipStream_t s = c->stream;
    const size_t N = c->N;
    HIP_TRY(hipMemcpyAsync(c->d_depth, src, N * sizeof(int16_t), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(c->d_depth + N, dst, N * sizeof(int16_t), hipMemcpyHostToDevice, s));
    rc = launch_prep(c, s, c->d_depth + N, 1, 1, false);  // target -> record frame 1
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(c->d_T32, T12, 12 * sizeof(float), hipMemcpyHostToDevice, s));
    int nb = 0;
    rc = launch_reduce(c, s, c->d_depth, PairMap{0, 1}, 1, assoc != nullptr, &nb);
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
// One cached context per device (guarded by that device's mutex), reused while
// the frame size, intrinsics and capacity fit.
static std::mutex g_batch_mu[64];
static youth_icp_ctx* g_batch_ctx[64] = {};

// Pairs per pipelined chunk of the host-buffer batch API (n_pairs: no
// pipelining).  YOUTH_ICP_BATCH_CHUNK overrides (0 disables).
static int batch_chunk(int n_pairs)
{
    if (const char* e = getenv("YOUTH_ICP_BATCH_CHUNK")) {
        const int v = atoi(e);
        return v <= 0 ? n_pairs : std::min(v, n_pairs);
    }
    // 16-pair chunks run the persistent kernel: copy ~ align.  8-pair chunks
    // (cooperative kernel) ran at 34 K on one box and 20-24 K on another, next to
    // the in-flight copies (profiles/r01/hostio_sweep.txt)
    return n_pairs >= 32 ? 16 : n_pairs;
}

// Workspace for an align of n_pairs whichever kernel path it takes
// (cooperative, persistent or per-iteration), so that no hipFree/hipMalloc
// runs while earlier chunks of a pipelined call are in flight.
static int reserve_for(youth_icp_ctx* c, int n_pairs)
{
    int chunk = 0;
    const int nb = reduce_geometry(c, n_pairs, &chunk);
    size_t need = (size_t)nb * n_pairs * kPartStride;
    int npx = 0, G = 0;
    if (coop_plan(c, n_pairs, &npx, &G))
        need = std::max(need, (size_t)2 * n_pairs * G * kPartStride);
    int rc = ensure_partials(c, need);
    if (rc) return rc;
    return ensure_stats(c, c->prm.iters > 0 ? c->prm.iters : 1);
}

// The host batch align of n_pairs pairs on ONE device: H2D of both depth
// stacks, align, poses (and per-pair status, nullable) back into the
// caller's rows.  Batches of >= 32 pairs are pipelined in chunks: chunk k's
// H2D on a transfer stream overlaps the align of chunk k-1 (every chunk has
// its own device frames, so nothing is reused inside one call).  On any error
// both streams are drained before returning, so no copy still reads the
// caller's buffers.  Caller holds g_batch_mu[dev].
static int batch_on_device(int dev, const int16_t* src, const int16_t* dst, int n_pairs, int W,
                           int H, const youth_intrinsics& Kd, int iters, float* T_out,
                           int32_t* status_out, int32_t* assoc_out)
{
    youth_icp_params P = youth_default_params();
    P.iters = iters;
    youth_icp_ctx*& slot = g_batch_ctx[dev];
    youth_icp_ctx* c = slot;
    const bool same = c && c->W == W && c->H == H && c->max_frames >= 2 * n_pairs &&
                      c->K.fx == Kd.fx && c->K.fy == Kd.fy && c->K.cx == Kd.cx &&
                      c->K.cy == Kd.cy && c->K.ds == Kd.depth_scale;
    if (!same) {
        if (c) youth_icp_destroy(c);
        slot = nullptr;
        c = youth_icp_create(dev, W, H, 2 * n_pairs, &Kd, &P);
        if (!c)
            return g_last_error.find("no HIP device") != std::string::npos ? YOUTH_ENODEV
                                                                          : YOUTH_EHIP;
        slot = c;
    }
    c->prm = P;
    int rc = bind_device(c);
    if (rc) return rc;
    hipStream_t s = c->stream;
    if (!c->xfer) HIP_TRY(hipStreamCreateWithFlags(&c->xfer, hipStreamNonBlocking));
    // per-pair status on every call: a timed-out cooperative chunk is realigned below
    if (!c->d_status_out)
        HIP_TRY(hipMalloc(&c->d_status_out, (size_t)c->max_frames * sizeof(int32_t)));
    auto drain = [c, s](int code) {
        (void)hipStreamSynchronize(c->xfer);
        (void)hipStreamSynchronize(s);
        return code;
    };
    const size_t N = c->N;
    int16_t* d_s = c->d_depth;
    int16_t* d_d = c->d_depth + (size_t)n_pairs * N;
    const int chunk = assoc_out ? n_pairs : batch_chunk(n_pairs);
    const int n_chunks = (n_pairs + chunk - 1) / chunk;
    rc = reserve_for(c, chunk);
    if (!rc && n_pairs % chunk) rc = reserve_for(c, n_pairs % chunk);
    if (rc) return rc;
    while ((int)c->xfer_ev.size() < n_chunks) {
        hipEvent_t e;
        HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        c->xfer_ev.push_back(e);
    }
    youth_lanes first_lanes{};
    bool mixed = false;
    for (int k = 0; k < n_chunks; ++k) {
        const size_t p0 = (size_t)k * chunk;
        const int cnt = (int)std::min<size_t>(chunk, n_pairs - p0);
        const size_t bytes = (size_t)cnt * N * sizeof(int16_t);
        hipError_t e = hipMemcpyAsync(d_s + p0 * N, src + p0 * N, bytes, hipMemcpyHostToDevice,
                                      c->xfer);
        if (e == hipSuccess)
            e = hipMemcpyAsync(d_d + p0 * N, dst + p0 * N, bytes, hipMemcpyHostToDevice, c->xfer);
        if (e == hipSuccess) e = hipEventRecord(c->xfer_ev[k], c->xfer);
        if (e == hipSuccess) e = hipStreamWaitEvent(s, c->xfer_ev[k], 0);
        if (e != hipSuccess)
            return drain(set_error(YOUTH_EHIP, "align_batch: %s", hipGetErrorString(e)));
        rc = youth_icp_align_pairs_device(c, d_s + p0 * N, d_d + p0 * N, cnt, nullptr,
                                          c->d_Tout + p0 * 16, s);
        if (rc) return drain(rc);
        // a tail chunk may take another kernel (and lane partition) than the
        // full chunks: youth_icp_get_lanes then reports the call as mixed
        if (k == 0)
            first_lanes = c->lanes;
        else
            mixed |= memcmp(&first_lanes, &c->lanes, sizeof(youth_lanes)) != 0;
        hipLaunchKernelGGL(k_status_out, dim3((cnt + 255) / 256), dim3(256), 0, s,
                           c->d_status, cnt, (const unsigned*)(c->d_head + kQError),
                           c->d_status_out + p0);
        if ((e = hipGetLastError()) != hipSuccess)
            return drain(set_error(YOUTH_EHIP, "align_batch: %s", hipGetErrorString(e)));
    }
    // A chunk of <= 16 pairs is one cooperative launch sized to an idle
    // device; on a GPU shared with other processes its grid may not be
    // co-resident, and it then times out (kCoopSpinMax polls, ~50 ms) with
    // partly iterated poses.  Such a chunk is aligned again, synchronously, on
    // the persistent k_prep + k_icp, which waits only on running workgroups:
    // the same poses up to fp64 summation order (its depth frames are still
    // on the device).  The caller never receives a TIMEOUT pose from here.
    {
        std::vector<int32_t> st((size_t)n_pairs);
        hipError_t e = hipMemcpyAsync(st.data(), c->d_status_out, (size_t)n_pairs * sizeof(int32_t),
                                      hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) return drain(set_error(YOUTH_EHIP, "align_batch: %s", hipGetErrorString(e)));
        for (int k = 0; k < n_chunks; ++k) {
            const size_t p0 = (size_t)k * chunk;
            const int cnt = (int)std::min<size_t>(chunk, n_pairs - p0);
            bool to = false;
            for (int i = 0; i < cnt; ++i) to |= (st[p0 + i] & YOUTH_STATUS_TIMEOUT) != 0;
            if (!to) continue;
            fprintf(stderr, "youth_icp: align_batch: a cooperative launch of %d pair(s) timed out "
                            "(GPU shared with another process?); realigned on the persistent kernel\n",
                    cnt);
            const bool coop_was = c->coop;
            c->coop = false;
            rc = youth_icp_align_pairs_device(c, d_s + p0 * N, d_d + p0 * N, cnt, nullptr,
                                              c->d_Tout + p0 * 16, s);
            c->coop = coop_was;
            if (rc) return drain(rc);
            ++c->batch_realigned;
            mixed = true;  // this chunk's lane partition is the persistent kernel's
            hipLaunchKernelGGL(k_status_out, dim3((cnt + 255) / 256), dim3(256), 0, s,
                               c->d_status, cnt, (const unsigned*)(c->d_head + kQError),
                               c->d_status_out + p0);
            if ((e = hipGetLastError()) != hipSuccess)
                return drain(set_error(YOUTH_EHIP, "align_batch: %s", hipGetErrorString(e)));
        }
    }
    if (assoc_out) {
        int nb = 0;
        const youth_lanes align_lanes = c->lanes;  // youth_icp_get_lanes reports the align's
        rc = launch_reduce(c, s, d_s, PairMap{0, 0}, n_pairs, true, &nb);
        c->lanes = align_lanes;
        if (rc) return drain(rc);
        hipError_t e = hipMemcpyAsync(assoc_out, c->d_assoc, (size_t)n_pairs * N * sizeof(int32_t),
                                      hipMemcpyDeviceToHost, s);
        if (e != hipSuccess)
            return drain(set_error(YOUTH_EHIP, "align_batch: %s", hipGetErrorString(e)));
    }
    c->lanes_mixed = mixed;
    hipError_t e = hipMemcpyAsync(T_out, c->d_Tout, (size_t)n_pairs * 16 * sizeof(float),
                                  hipMemcpyDeviceToHost, s);
    if (e == hipSuccess && status_out)
        e = hipMemcpyAsync(status_out, c->d_status_out, (size_t)n_pairs * sizeof(int32_t),
                           hipMemcpyDeviceToHost, s);
    if (e != hipSuccess) return drain(set_error(YOUTH_EHIP, "align_batch: %s", hipGetErrorString(e)));
    HIP_TRY(hipStreamSynchronize(s));
    return YOUTH_OK;
}

int youth_icp_align_batch(const int16_t* src, const int16_t* dst, int n_pairs, int W, int H,
                          const youth_intrinsics* K, int iters, float* T_out,
                          int32_t* assoc_out)
{
    if (!src || !dst || n_pairs <= 0 || W < 3 || H < 3 || iters < 0 || !T_out)
        return set_error(YOUTH_EINVAL, "align_batch: bad arguments %d", n_pairs);
    std::lock_guard<std::mutex> lk(g_batch_mu[0]);
    const youth_intrinsics Kd = K ? *K : youth_default_intrinsics(W, H);
    return batch_on_device(0, src, dst, n_pairs, W, H, Kd, iters, T_out, nullptr, assoc_out);
}

// Contiguous shard [first, first + count) of n pairs for part r of k (the
// first n % k parts get one more), as youth_dist.pair_range on the bench side.
static void shard_range(int n, int k, int r, int* first, int* count)
{
    const int q = n / k, m = n % k;
    *first = r * q + std::min(r, m);
    *count = q + (r < m ? 1 : 0);
}

int youth_icp_shard_range(int n_pairs, int n_parts, int part, int* first, int* count)
{
    if (n_pairs < 0 || n_parts <= 0 || part < 0 || part >= n_parts || !first || !count)
        return set_error(YOUTH_EINVAL, "shard_range: bad arguments");
    shard_range(n_pairs, n_parts, part, first, count);
    return YOUTH_OK;
}

int youth_icp_align_batch_multi(const int16_t* src, const int16_t* dst, int n_pairs, int W,
                                int H, const youth_intrinsics* K, int iters, const int* devices,
                                int n_devices, float* T_out, int32_t* status_out)
{
    if (!src || !dst || n_pairs <= 0 || W < 3 || H < 3 || iters < 0 || !T_out)
        return set_error(YOUTH_EINVAL, "align_batch_multi: bad arguments %d", n_pairs);
    const int ndev = youth_icp_device_count();
    if (ndev <= 0) return set_error(YOUTH_ENODEV, "align_batch_multi: no HIP device");
    std::vector<int> devs;
    if (devices && n_devices > 0) {
        for (int i = 0; i < n_devices; ++i) {
            if (devices[i] < 0 || devices[i] >= ndev || devices[i] >= 64)
                return set_error(YOUTH_EINVAL, "align_batch_multi: no HIP device %d", devices[i]);
            if (std::find(devs.begin(), devs.end(), devices[i]) != devs.end())
                return set_error(YOUTH_EINVAL, "align_batch_multi: device %d listed twice",
                                 devices[i]);
            devs.push_back(devices[i]);
        }
    } else {
        for (int d = 0; d < std::min(ndev, 64); ++d) devs.push_back(d);
    }
    const int parts = std::min((int)devs.size(), n_pairs);
    const youth_intrinsics Kd = K ? *K : youth_default_intrinsics(W, H);
    const size_t N = (size_t)W * H;
    std::vector<int> rcs(parts, YOUTH_OK);
    std::vector<std::string> errs(parts);
    auto work = [&](int r) {
        int first = 0, cnt = 0;
        shard_range(n_pairs, parts, r, &first, &cnt);
        std::lock_guard<std::mutex> lk(g_batch_mu[devs[r]]);
        rcs[r] = batch_on_device(devs[r], src + (size_t)first * N, dst + (size_t)first * N, cnt, W,
                                 H, Kd, iters, T_out + (size_t)first * 16,
                                 status_out ? status_out + first : nullptr, nullptr);
        if (rcs[r]) errs[r] = g_last_error;  // thread-local: carried to the caller below
    };
    // one host thread per device; shard 0 runs on the calling thread
    std::vector<std::thread> th;
    for (int r = 1; r < parts; ++r) th.emplace_back(work, r);
    work(0);
    for (auto& t : th) t.join();
    for (int r = 0; r < parts; ++r)
        if (rcs[r]) {
            g_last_error = "device " + std::to_string(devs[r]) + ": " + errs[r];
            return rcs[r];
        }
    return YOUTH_OK;
}

// ------------------------------------------------------ frame tracking --
// Lazily: the transfer stream and the ring's events.  The pinned staging
// frame and result slot of a ring entry are allocated when a submission first
// uses that entry (track_entry_pinned), so a context that keeps at most two
// frames in flight (the SLAM worker) pins two frames, not the ring's 16
// (16 x W x H x 2 bytes is 512 MB at 4096 x 4096).
static int ensure_track(youth_icp_ctx* c)
{
    if (c->trk[kTrackDepth - 1].done_nf) return YOUTH_OK;
    if (!c->xfer) HIP_TRY(hipStreamCreateWithFlags(&c->xfer, hipStreamNonBlocking));
    for (auto& q : c->trk) {
        if (!q.h2d) HIP_TRY(hipEventCreateWithFlags(&q.h2d, hipEventDisableTiming));
        if (!q.done) HIP_TRY(hipEventCreateWithFlags(&q.done, hipEventDisableTiming));
        if (!q.done_nf)
            HIP_TRY(hipEventCreateWithFlags(&q.done_nf,
                                            hipEventDisableTiming | hipEventDisableSystemFence));
    }
    return YOUTH_OK;
}

// The ring holds trk_cap entries and grows only when a submission would put
// more than trk_cap frames in flight: it is rotated so the oldest in-flight
// entry is entry 0 (indices in trk_dslot_last follow), then extended, so the
// in-flight entries stay consecutive modulo the new size.
static void track_grow(youth_icp_ctx* c, int need)
{
    if (need <= c->trk_cap) return;
    const int cap = c->trk_cap, h = c->trk_head;
    if (h) {
        youth_icp_ctx::TrackSlot tmp[kTrackDepth];
        for (int i = 0; i < cap; ++i) tmp[i] = c->trk[(h + i) % cap];
        for (int i = 0; i < cap; ++i) c->trk[i] = tmp[i];
        for (int& d : c->trk_dslot_last)
            if (d >= 0) d = (d - h + cap) % cap;
        c->trk_head = 0;
    }
    c->trk_cap = std::min(kTrackDepth, need);
}

static int track_entry_pinned(youth_icp_ctx* c, int e, bool staging)
{
    auto& q = c->trk[e];
    if (staging && !q.pinned)
        HIP_TRY(hipHostMalloc((void**)&q.pinned, (size_t)c->N * sizeof(int16_t),
                              hipHostMallocDefault));
    if (!q.res) HIP_TRY(hipHostMalloc((void**)&q.res, 17 * sizeof(double), hipHostMallocCoherent));
    return YOUTH_OK;
}

// Depth slots of the tracker (device staging of host frames): two halves of
// B slots (B = the largest micro-batch the context has room for: a launch
// takes consecutive slots of one half, the other half stays with the launch
// before), or 2 (one frame per launch).  Record slots: B + 1 (a micro-batch
// preps its B new frames beside the reference), at least 2.
static int trk_half(const youth_icp_ctx* c)
{
    return std::max(1, std::min(kCoopMaxChain, c->max_frames / 2));
}
static int trk_depth_slots(const youth_icp_ctx* c) { return 2 * trk_half(c); }
static int trk_record_slots(const youth_icp_ctx* c)
{
    return std::max(2, std::min(kCoopMaxChain + 1, c->max_frames));
}

// Whether m consecutive frames can be aligned as one k_icp_coop micro-batch:
// every pair on the single-pair plan (bit-identical to track_frame), the m
// grids co-resident, room for the slots.
static bool trk_chain_fits(const youth_icp_ctx* c, int m)
{
    if (m < 2 || m > kCoopMaxChain || m > trk_half(c) || trk_record_slots(c) < m + 1 ||
        c->prm.iters <= 0 || c->coop_refuse)
        return false;
    int npx = 0, G = 0;
    if (!coop_plan(c, 1, &npx, &G)) return false;
    return (long long)m * G <=
           (long long)c->n_cu *
               c->coop_bpc[c->coop_threads == 256][variant(c) * 2 + (c->fast ? 1 : 0)][npx];
}

// m consecutive host frames (m = 1, or a micro-batch that trk_chain_fits):
// staged into m consecutive depth slots not read by the previous launch,
// H2D on the transfer stream (after the last launch that read those slots),
// then ONE launch on the context stream: prep only (no reference yet), the
// single-pair align with the fused prep of the new frame, or the chained
// micro-batch (pair i aligns frame i to frame i-1, frame -1 = the
// reference).  One completion event for the launch, shared by its entries.
// frames (nullable): the m frames are the caller's page-locked buffers,
// copied H2D in place (no staging copy; youth_icp_track_submit_pinned).
// Page-locked buffers handed out by youth_icp_host_alloc, by base address:
// k_pull_frames reads a caller's frame in place only when it lies inside one
// of them (youth_icp_track_submit_pinned); any other pointer goes through
// hipMemcpyAsync, so a pageable buffer passed by mistake is copied by the
// runtime instead of faulting the GPU.
static std::mutex g_host_mu;
static std::map<uintptr_t, size_t> g_host_bufs;  // base -> bytes

static bool host_alloc_covers(const int16_t* p, size_t values)
{
    const uintptr_t a = (uintptr_t)p;
    std::lock_guard<std::mutex> lk(g_host_mu);
    auto it = g_host_bufs.upper_bound(a);
    if (it == g_host_bufs.begin()) return false;
    --it;
    return a >= it->first && a + values * sizeof(int16_t) <= it->first + it->second;
}

// the SLAM module's event trace (slam_api.cpp, youth_slam_trace_enable):
// steps inside a submission, YOUTH_SLAM_EV_SUBMIT_STEP.  Weak: tools that
// compile this file without slam_api.cpp (tools/coopbench ...) record nothing.
extern "C" __attribute__((weak)) void youth_slam_trace_hook(int kind, int arg);
static inline void trace_step(int step)
{
    if (youth_slam_trace_hook) youth_slam_trace_hook(YOUTH_SLAM_EV_SUBMIT_STEP, step);
}

static int track_submit_frames(youth_icp_ctx* c, const int16_t* depth, int m,
                               const double* T_init, const int16_t* const* frames = nullptr)
{
    hipStream_t s = c->stream;
    const size_t N = c->N;
    const int nds = trk_depth_slots(c), nrs = trk_record_slots(c);
    // depth slots: the half the previous launch did not use
    const int half = nds / 2;
    const int d0 = c->trk_prev_d0 >= half || c->trk_prev_d0 < 0 ? 0 : half;
    // record slots for the new frames: the first m that are not the reference
    const int ref = c->track_ref;
    int rs[kCoopMaxChain] = {};
    for (int r = 0, k = 0; r < nrs && k < m; ++r)
        if (r != ref) rs[k++] = r;
    int qi[kCoopMaxChain];
    track_grow(c, c->trk_n + m);
    for (int i = 0; i < m; ++i) {
        qi[i] = (c->trk_head + c->trk_n + i) % c->trk_cap;
        const int rc = track_entry_pinned(c, qi[i], !frames);  // before anything is enqueued
        if (rc) return rc;
    }
    trace_step(1);
    auto& ql = c->trk[qi[m - 1]];
    // the caller's buffers are free on return: copy into the entries' pinned
    // staging, then H2D after the last launch that read these depth slots
    // the copies' stream: the transfer stream (overlaps the launch before),
    // or with YOUTH_ICP_TRACK_COPY=compute the launch stream itself (A/B)
    hipStream_t xs = c->trk_copy_compute ? s : c->xfer;
    if (!frames) {
        const size_t fb = N * sizeof(int16_t);
        if (c->trk_copy_helpers > 0 && (size_t)m * fb >= c->trk_copy_min) {
            if (!c->copy_pool) c->copy_pool.reset(new youth::HostCopyPool(c->trk_copy_helpers));
            youth::HostCopyPool::Seg seg[kCoopMaxChain];
            for (int i = 0; i < m; ++i) seg[i] = {c->trk[qi[i]].pinned, depth + (size_t)i * N, fb};
            // ~4 pieces per copier per micro-batch: late wake-ups even out
            const size_t piece = (size_t)m * fb / (4 * (c->trk_copy_helpers + 1));
            c->copy_pool->run(seg, m, std::max(piece, (size_t)64 << 10));
        } else {
            for (int i = 0; i < m; ++i) memcpy(c->trk[qi[i]].pinned, depth + (size_t)i * N, fb);
        }
    }
    hipEvent_t waited[kCoopMaxChain];
    int nw = 0;
    for (int i = 0; i < m; ++i) {
        const int last = c->trk_dslot_last[d0 + i];
        if (last < 0 || xs == s) continue;
        // the slots of one earlier launch share its event: wait once per event
        hipEvent_t ev = c->trk[last].ev;
        bool dup = false;
        for (int k = 0; k < nw; ++k) dup |= waited[k] == ev;
        if (!dup) {
            HIP_TRY(hipStreamWaitEvent(xs, ev, 0));
            waited[nw++] = ev;
        }
    }
    trace_step(2);
    // the caller's frames are pulled in place only when youth_icp_host_alloc
    // made them (the staging buffers always are page-locked)
    bool pull = !c->trk_copy_sdma;
    for (int i = 0; pull && frames && i < m; ++i) pull = host_alloc_covers(frames[i], N);
    if (pull) {
        FramePtrs fp{};
        for (int i = 0; i < m; ++i) fp.src[i] = frames ? frames[i] : c->trk[qi[i]].pinned;
        // ~16 workgroups per launch: 2 per frame in a micro-batch of 8 (one
        // per free CU, profiles/r05/slam_pull_reserve_r5s.txt), 16 for a
        // single frame (its latency)
        const int wg = c->trk_pull_wg > 0 ? c->trk_pull_wg : std::max(2, 16 / m);
        // its LDS reservation (unused) keeps a workgroup off the CUs where a
        // micro-batch grid's workgroup sits (~143 KB of 160 at 640x480), so
        // the pull runs on the CUs the plan left free instead of slowing the
        // grid's barriers (youth_icp_track_set_batch)
        hipLaunchKernelGGL(k_pull_frames, dim3(wg, m), dim3(64), (unsigned)c->trk_pull_lds, xs, fp,
                           c->d_depth + (size_t)d0 * N, (int)N, m);
        HIP_TRY(hipGetLastError());
    } else {
        for (int i = 0; i < m; ++i)
            HIP_TRY(hipMemcpyAsync(c->d_depth + (size_t)(d0 + i) * N,
                                   frames ? frames[i] : c->trk[qi[i]].pinned, N * sizeof(int16_t),
                                   hipMemcpyHostToDevice, xs));
    }
    trace_step(3);
    if (xs != s) {
        HIP_TRY(hipEventRecord(ql.h2d, xs));
        HIP_TRY(hipStreamWaitEvent(s, ql.h2d, 0));
    }
    trace_step(4);
    const int16_t* dsrc = c->d_depth + (size_t)d0 * N;
    int rc = YOUTH_OK;
    bool kernel_result = false;  // k_icp_coop stored the result(s) to host memory
    if (ref < 0) {
        // first frame of a sequence: prep only (m == 1)
        rc = launch_prep(c, s, dsrc, 1, rs[0], false);
    } else if (m == 1) {
        // source: the new frame's depth; target: ref's records; the new frame
        // is prepped beside the iterations as the next reference.  k_icp_coop
        // writes the result into the pinned slot itself; any other kernel path
        // copies it
        const PrepJob job{dsrc, 1, rs[0], false};
        c->coop_res_host = ql.res;
        rc = run_iterations(c, s, dsrc, PairMap{0, ref}, 1, T_init, nullptr, nullptr, &job);
        c->coop_res_host = nullptr;
        kernel_result = c->last_coop;
        if (rc == YOUTH_OK && !c->last_coop) {
            HIP_TRY(hipMemcpyAsync(ql.res, c->d_T64, 16 * sizeof(double), hipMemcpyDeviceToHost, s));
            HIP_TRY(hipMemcpyAsync(ql.res + 16, c->d_status, sizeof(int32_t),
                                   hipMemcpyDeviceToHost, s));
        }
    } else {
        PrepJob job{dsrc, m, 0, false};
        job.chain = true;
        for (int i = 0; i < m; ++i) {
            job.tgt_slot[i] = i == 0 ? ref : rs[i - 1];
            job.prep_slot[i] = rs[i];
            job.res[i] = c->trk[qi[i]].res;
        }
        rc = run_iterations(c, s, dsrc, PairMap{0, 0}, m, nullptr, nullptr, nullptr, &job);
        kernel_result = true;
        if (rc == YOUTH_OK) ++c->trk_chained;
    }
    trace_step(5);
    if (rc) {
        // nothing of these frames is kept; wait for what was enqueued so the
        // staging buffers and the slots are not in use by dropped frames
        (void)hipStreamSynchronize(s);
        (void)hipStreamSynchronize(c->xfer);
        return rc;
    }
    // no result to publish (first frame) or k_icp_coop stored it to host
    // memory itself: no system-scope fence; else the copies' result needs it
    hipEvent_t ev = (ref < 0 || kernel_result) ? ql.done_nf : ql.done;
    HIP_TRY(hipEventRecord(ev, s));
    for (int i = 0; i < m; ++i) {
        auto& q = c->trk[qi[i]];
        q.ev = ev;
        q.has_ref = (i > 0 || ref >= 0) ? 1 : 0;
        c->trk_dslot_last[d0 + i] = qi[m - 1];
    }
    c->trk_prev_d0 = d0;
    c->track_ref = rs[m - 1];
    c->trk_n += m;
    return YOUTH_OK;
}

int youth_icp_track_submit(youth_icp_ctx* c, const int16_t* depth, const double* T_init)
{
    if (!c || !depth) return set_error(YOUTH_EINVAL, "track_submit: bad arguments");
    if (c->trk_n >= kTrackDepth)
        return set_error(YOUTH_EINVAL, "track_submit: %d frames in flight (collect one first)",
                         kTrackDepth);
    if (T_init)
        for (int i = 0; i < 16; ++i)
            if (!std::isfinite(T_init[i]))
                return set_error(YOUTH_EINVAL, "T_init: non-finite entry in pair 0");
    int rc = bind_device(c);
    if (rc) return rc;
    rc = ensure_track(c);
    if (rc) return rc;
    return track_submit_frames(c, depth, 1, T_init);
}

// youth_icp_track_submit_batch (depth: n_frames consecutive frames, staged)
// and youth_icp_track_submit_pinned (frames: the caller's page-locked buffers).
static int track_submit_many(youth_icp_ctx* c, const int16_t* depth,
                             const int16_t* const* frames, int n_frames)
{
    if (c->trk_n + n_frames > kTrackDepth)
        return set_error(YOUTH_EINVAL, "track_submit_batch: %d + %d frames in flight (max %d)",
                         c->trk_n, n_frames, kTrackDepth);
    int rc = bind_device(c);
    if (rc) return rc;
    rc = ensure_track(c);
    if (rc) return rc;
    const size_t N = c->N;
    int done = 0;
    if (c->track_ref < 0) {  // no reference yet: the first frame is only prepped
        rc = track_submit_frames(c, depth, 1, nullptr, frames);
        if (rc) return rc;
        done = 1;
    }
    // the rest in the longest chains that fit, else one launch per frame
    while (done < n_frames) {
        int m = n_frames - done;
        while (m > 1 && !trk_chain_fits(c, m)) --m;
        rc = track_submit_frames(c, frames ? nullptr : depth + (size_t)done * N, m, nullptr,
                                 frames ? frames + done : nullptr);
        if (rc) return rc;
        if (m > 1) c->trk_chained_frames += m;
        done += m;
    }
    return YOUTH_OK;
}

int youth_icp_track_submit_batch(youth_icp_ctx* c, const int16_t* depth, int n_frames)
{
    if (!c || !depth || n_frames < 1 || n_frames > YOUTH_TRACK_MAX_BATCH)
        return set_error(YOUTH_EINVAL, "track_submit_batch: bad arguments (%d frames)", n_frames);
    return track_submit_many(c, depth, nullptr, n_frames);
}

int youth_icp_track_submit_pinned(youth_icp_ctx* c, const int16_t* const* frames, int n_frames)
{
    if (!c || !frames || n_frames < 1 || n_frames > YOUTH_TRACK_MAX_BATCH)
        return set_error(YOUTH_EINVAL, "track_submit_pinned: bad arguments (%d frames)", n_frames);
    for (int i = 0; i < n_frames; ++i)
        if (!frames[i]) return set_error(YOUTH_EINVAL, "track_submit_pinned: frame %d is null", i);
    return track_submit_many(c, nullptr, frames, n_frames);
}

int16_t* youth_icp_host_alloc(size_t values)
{
    if (!values) return nullptr;
    int16_t* p = nullptr;
    if (hipHostMalloc((void**)&p, values * sizeof(int16_t), hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    std::lock_guard<std::mutex> lk(g_host_mu);
    g_host_bufs[(uintptr_t)p] = values * sizeof(int16_t);
    return p;
}

void youth_icp_host_free(int16_t* p)
{
    if (!p) return;
    {
        std::lock_guard<std::mutex> lk(g_host_mu);
        g_host_bufs.erase((uintptr_t)p);
    }
    (void)hipHostFree(p);
}

// A collect waits for its frame by polling the event for up to 2 ms before
// the runtime's blocking wait: a sleeping wait's wake-up cost a backlogged
// SLAM worker up to ~0.6 ms per micro-batch (profiles/r04/slamtrace_r4k.txt).
// YOUTH_ICP_TRACK_WAIT=sync keeps the blocking wait only (A/B).
static hipError_t track_wait(hipEvent_t ev)
{
    static const bool poll = [] {
        const char* e = getenv("YOUTH_ICP_TRACK_WAIT");
        return !(e && strcmp(e, "sync") == 0);
    }();
    if (poll) {
        const auto t0 = std::chrono::steady_clock::now();
        for (;;) {
            const hipError_t r = hipEventQuery(ev);
            if (r != hipErrorNotReady) return r;
            if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) break;
        }
    }
    return hipEventSynchronize(ev);
}

int youth_icp_track_collect(youth_icp_ctx* c, double* T_rel, int* has_ref)
{
    if (!c || !T_rel) return set_error(YOUTH_EINVAL, "track_collect: bad arguments");
    if (c->trk_n == 0) return set_error(YOUTH_EINVAL, "track_collect: no frame in flight");
    int rc = bind_device(c);
    if (rc) return rc;
    auto& q = c->trk[c->trk_head];
    c->trk_head = (c->trk_head + 1) % c->trk_cap;
    --c->trk_n;
    HIP_TRY(track_wait(q.ev));
    if (has_ref) *has_ref = q.has_ref;
    if (!q.has_ref) {
        for (int i = 0; i < 16; ++i) T_rel[i] = (i % 5) == 0 ? 1.0 : 0.0;
        return 0;
    }
    for (int i = 0; i < 12; ++i) T_rel[i] = q.res[i];
    T_rel[12] = 0.0;
    T_rel[13] = 0.0;
    T_rel[14] = 0.0;
    T_rel[15] = 1.0;
    int32_t st;
    memcpy(&st, q.res + 16, sizeof(st));
    return st;
}

int youth_icp_track_pending(const youth_icp_ctx* c)
{
    return c ? c->trk_n : 0;
}

// A tracker align that came back with YOUTH_STATUS_TIMEOUT (its cooperative
// grid was not co-resident: another process held CUs, or the test hook) is
// aligned again here from host copies of its two frames, synchronously.
// Everything the tracker has enqueued finishes first, so the depth slots
// 0 / 1 and a record slot other than the reference's are free to use, and
// the tracker continues afterwards as if nothing had happened (its reference
// records are untouched; a timed-out launch still preps every tile of its
// frames, because its workgroups prep before they wait).
//   1. the context's own single-pair plan: the cooperative kernel preps the
//      target and aligns, with the npx / G / tile mapping the tracker's
//      single-frame and chained launches use, so a successful retry gives the
//      pose the undisturbed launch would have, bit for bit;
//   2. if that times out too, the persistent k_prep + k_icp, which waits only
//      on workgroups that are running (no co-residency assumption): the same
//      pose up to fp64 summation order (~1e-16 relative).
int youth_icp_track_realign(youth_icp_ctx* c, const int16_t* ref_depth, const int16_t* depth,
                            const double* T_init, double* T_rel)
{
    if (!c || !ref_depth || !depth || !T_rel)
        return set_error(YOUTH_EINVAL, "track_realign: bad arguments");
    if (T_init)
        for (int i = 0; i < 16; ++i)
            if (!std::isfinite(T_init[i]))
                return set_error(YOUTH_EINVAL, "T_init: non-finite entry in pair 0");
    int rc = bind_device(c);
    if (rc) return rc;
    hipStream_t s = c->stream;
    HIP_TRY(hipStreamSynchronize(s));
    if (c->xfer) HIP_TRY(hipStreamSynchronize(c->xfer));
    const size_t N = c->N;
    const int rslot = c->track_ref == 0 ? 1 : 0;
    HIP_TRY(hipMemcpyAsync(c->d_depth, depth, N * sizeof(int16_t), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(c->d_depth + N, ref_depth, N * sizeof(int16_t), hipMemcpyHostToDevice, s));
    const PrepJob job{c->d_depth + N, 1, rslot, true};
    c->coop_res_host = nullptr;
    int32_t st = YOUTH_STATUS_TIMEOUT;
    for (int attempt = 0; attempt < 2 && (st & YOUTH_STATUS_TIMEOUT); ++attempt) {
        const bool coop_was = c->coop;
        if (attempt == 1) c->coop = false;  // the persistent kernel
        if (attempt == 0 && c->realign_stall) {  // test hook: this coop launch loses a row
            c->coop_stall_once = 0;
            c->coop_stall_left = 1;
        }
        rc = run_iterations(c, s, c->d_depth, PairMap{0, rslot}, 1, T_init, nullptr, nullptr, &job);
        const bool ran_coop = c->last_coop;
        if (attempt == 1) c->coop = coop_was;
        if (rc) return rc;
        double T[16];
        unsigned err = 0;
        HIP_TRY(hipMemcpyAsync(T, c->d_T64, sizeof(T), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(&st, c->d_status, sizeof(st), hipMemcpyDeviceToHost, s));
        if (!ran_coop)  // the persistent kernel's spin bound lands in the queue's error word
            HIP_TRY(hipMemcpyAsync(&err, c->d_head + kQError, sizeof(err), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        if (err) st |= YOUTH_STATUS_TIMEOUT;
        for (int i = 0; i < 12; ++i) T_rel[i] = T[i];
        T_rel[12] = T_rel[13] = T_rel[14] = 0.0;
        T_rel[15] = 1.0;
        if (!(st & YOUTH_STATUS_TIMEOUT)) ++c->trk_realigned[ran_coop ? 0 : 1];
        // a refused cooperative launch already ran the persistent path
        if (!ran_coop) break;
    }
    if (st & YOUTH_STATUS_TIMEOUT) ++c->trk_realigned[2];
    return st;
}

long long youth_icp_track_realigned(const youth_icp_ctx* c, long long* persistent, long long* failed)
{
    if (persistent) *persistent = c ? c->trk_realigned[1] : 0;
    if (failed) *failed = c ? c->trk_realigned[2] : 0;
    return c ? c->trk_realigned[0] : 0;
}

int youth_icp_track_host_sequence(youth_icp_ctx* c, const int16_t* frames, int n_frames,
                                  double* T_rel, int32_t* status)
{
    if (!c || !frames || n_frames < 0 || !T_rel)
        return set_error(YOUTH_EINVAL, "track_host_sequence: bad arguments");
    if (c->trk_n) return set_error(YOUTH_EINVAL, "track_host_sequence: submitted frames not collected");
    const size_t N = c->N;
    int written = 0, collected = 0;
    auto collect = [&]() -> int {
        double T[16];
        int has = 0;
        int st = youth_icp_track_collect(c, T, &has);
        const int f = collected++;  // sequence index of the collected frame
        if (st < 0) return st;
        // a timed-out align is aligned again against the frame before it
        // (frame 0's reference came from an earlier call: its status keeps
        // the TIMEOUT bit)
        if (has && (st & YOUTH_STATUS_TIMEOUT) && f >= 1) {
            const int st2 = youth_icp_track_realign(c, frames + (size_t)(f - 1) * N,
                                                    frames + (size_t)f * N, nullptr, T);
            if (st2 < 0) return st2;
            st = st2;
        }
        if (has) {
            memcpy(T_rel + (size_t)written * 16, T, sizeof(T));
            if (status) status[written] = st;
            ++written;
        }
        return YOUTH_OK;
    };
    // batch: frames per submission (1: one launch per frame, as the SLAM
    // worker at camera rate; 2: micro-batches of two frames when they fit one
    // cooperative grid, the pose of each frame bit-identical either way)
    const int batch = c->trk_batch;
    for (int f = 0; f < n_frames;) {
        const int m = std::min(batch, n_frames - f);
        // keep two submissions in flight: two frames, or two micro-batches
        while (c->trk_n + m > (batch > 1 ? 2 * batch : 2)) {
            const int rc = collect();
            if (rc) {
                while (c->trk_n) (void)collect();
                return rc;
            }
        }
        const int rc = m == 1 ? youth_icp_track_submit(c, frames + (size_t)f * N, nullptr)
                              : youth_icp_track_submit_batch(c, frames + (size_t)f * N, m);
        if (rc) {
            while (c->trk_n) (void)collect();
            return rc;
        }
        f += m;
    }
    while (c->trk_n) {
        const int rc = collect();
        if (rc) {
            while (c->trk_n) (void)collect();
            return rc;
        }
    }
    return written;
}

int youth_icp_track_frame(youth_icp_ctx* c, const int16_t* depth, const double* T_init,
                          double* T_rel, int* has_ref)
{
    if (!c || !depth || !T_rel) return set_error(YOUTH_EINVAL, "track_frame: bad arguments");
    if (c->trk_n) return set_error(YOUTH_EINVAL, "track_frame: submitted frames not collected");
    const int rc = youth_icp_track_submit(c, depth, T_init);
    if (rc) return rc;
    return youth_icp_track_collect(c, T_rel, has_ref);
}

int youth_icp_track_set_batch(youth_icp_ctx* c, int frames)
{
    if (!c || frames < 1 || frames > YOUTH_TRACK_MAX_BATCH)
        return set_error(YOUTH_EINVAL, "track_set_batch: bad arguments (%d)", frames);
    const int old = c->trk_batch;
    c->trk_batch = frames;
    // batch mode: the fewest source pixels per lane whose workgroups for
    // `frames` pairs fit one grid (512-thread workgroups at 221 VGPRs are one
    // per CU: 256 per grid; 640x480: 5 px per lane, 120 workgroups per pair),
    // for every coop launch of the context, so batched and per-frame
    // submissions stay bit-identical
    c->coop_px = c->coop_px_env;
    if (frames > 1) {
        const int v = variant(c) * 2 + (c->fast ? 1 : 0);
        // the plan leaves trk_pull_reserve CUs free for the next micro-batch's
        // k_pull_frames (the co-residency limit itself stays the whole chip);
        // the same plan on either copy path, so their poses are bit-identical
        const int free_cu = std::min(c->trk_pull_reserve, c->n_cu / 2);
        for (int npx = 1; npx <= kCoopMaxPx; ++npx) {
            const long long G = (c->N + (long long)npx * c->coop_threads - 1) /
                                ((long long)npx * c->coop_threads);
            if (frames * G <= (long long)(c->n_cu - free_cu) * c->coop_bpc[c->coop_threads == 256][v][npx]) {
                c->coop_px = npx;
                break;
            }
        }
    }
    return old;
}

long long youth_icp_track_chained(const youth_icp_ctx* c) { return c ? c->trk_chained : 0; }

long long youth_icp_track_chained_frames(const youth_icp_ctx* c)
{
    return c ? c->trk_chained_frames : 0;
}

void youth_icp_track_reset(youth_icp_ctx* c)
{
    if (c) c->track_ref = -1;
}

}  // extern "C"
