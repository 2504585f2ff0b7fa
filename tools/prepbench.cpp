// prepbench — k_prep against its memory floor, in ONE process.
//
// Build: make -C tools prepbench      Run (GPU box): tools/prepbench [frames] [reps]
// Includes the production translation unit, so "prod" is the shipped k_prep
// (records only, as in the align path).  Beside it:
//   w16  a dwordx4 store stream of the same 16 B/px (records' footprint);
//   c18  int16 depth in -> float4 out per pixel, trivial compute (the
//        kernel's algorithmic 18 B/px with no halo, no normals);
//   c18t the same in k_prep's 64x16 tiles and grid (halo rows re-read).
// Interleaved rounds; medians.
#include "../slam-rgbd_amd/csrc/icp_kernels.hip"

#include <algorithm>
#include <functional>

#include "youth_synth.h"

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

namespace {

__global__ __launch_bounds__(256) void k_write16(float4* __restrict__ out, size_t n4)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride)
        out[i] = make_float4((float)i, 0.0f, 1.0f, 2.0f);
}

// one pixel per thread, frames along y
__global__ __launch_bounds__(256) void k_copy18(const int16_t* __restrict__ d, int N, size_t P,
                                                float4* __restrict__ out)
{
    const int f = blockIdx.y;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const float z = (float)d[(size_t)f * N + i];
    out[(size_t)f * P + i] = make_float4(z, z * 0.5f, z * 0.25f, z * 0.125f);
}

// k_prep's tile and grid: each thread reads its 4 rows' depth plus the
// block reads one halo row above and below, writes 4 records
__global__ __launch_bounds__(256) void k_copy18_tiles(const int16_t* __restrict__ d, int W, int H,
                                                      size_t P, float4* __restrict__ out)
{
    __shared__ float s[kTileH + 2][kTileW];
    const int f = blockIdx.z;
    const int x0 = blockIdx.x * kTileW, y0 = blockIdx.y * kTileH;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    const int16_t* dep = d + (size_t)f * W * H;
    for (int r = ty; r < kTileH + 2; r += 4) {
        const int gy = y0 - 1 + r, gx = x0 + tx;
        s[r][tx] = (gy >= 0 && gy < H && gx < W) ? (float)dep[(size_t)gy * W + gx] : 0.0f;
    }
    __syncthreads();
    for (int k = 0; k < kTileH / 4; ++k) {
        const int row = ty + 4 * k, gx = x0 + tx, gy = y0 + row;
        if (gx >= W || gy >= H) continue;
        const float z = s[row + 1][tx];
        const float a = s[row][tx] + s[row + 2][tx];
        out[(size_t)f * P + (size_t)gy * W + gx] = make_float4(z, a, z * 0.25f, a * 0.125f);
    }
}


// S 64x16 tiles per workgroup, stacked vertically; the next tile's halo
// depth words are loaded into registers before the current tile's normals
// are computed, so their latency overlaps that work (wide path only).
template <bool kFast, int S>
__global__ __launch_bounds__(256) void k_prep_pf(const int16_t* __restrict__ depth, int W, int H,
                                                 size_t P, Intr K, FastK F,
                                                 float4* __restrict__ recs)
{
    __shared__ float sX[kLdsH][kLdsW];
    __shared__ float sY[kLdsH][kLdsW];
    __shared__ float sZ[kLdsH][kLdsW];
    constexpr int kWords = (kTileW + 8) / 4;  // 18 per halo row
    constexpr int kE = kLdsH * kWords;        // 324 words per tile
    const int f = blockIdx.z;
    const int16_t* dep = depth + (size_t)f * W * H;
    float4* R = recs + (size_t)f * P;
    const int x0 = blockIdx.x * kTileW;
    const int ybase = blockIdx.y * kTileH * S;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    const int e0 = threadIdx.x, e1 = threadIdx.x + kPrepThreads;
    short4 w[2];
    auto load = [&](int y0) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int e = q ? e1 : e0;
            const int ly = e / kWords, m = e - ly * kWords;
            const int gy = y0 - 1 + ly, c = x0 - 4 + 4 * m;
            w[q] = make_short4(0, 0, 0, 0);
            if (e < kE && gy >= 0 && gy < H && c >= 0 && c < W)
                w[q] = *reinterpret_cast<const short4*>(dep + (size_t)gy * W + c);
        }
    };
    auto stage = [&](int y0) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int e = q ? e1 : e0;
            if (e >= kE) continue;
            const int ly = e / kWords, m = e - ly * kWords;
            const int gy = y0 - 1 + ly, c = x0 - 4 + 4 * m;
            const int dv[4] = {w[q].x, w[q].y, w[q].z, w[q].w};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int lx = 4 * m - 3 + r;
                if (lx < 0 || lx >= kLdsW) continue;
                float x, y, z;
                backproject<kFast>(dv[r], c + r, gy, K, F, x, y, z);
                sX[ly][lx] = x;
                sY[ly][lx] = y;
                sZ[ly][lx] = z;
            }
        }
    };
    load(ybase);
    for (int t = 0; t < S; ++t) {
        const int y0 = ybase + kTileH * t;
        if (y0 >= H) break;
        if (t) __syncthreads();  // previous tile's LDS reads done
        stage(y0);
        __syncthreads();
        if (t + 1 < S && y0 + kTileH < H) load(y0 + kTileH);
#pragma unroll
        for (int k = 0; k < kTileH / 4; ++k) {
            const int row = ty + 4 * k;
            const int gx = x0 + tx, gy = y0 + row;
            if (gx >= W || gy >= H) continue;
            const int i = gy * W + gx;
            const int ly = row + 1, lx = tx + 1;
            const float px = sX[ly][lx], py = sY[ly][lx], pz = sZ[ly][lx];
            float nx = 0.0f, ny = 0.0f, nz = 0.0f;
            bool has_n = false;
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
                        if (norm_fast_ok(len2, cx, cy, cz)) {
                            const float len = sqrt_rn_mid(len2);
                            const float r = proj_recip(len);
                            nx = norm_div(cx, len, r);
                            ny = norm_div(cy, len, r);
                            nz = norm_div(cz, len, r);
                        } else {
                            const float len = sqrtf(len2);
                            nx = cx / len;
                            ny = cy / len;
                            nz = cz / len;
                        }
                        has_n = true;
                        if (((nx * px + ny * py) + nz * pz) > 0.0f) {
                            nx = -nx;
                            ny = -ny;
                            nz = -nz;
                        }
                    }
                }
            }
            R[i] = make_float4(has_n ? pz : 0.0f, nx, ny, nz);
        }
    }
}

}  // namespace

int main(int argc, char** argv)
{
    const int n = argc > 1 ? atoi(argv[1]) : 64;
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    const int W = 640, H = 480, N = W * H;
    youth_intrinsics K = youth_default_intrinsics(W, H);
    youth_icp_params P = youth_default_params();
    std::vector<int16_t> src((size_t)n * N), dst((size_t)n * N);
    youth_synth_pairs(YOUTH_SYNTH_PAIR_SEED, 0, n, W, H, &K, YOUTH_SYNTH_NOISE | YOUTH_SYNTH_HOLES,
                      src.data(), dst.data(), nullptr);
    youth_icp_ctx* c = youth_icp_create(0, W, H, n, &K, &P);
    if (!c) {
        fprintf(stderr, "create: %s\n", youth_icp_last_error());
        return 1;
    }
    int16_t* d_dst;
    CK(hipMalloc(&d_dst, dst.size() * 2));
    CK(hipMemcpy(d_dst, dst.data(), dst.size() * 2, hipMemcpyHostToDevice));
    float4* d_out;
    CK(hipMalloc(&d_out, (size_t)n * c->P * sizeof(float4)));
    hipStream_t st = c->stream;
    const size_t Pp = c->P;
    auto launch_pf = [&]<int S>() {
        auto kern = k_prep_pf<true, S>;
        hipLaunchKernelGGL(kern,
                           dim3((W + kTileW - 1) / kTileW, (H + kTileH * S - 1) / (kTileH * S), n),
                           dim3(256), 0, st, d_dst, W, H, Pp, c->K, c->F, d_out);
    };
    struct V {
        const char* name;
        std::function<void()> launch;
    };
    std::vector<V> vs = {
        {"prod k_prep", [&] { (void)launch_prep(c, st, d_dst, n, 0, false); }},
        {"pf S=1 (hoisted halo)", [&] { launch_pf.template operator()<1>(); }},
        {"pf S=2", [&] { launch_pf.template operator()<2>(); }},
        {"pf S=3", [&] { launch_pf.template operator()<3>(); }},
        {"pf S=4", [&] { launch_pf.template operator()<4>(); }},
        {"pf S=6", [&] { launch_pf.template operator()<6>(); }},
        {"w16 store stream", [&] {
             hipLaunchKernelGGL(k_write16, dim3(8192), dim3(256), 0, st, d_out, (size_t)n * N);
         }},
        {"c18 depth->float4", [&] {
             hipLaunchKernelGGL(k_copy18, dim3((N + 255) / 256, n), dim3(256), 0, st, d_dst, N, Pp,
                                d_out);
         }},
        {"c18t tiles+halo", [&] {
             hipLaunchKernelGGL(k_copy18_tiles,
                                dim3((W + kTileW - 1) / kTileW, (H + kTileH - 1) / kTileH, n),
                                dim3(256), 0, st, d_dst, W, H, Pp, d_out);
         }},
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> t(vs.size());
    for (int r = 0; r < 7; ++r)
        for (size_t v = 0; v < vs.size(); ++v) {
            vs[v].launch();
            CK(hipEventRecord(e0, st));
            for (int k = 0; k < reps; ++k) vs[v].launch();
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t[v].push_back(ms * 1000.0f / reps);
        }
    // bitwise check of every pf variant's records against production k_prep's
    std::vector<float4> ref((size_t)n * Pp), got((size_t)n * Pp);
    (void)launch_prep(c, st, d_dst, n, 0, false);
    CK(hipMemcpyAsync(ref.data(), c->d_rec, ref.size() * 16, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    std::vector<long> mism(vs.size(), -1);
    for (size_t v = 0; v < vs.size(); ++v) {
        if (strncmp(vs[v].name, "pf", 2) != 0) continue;
        CK(hipMemsetAsync(d_out, 0xFF, got.size() * 16, st));
        vs[v].launch();
        CK(hipMemcpyAsync(got.data(), d_out, got.size() * 16, hipMemcpyDeviceToHost, st));
        CK(hipStreamSynchronize(st));
        long bad = 0;
        for (int fr = 0; fr < n; ++fr)
            for (int i = 0; i < N; ++i)
                bad += memcmp(&ref[(size_t)fr * Pp + i], &got[(size_t)fr * Pp + i], 16) != 0;
        mism[v] = bad;
    }
    const double px = (double)N * n;
    printf("frames %d @%dx%d, fast division %d\n", n, W, H, youth_icp_fastdiv_enabled(c));
    printf("%-22s %9s %9s %12s %12s %10s\n", "variant", "med_us", "min_us", "GB/s@18B/px",
           "store GB/s", "recs!=prod");
    for (size_t v = 0; v < vs.size(); ++v) {
        std::sort(t[v].begin(), t[v].end());
        const double med = t[v][t[v].size() / 2];
        printf("%-22s %9.1f %9.1f %12.0f %12.0f %10ld\n", vs[v].name, med, t[v][0],
               18.0 * px / (med * 1e-6) / 1e9, 16.0 * px / (med * 1e-6) / 1e9, mism[v]);
    }
    youth_icp_destroy(c);
    return 0;
}
