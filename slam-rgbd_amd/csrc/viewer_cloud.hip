// Viewer point list on gfx950 (C-ABI: include/youth_viewer.h).
//
// The reference's 3-D view (Youth.Source/ViewerModule/viewerModule.c:336-357)
// walks the latest frame on the CPU and emits glColor3f + glVertex3f for
// every pixel with depth > 0.  Here the same list, in the same order and with
// the same fp32 expressions, is built as a packed vertex array
// {-x, -y, -z, r, g, b} in HBM by three launches per batch of frames:
//
//   k_cloud_count  one 2048-pixel tile per workgroup: valid pixels per tile
//                  (2 B/px read)
//   k_cloud_scan   one workgroup per frame: exclusive scan of the tile counts
//                  -> each tile's first vertex, and the frame's vertex count
//   k_cloud_emit   the tile again with its colour (5 B/px read): each thread
//                  owns 8 consecutive pixels, its vertices' in-tile slots come
//                  from a wave prefix of the per-thread counts plus the waves
//                  before it; the tile's vertices are staged in LDS in final
//                  order and written out as one contiguous run (24 B/vertex)
//
// Integer / byte work plus three IEEE fp32 quotients per pixel: HBM-bound,
// no MFMA.  The order of the list is the reference's loop order (row-major
// over valid pixels), so the output is deterministic and bit-identical to
// the C oracle (oracle_viewer_cloud).
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "youth_viewer.h"

namespace {

constexpr int kCloudThreads = 256;
constexpr int kVF = YOUTH_CLOUD_FLOATS_PER_VERTEX;      // 6 floats per vertex

struct CloudK {
    float fx, fy, cx, cy, ds;
};

// kPx depth values of pixels [i, i+kPx) of one frame.  kVec: one 8-/16-byte
// load (frame base aligned, N % kPx == 0, so i + kPx <= N whenever i < N).
template <bool kVec, int kPx>
__device__ __forceinline__ void load_depth(const int16_t* __restrict__ d, int i, int N, int* dd)
{
    if (kVec) {
        int v[kPx / 2];
        if (i < N) {
            if constexpr (kPx == 8) {
                const int4 w = *reinterpret_cast<const int4*>(d + i);
                v[0] = w.x;
                v[1] = w.y;
                v[2] = w.z;
                v[3] = w.w;
            } else {
                const int2 w = *reinterpret_cast<const int2*>(d + i);
                v[0] = w.x; v[1] = w.y;
            }
        } else {
#pragma unroll
            for (int k = 0; k < kPx / 2; ++k) v[k] = 0;
        }
#pragma unroll
        for (int k = 0; k < kPx / 2; ++k) {
            dd[2 * k] = (int)(short)(v[k] & 0xffff);   // little-endian: low half first
            dd[2 * k + 1] = v[k] >> 16;                // arithmetic shift: sign kept
        }
    } else {
#pragma unroll
        for (int k = 0; k < kPx; ++k) dd[k] = (i + k) < N ? (int)d[i + k] : 0;
    }
}

// kPx * 3 colour bytes of pixels [i, i+kPx) (viewerModule.c:348-352): kVec
// loads 8-byte (kPx 8) or 4-byte (kPx 4) words, the offset (fN + i) * 3
// being a multiple of 24 / 12.
template <bool kVec, int kPx>
__device__ __forceinline__ void load_rgb(const uint8_t* __restrict__ c, int i, int N,
                                         unsigned char* cc)
{
    if (kVec && i < N) {
        unsigned wds[kPx * 3 / 4];
        if constexpr (kPx == 8) {
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const uint2 w = *reinterpret_cast<const uint2*>(c + 8 * k);
                wds[2 * k] = w.x;
                wds[2 * k + 1] = w.y;
            }
        } else {
#pragma unroll
            for (int k = 0; k < 3; ++k) wds[k] = *reinterpret_cast<const unsigned*>(c + 4 * k);
        }
#pragma unroll
        for (int k = 0; k < kPx * 3; ++k) cc[k] = (unsigned char)(wds[k >> 2] >> (8 * (k & 3)));
    } else {
#pragma unroll
        for (int k = 0; k < kPx * 3; ++k) cc[k] = (i + k / 3) < N ? c[k] : (unsigned char)0;
    }
}

__device__ __forceinline__ int wave_sum_i32(int x)
{
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) x += __shfl_xor(x, m, 64);
    return x;
}

// Inclusive prefix over the 64 lanes (Hillis-Steele, 6 steps).
__device__ __forceinline__ int wave_incl_scan_i32(int x, int lane)
{
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) {
        const int y = __shfl_up(x, m, 64);
        x += lane >= m ? y : 0;
    }
    return x;
}

template <bool kVec, int kPx>
__global__ __launch_bounds__(kCloudThreads) void k_cloud_count(const int16_t* __restrict__ depth,
                                                                int N, int tiles,
                                                                int32_t* __restrict__ tile_cnt)
{
    __shared__ int sw[kCloudThreads / 64];
    const int f = blockIdx.y, tile = blockIdx.x;
    const int i = (tile * kCloudThreads + threadIdx.x) * kPx;
    int dd[kPx];
    load_depth<kVec, kPx>(depth + (size_t)f * N, i, N, dd);
    int c = 0;
#pragma unroll
    for (int k = 0; k < kPx; ++k) c += dd[k] > 0 ? 1 : 0;   // viewerModule.c:342
    c = wave_sum_i32(c);
    if ((threadIdx.x & 63) == 0) sw[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        int s = 0;
#pragma unroll
        for (int w = 0; w < kCloudThreads / 64; ++w) s += sw[w];
        tile_cnt[(size_t)f * tiles + tile] = s;
    }
}

// Exclusive scan of one frame's tile counts: thread t owns the contiguous run
// of tiles [t R, t R + R), R = ceil(tiles / 256).
__global__ __launch_bounds__(kCloudThreads) void k_cloud_scan(const int32_t* __restrict__ tile_cnt,
                                                               int tiles,
                                                               int32_t* __restrict__ tile_off,
                                                               int32_t* __restrict__ counts)
{
    __shared__ int sw[kCloudThreads / 64];
    const int f = blockIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int R = (tiles + kCloudThreads - 1) / kCloudThreads;
    const int t0 = threadIdx.x * R;
    const int t1 = min(t0 + R, tiles);
    const int32_t* cnt = tile_cnt + (size_t)f * tiles;
    int s = 0;
    for (int t = t0; t < t1; ++t) s += cnt[t];
    const int incl = wave_incl_scan_i32(s, lane);
    if (lane == 63) sw[wave] = incl;
    __syncthreads();
    int woff = 0;
    for (int w = 0; w < wave; ++w) woff += sw[w];
    int run = woff + incl - s;   // exclusive prefix of this thread's run
    int32_t* off = tile_off + (size_t)f * tiles;
    for (int t = t0; t < t1; ++t) {
        off[t] = run;
        run += cnt[t];
    }
    if (threadIdx.x == kCloudThreads - 1) counts[f] = woff + incl;
}

// The tile's vertices are staged in LDS in list order, placed so that LDS
// float j and output float (run start - head + j) share their offset mod 4
// (head = the run start's float offset within its 16-byte granule); the run
// is then copied out in 16-byte stores, element stores only for the partial
// granules at its two ends.  (Storing each vertex straight from registers,
// 3 x 8-byte stores, measured 1.7x slower: 64 lanes' partial lines per
// instruction; profiles/r01/cloud_ab.txt.)
template <bool kVec, int kPx>
__global__ __launch_bounds__(kCloudThreads) void k_cloud_emit(
    const int16_t* __restrict__ depth, const uint8_t* __restrict__ rgb, int W, int N, int tiles,
    CloudK K, const int32_t* __restrict__ tile_off, const float* __restrict__ T_world,
    float* __restrict__ vertices)
{
    constexpr int kTile = kCloudThreads * kPx;
    __shared__ __align__(16) float stage[kTile * kVF + 4];   // the tile's vertices, list order
    __shared__ int sw[kCloudThreads / 64];
    const int f = blockIdx.y, tile = blockIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int i = (tile * kCloudThreads + threadIdx.x) * kPx;
    int dd[kPx];
    load_depth<kVec, kPx>(depth + (size_t)f * N, i, N, dd);
    unsigned char cc[kPx * 3];
    if (rgb) {
        load_rgb<kVec, kPx>(rgb + ((size_t)f * N + i) * 3, i, N, cc);
    } else {
#pragma unroll
        for (int k = 0; k < kPx * 3; ++k) cc[k] = 0;
    }
    int c = 0;
#pragma unroll
    for (int k = 0; k < kPx; ++k) c += dd[k] > 0 ? 1 : 0;
    const int incl = wave_incl_scan_i32(c, lane);
    if (lane == 63) sw[wave] = incl;
    __syncthreads();
    int woff = 0, total = 0;
#pragma unroll
    for (int w = 0; w < kCloudThreads / 64; ++w) {
        woff += w < wave ? sw[w] : 0;
        total += sw[w];
    }
    int slot = woff + incl - c;
    // frame f's camera -> world pose (row-major 3x4), or none
    float Tw[12];
    if (T_world) {
#pragma unroll
        for (int q = 0; q < 12; ++q) Tw[q] = T_world[(size_t)f * 12 + q];
    }
    float* out = vertices + ((size_t)f * N + (size_t)tile_off[(size_t)f * tiles + tile]) * kVF;
    const int head = (int)(((uintptr_t)out >> 2) & 3);
    // (u, v) of pixel i; a thread's pixels may wrap rows (any W >= 1)
    int v = i / W;
    int u = i - v * W;
#pragma unroll
    for (int k = 0; k < kPx; ++k) {
        if (dd[k] > 0) {
            // viewerModule.c:343-345, evaluated as written (IEEE quotients)
            const float z = (float)dd[k] / K.ds;
            const float x = (((float)u - K.cx) * z) / K.fx;
            const float y = (((float)v - K.cy) * z) / K.fy;
            // world frame (youth_cloud_build_device_posed): P_w = R P + t as
            // three fma chains, the ICP transform's order (spec a7)
            const float px = T_world ? fmaf(Tw[2], z, fmaf(Tw[1], y, fmaf(Tw[0], x, Tw[3]))) : x;
            const float py = T_world ? fmaf(Tw[6], z, fmaf(Tw[5], y, fmaf(Tw[4], x, Tw[7]))) : y;
            const float pz = T_world ? fmaf(Tw[10], z, fmaf(Tw[9], y, fmaf(Tw[8], x, Tw[11]))) : z;
            // glVertex3f(-x_pos, -y_pos, -z_pos) (:354), glColor3f(r, g, b) (:349-351)
            const float o[kVF] = {-px, -py, -pz, (float)cc[3 * k + 0] / 255.0f,
                                  (float)cc[3 * k + 1] / 255.0f, (float)cc[3 * k + 2] / 255.0f};
#pragma unroll
            for (int q = 0; q < kVF; ++q) stage[head + slot * kVF + q] = o[q];
            ++slot;
        }
        ++u;
        while (u >= W) {
            u -= W;
            ++v;
        }
    }
    __syncthreads();
    // the tile's run of the frame's list, floats [head, head + nf) of the
    // 16-byte granules starting at out - head
    const int nf = total * kVF;
    const int end = head + nf;
    float* base = out - head;
    for (int g = threadIdx.x; g * 4 < end; g += kCloudThreads) {
        const int j = g * 4;
        if (j >= head && j + 4 <= end) {
            // non-temporal: the list is for the renderer, not re-read here
            // (111 vs 121 us per 64-frame call, profiles/r02/ab_s31.txt)
            typedef float f4nt __attribute__((ext_vector_type(4)));
            __builtin_nontemporal_store(*reinterpret_cast<const f4nt*>(stage + j),
                                        reinterpret_cast<f4nt*>(base + j));
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (j + q >= head && j + q < end) base[j + q] = stage[j + q];
        }
    }
}

}  // namespace

// =============================================================== host side ==

static thread_local std::string g_cloud_error;

__attribute__((format(printf, 2, 3))) static int cloud_error(int code, const char* fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_cloud_error = buf;
    return code;
}

#define CLOUD_TRY(expr)                                                                   \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess)                                                             \
            return cloud_error(YOUTH_EHIP, "%s (line %d)", hipGetErrorString(e_), __LINE__); \
    } while (0)

struct youth_cloud_ctx {
    int device = 0;
    int W = 0, H = 0, N = 0, max_frames = 0, max_tiles = 0;
    int px = 8;   // pixels per thread (tile = 256 px): YOUTH_CLOUD_PX=4|8
    hipStream_t stream = nullptr;
    int32_t* d_tile_cnt = nullptr;   // [max_frames][max_tiles]
    int32_t* d_tile_off = nullptr;   // [max_frames][max_tiles]
    int16_t* d_depth = nullptr;      // host API staging, one frame
    uint8_t* d_rgb = nullptr;
    float* d_vert = nullptr;         // [N][6]
    int32_t* d_count = nullptr;      // [1]
};

static void cloud_free(youth_cloud_ctx* c)
{
    if (!c) return;
    if (c->device >= 0 && hipSetDevice(c->device) == hipSuccess) {
        (void)hipFree(c->d_tile_cnt);
        (void)hipFree(c->d_tile_off);
        (void)hipFree(c->d_depth);
        (void)hipFree(c->d_rgb);
        (void)hipFree(c->d_vert);
        (void)hipFree(c->d_count);
        if (c->stream) (void)hipStreamDestroy(c->stream);
    }
    delete c;
}

extern "C" {

const char* youth_cloud_last_error(void) { return g_cloud_error.c_str(); }

youth_cloud_ctx* youth_cloud_create(int device, int W, int H, int max_frames)
{
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        cloud_error(YOUTH_ENODEV, "youth_cloud_create: no HIP device visible");
        return nullptr;
    }
    if (device < 0 || device >= ndev) {
        cloud_error(YOUTH_EINVAL, "youth_cloud_create: device %d of %d", device, ndev);
        return nullptr;
    }
    if (W < 1 || H < 1 || W > 16384 || H > 16384 || (long long)W * H > (1LL << 26) ||
        max_frames < 1 || max_frames > 65535) {
        cloud_error(YOUTH_EINVAL,
                    "youth_cloud_create: %dx%d x %d frames (need 1 <= W,H <= 16384, W*H <= 2^26, "
                    "1 <= frames <= 65535)",
                    W, H, max_frames);
        return nullptr;
    }
    auto* c = new youth_cloud_ctx;
    c->device = device;
    c->W = W;
    c->H = H;
    c->N = W * H;
    c->max_frames = max_frames;
    if (const char* e = getenv("YOUTH_CLOUD_PX")) c->px = atoi(e) == 4 ? 4 : 8;
    c->max_tiles = (c->N + kCloudThreads * 4 - 1) / (kCloudThreads * 4);   // room for px = 4
    const size_t nt = (size_t)max_frames * c->max_tiles;
    if (hipSetDevice(device) != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&c->d_tile_cnt, nt * sizeof(int32_t)) != hipSuccess ||
        hipMalloc(&c->d_tile_off, nt * sizeof(int32_t)) != hipSuccess ||
        hipMalloc(&c->d_depth, (size_t)c->N * sizeof(int16_t)) != hipSuccess ||
        hipMalloc(&c->d_rgb, (size_t)c->N * 3) != hipSuccess ||
        hipMalloc(&c->d_vert, (size_t)c->N * kVF * sizeof(float)) != hipSuccess ||
        hipMalloc(&c->d_count, sizeof(int32_t)) != hipSuccess) {
        cloud_error(YOUTH_ENOMEM, "youth_cloud_create: device allocation failed (%dx%d x %d)", W,
                    H, max_frames);
        cloud_free(c);
        return nullptr;
    }
    return c;
}

void youth_cloud_destroy(youth_cloud_ctx* c) { cloud_free(c); }

int youth_cloud_build_device(youth_cloud_ctx* c, const int16_t* d_depth, const uint8_t* d_rgb,
                             int n_frames, int W, int H, const youth_intrinsics* K,
                             float* d_vertices, int32_t* d_counts, void* stream)
{
    return youth_cloud_build_device_posed(c, d_depth, d_rgb, n_frames, W, H, K, nullptr,
                                          d_vertices, d_counts, stream);
}

int youth_cloud_build_device_posed(youth_cloud_ctx* c, const int16_t* d_depth,
                                   const uint8_t* d_rgb, int n_frames, int W, int H,
                                   const youth_intrinsics* K, const float* d_T_world,
                                   float* d_vertices, int32_t* d_counts, void* stream)
{
    if (!c || !d_depth || !d_vertices || !d_counts)
        return cloud_error(YOUTH_EINVAL, "youth_cloud_build_device: null argument");
    if (n_frames < 0 || n_frames > c->max_frames || W < 1 || H < 1 || W > c->W || H > c->H ||
        (long long)W * H > c->N)
        return cloud_error(YOUTH_EINVAL,
                           "youth_cloud_build_device: %d frames of %dx%d (context: %d of %dx%d)",
                           n_frames, W, H, c->max_frames, c->W, c->H);
    if (n_frames == 0) return YOUTH_OK;
    CLOUD_TRY(hipSetDevice(c->device));
    const int N = W * H;
    const int tile_px = kCloudThreads * c->px;
    const int tiles = (N + tile_px - 1) / tile_px;
    CloudK k{570.3f, 570.3f, (float)(W / 2), (float)(H / 2), 1000.0f};   // viewerModule.c:343-345
    if (K) k = CloudK{K->fx, K->fy, K->cx, K->cy, K->depth_scale};
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    // vector loads: every frame base and thread offset aligned for the
    // 2 px-byte depth word and the 3 px-byte colour words
    const bool vec = (N % c->px) == 0 && ((uintptr_t)d_depth % (2 * c->px)) == 0 &&
                     (!d_rgb || ((uintptr_t)d_rgb % (c->px == 8 ? 8 : 4)) == 0);
    using CountFn = void (*)(const int16_t*, int, int, int32_t*);
    using EmitFn = void (*)(const int16_t*, const uint8_t*, int, int, int, CloudK, const int32_t*,
                            const float*, float*);
    static const CountFn count_fn[2][2] = {{k_cloud_count<false, 4>, k_cloud_count<true, 4>},
                                           {k_cloud_count<false, 8>, k_cloud_count<true, 8>}};
    static const EmitFn emit_fn[2][2] = {{k_cloud_emit<false, 4>, k_cloud_emit<true, 4>},
                                         {k_cloud_emit<false, 8>, k_cloud_emit<true, 8>}};
    const int pi = c->px == 8 ? 1 : 0;
    const dim3 grid(tiles, n_frames);
    hipLaunchKernelGGL(count_fn[pi][vec], grid, dim3(kCloudThreads), 0, s, d_depth, N, tiles,
                       c->d_tile_cnt);
    CLOUD_TRY(hipGetLastError());
    k_cloud_scan<<<n_frames, kCloudThreads, 0, s>>>(c->d_tile_cnt, tiles, c->d_tile_off, d_counts);
    CLOUD_TRY(hipGetLastError());
    hipLaunchKernelGGL(emit_fn[pi][vec], grid, dim3(kCloudThreads), 0, s, d_depth,
                       d_rgb, W, N, tiles, k, (const int32_t*)c->d_tile_off, d_T_world, d_vertices);
    CLOUD_TRY(hipGetLastError());
    return YOUTH_OK;
}

int youth_cloud_build_host(youth_cloud_ctx* c, const int16_t* depth, const uint8_t* rgb, int W,
                           int H, const youth_intrinsics* K, float* vertices, int cap)
{
    if (!c || !depth || !vertices || cap < 0)
        return cloud_error(YOUTH_EINVAL, "youth_cloud_build_host: null argument");
    if (W < 1 || H < 1 || W > c->W || H > c->H || (long long)W * H > c->N)
        return cloud_error(YOUTH_EINVAL, "youth_cloud_build_host: %dx%d frame (context %dx%d)", W,
                           H, c->W, c->H);
    CLOUD_TRY(hipSetDevice(c->device));
    const size_t N = (size_t)W * H;
    CLOUD_TRY(hipMemcpyAsync(c->d_depth, depth, N * sizeof(int16_t), hipMemcpyHostToDevice,
                             c->stream));
    if (rgb)
        CLOUD_TRY(hipMemcpyAsync(c->d_rgb, rgb, N * 3, hipMemcpyHostToDevice, c->stream));
    const int rc = youth_cloud_build_device(c, c->d_depth, rgb ? c->d_rgb : nullptr, 1, W, H, K,
                                            c->d_vert, c->d_count, c->stream);
    if (rc < 0) return rc;
    int32_t n = 0;
    CLOUD_TRY(hipMemcpyAsync(&n, c->d_count, sizeof(n), hipMemcpyDeviceToHost, c->stream));
    CLOUD_TRY(hipStreamSynchronize(c->stream));
    if (n > cap)
        return cloud_error(YOUTH_EINVAL, "youth_cloud_build_host: %d vertices, room for %d", n,
                           cap);
    if (n > 0)
        CLOUD_TRY(hipMemcpy(vertices, c->d_vert, (size_t)n * kVF * sizeof(float),
                            hipMemcpyDeviceToHost));
    return n;
}

int youth_cloud_sync(youth_cloud_ctx* c, void* stream)
{
    if (!c) return cloud_error(YOUTH_EINVAL, "youth_cloud_sync: null context");
    CLOUD_TRY(hipSetDevice(c->device));
    CLOUD_TRY(hipStreamSynchronize(stream ? (hipStream_t)stream : c->stream));
    return YOUTH_OK;
}

}  // extern "C"
