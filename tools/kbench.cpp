// kbench — A/B timing of k_reduce variants in ONE process (§5.4 rule 24).
//
// Build: make -C tools kbench      Run (GPU box): tools/kbench [pairs] [reps]
// Includes the production translation unit (so "prod" is the shipped kernel)
// plus tools/kernel_variants.inc.  Frames are prepared once by the production
// k_prep (XYZ planes for every frame, records for targets), the pose is the
// converged pose of one production align, then every variant re-runs the
// reduction at that fixed fp32 pose in interleaved rounds; per-pair sums are
// compared with the first (reference) variant.
#include "../slam-rgbd_amd/csrc/icp_kernels.hip"
#include "kernel_variants.inc"

#include <algorithm>
#include <cmath>
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

static int geometry(int N, int n_pairs, int target_blocks, int* chunk_out)
{
    int nb = (target_blocks + n_pairs - 1) / n_pairs;
    const int max_nb = (N + 2 * kRedStep - 1) / (2 * kRedStep);
    nb = std::max(1, std::min(nb, max_nb));
    int chunk = (N + nb - 1) / nb;
    chunk = (chunk + kRedStep - 1) / kRedStep * kRedStep;
    *chunk_out = chunk;
    return (N + chunk - 1) / chunk;
}

struct Variant {
    const char* name;
    int tb;             // target workgroups
    double bpp;         // kernel's own bytes per pixel
    std::function<void(dim3, int, double*)> launch;
};

int main(int argc, char** argv)
{
    const int n = argc > 1 ? atoi(argv[1]) : 64;
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    const char* filter = argc > 3 ? argv[3] : "";
    const int W = 640, H = 480, N = W * H;
    youth_intrinsics K = youth_default_intrinsics(W, H);
    youth_icp_params P = youth_default_params();
    std::vector<int16_t> src((size_t)n * N), dst((size_t)n * N);
    youth_synth_pairs(YOUTH_SYNTH_PAIR_SEED, 0, n, W, H, &K, YOUTH_SYNTH_NOISE | YOUTH_SYNTH_HOLES,
                      src.data(), dst.data(), nullptr);
    youth_icp_ctx* c = youth_icp_create(0, W, H, 2 * n, &K, &P);
    if (!c) {
        fprintf(stderr, "create: %s\n", youth_icp_last_error());
        return 1;
    }
    int16_t *d_src, *d_dst;
    CK(hipMalloc(&d_src, src.size() * 2));
    CK(hipMalloc(&d_dst, dst.size() * 2));
    CK(hipMemcpy(d_src, src.data(), src.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_dst, dst.data(), dst.size() * 2, hipMemcpyHostToDevice));
    if (youth_icp_align_pairs_device(c, d_src, d_dst, n, nullptr, nullptr, nullptr) != 0) {
        fprintf(stderr, "align: %s\n", youth_icp_last_error());
        return 1;
    }
    // XYZ planes for every frame (the v0 reference reads SoA planes); sources
    // -> workspace frames [0, n), targets -> [n, 2n) (records + planes)
    if (launch_prep(c, c->stream, d_src, n, 0, true) != 0) return 1;
    if (launch_prep(c, c->stream, d_dst, n, n, true) != 0) return 1;
    float* d_nrm;
    CK(hipMalloc(&d_nrm, (size_t)2 * n * 3 * c->P * sizeof(float)));
    CK(hipMemset(d_nrm, 0, (size_t)2 * n * 3 * c->P * sizeof(float)));
    hipLaunchKernelGGL(k_unpack_normals, dim3((N + 255) / 256, 2 * n), dim3(256), 0, c->stream,
                       c->d_rec, c->P, N, d_nrm);
    float* d_big;  // streaming-calibration buffer: 28 B/px x pixels x pairs
    CK(hipMalloc(&d_big, (size_t)28 * N * n));
    CK(hipMemset(d_big, 0, (size_t)28 * N * n));
    CK(hipStreamSynchronize(c->stream));
    printf("fast division verified: %d\n", youth_icp_fastdiv_enabled(c));
    const float thr2 = P.dist_thresh * P.dist_thresh;
    hipStream_t st = c->stream;
    float* xyz = c->d_xyz;
    float4* rec = c->d_rec;
    const size_t Pp = c->P;
    const Intr Ki = c->K;
    const FastK Fk = c->F;
    const float* T32 = c->d_T32;
    const PairMap pm_v0{0, n};     // xyz frames: sources [0, n), targets [n, 2n)
    const PairMap pm_prod{0, n};   // depth frame p of d_src, record frame n + p
    auto V0 = [=](dim3 g, int chunk, double* part) {
        hipLaunchKernelGGL(k_reduce_v0<false>, g, dim3(kRedThreads), 0, st, (const float*)xyz,
                           (const float*)d_nrm, Pp, pm_v0, T32, W, H, Ki, thr2, chunk, part,
                           (int32_t*)nullptr);
    };
    auto PROD = [=](auto kern) {
        return [=](dim3 g, int chunk, double* part) {
            const PoseState ps{nullptr, const_cast<float*>(T32), nullptr, nullptr, nullptr, 0, 1};
            hipLaunchKernelGGL(kern, g, dim3(kRedThreads), 0, st, (const int16_t*)d_src,
                               (const float4*)rec, Pp, pm_prod, W, H, Ki, Fk, thr2, chunk, part,
                               (int32_t*)nullptr, ps);
        };
    };
    std::vector<Variant> all = {
        {"v0 planes fp64 tb2048", 2048, 36, V0},
        {"prod fast aligned tb2048", 2048, 18, PROD(k_reduce<false, true, true, false>)},
        {"prod fast aligned tb4096", 4096, 18, PROD(k_reduce<false, true, true, false>)},
        {"prod fast aligned tb1024", 1024, 18, PROD(k_reduce<false, true, true, false>)},
        {"prod fast aligned tb8192", 8192, 18, PROD(k_reduce<false, true, true, false>)},
        {"prod ieee aligned tb2048", 2048, 18, PROD(k_reduce<false, false, true, false>)},
        {"s0 stream dwordx4 28B/px", 2048, 28, [=](dim3, int, double* part) {
             hipLaunchKernelGGL(k_stream_read, dim3(2048), dim3(256), 0, st, (const float4*)d_big,
                                (size_t)28 * N * n / 16, (float*)part);
         }},
        {"s1 stream dword 28B/px", 2048, 28, [=](dim3, int, double* part) {
             hipLaunchKernelGGL(k_stream_read1, dim3(2048), dim3(256), 0, st, (const float*)d_big,
                                (size_t)28 * N * n / 4, (float*)part);
         }},
    };
    std::vector<Variant> vs;
    for (auto& v : all)
        if (v.name[0] == 'v' && v.name[1] == '0') vs.push_back(v);
        else if (!*filter || strstr(v.name, filter)) vs.push_back(v);

    double* d_part;
    CK(hipMalloc(&d_part, ((size_t)n * 160 + 8192) * kNeq * sizeof(double)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<std::vector<double>> sums(vs.size());
    std::vector<std::vector<double>> parts(vs.size());  // raw partials of round 0
    std::vector<std::vector<float>> times(vs.size());
    const int rounds = 5;
    for (int r = 0; r < rounds; ++r) {
        for (size_t v = 0; v < vs.size(); ++v) {
            int chunk;
            const int nb = geometry(N, n, vs[v].tb, &chunk);
            dim3 grid(nb, n);
            vs[v].launch(grid, chunk, d_part);
            vs[v].launch(grid, chunk, d_part);
            CK(hipEventRecord(e0, st));
            for (int k = 0; k < reps; ++k) vs[v].launch(grid, chunk, d_part);
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            times[v].push_back(ms * 1000.0f / reps);
            if (r == 0) {
                std::vector<double> part((size_t)n * nb * kNeq);
                CK(hipMemcpy(part.data(), d_part, part.size() * 8, hipMemcpyDeviceToHost));
                parts[v] = part;
                sums[v].assign((size_t)n * kNeq, 0.0);
                for (int p = 0; p < n; ++p)
                    for (int b = 0; b < nb; ++b)
                        for (int k = 0; k < kNeq; ++k)
                            sums[v][(size_t)p * kNeq + k] += part[((size_t)p * nb + b) * kNeq + k];
            }
        }
    }
    const double px = (double)N * n;
    // bitwise check of every partial word against the production kernel at
    // the same geometry (same summation tree => must be identical)
    int ref = -1;
    for (size_t v = 0; v < vs.size(); ++v)
        if (strncmp(vs[v].name, "prod fast aligned", 17) == 0 && ref < 0) ref = (int)v;
    printf("%-28s %9s %9s %10s %11s %12s %10s\n", "variant", "med_us", "min_us", "GB/s@36B",
           "GB/s(own)", "max_rel_diff", "bits!=prod");
    for (size_t v = 0; v < vs.size(); ++v) {
        auto t = times[v];
        std::sort(t.begin(), t.end());
        double md = 0;
        for (size_t k = 0; k < sums[v].size(); ++k) {
            const double a = sums[v][k], b = sums[0][k];
            if (std::fabs(b) > 1e-6) md = std::max(md, std::fabs(a - b) / std::fabs(b));
        }
        const double med = t[t.size() / 2] * 1e-6;
        long nbits = -1;
        if (ref >= 0 && vs[v].tb == vs[ref].tb && parts[v].size() == parts[ref].size()) {
            nbits = 0;
            for (size_t k = 0; k < parts[v].size(); ++k)
                nbits += memcmp(&parts[v][k], &parts[ref][k], 8) != 0;
        }
        printf("%-28s %9.1f %9.1f %10.0f %11.0f %12.3e %10ld\n", vs[v].name, t[t.size() / 2],
               t[0], 36.0 * px / med / 1e9, vs[v].bpp * px / med / 1e9, md, nbits);
    }
    youth_icp_destroy(c);
    return 0;
}
