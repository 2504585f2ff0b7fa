// coopbench — where an iteration of k_icp_coop spends its time (one pair).
//
// Build: make -C tools coopbench
// Run (GPU box): tools/coopbench [pairs] [px_per_lane (0: the plan's)] [W H iters]
// Includes the production translation unit with YOUTH_COOP_PHASES, so thread
// 0 of every workgroup stamps s_memrealtime (100 MHz) at 8 points of every
// iteration: 0 start, 1 pixel loop done, 2 workgroup reduction done,
// 3 partial row stored, 4 = 3 and 5 = 4 (no counter, no barrier since the
// counter-free hand-off), 6 every row seen and summed, 7 solved.  Prints per-phase medians over workgroups and
// iterations 1..iters-1, and the hand-off latency (last row stored -> first
// workgroup that saw them all).
#define YOUTH_COOP_PHASES 1
#include "../slam-rgbd_amd/csrc/icp_kernels.hip"

#include <algorithm>

#include "youth_synth.h"

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

static double median(std::vector<double> v)
{
    if (v.empty()) return 0.0;
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main(int argc, char** argv)
{
    const int n = argc > 1 ? atoi(argv[1]) : 1;
    if (argc > 2 && atoi(argv[2]) > 0) setenv("YOUTH_ICP_COOP_PX", argv[2], 1);
    setenv("YOUTH_ICP_COOP_MAX_PAIRS", "16", 1);
    const int W = argc > 4 ? atoi(argv[3]) : 640, H = argc > 4 ? atoi(argv[4]) : 480, N = W * H;
    youth_intrinsics K = youth_default_intrinsics(W, H);
    youth_icp_params prm = youth_default_params();
    if (argc > 5) prm.iters = atoi(argv[5]);
    if (prm.iters < 2 || prm.iters > 32) return 2;  // the phase buffer holds 32 iterations
    std::vector<int16_t> src((size_t)n * N), dst((size_t)n * N);
    std::vector<double> Tgt((size_t)n * 16);
    youth_synth_pairs(YOUTH_SYNTH_PAIR_SEED, 0, n, W, H, &K, YOUTH_SYNTH_NOISE | YOUTH_SYNTH_HOLES,
                      src.data(), dst.data(), Tgt.data());
    youth_icp_ctx* c = youth_icp_create(0, W, H, std::max(n, 2), &K, &prm);
    if (!c) {
        fprintf(stderr, "create: %s\n", youth_icp_last_error());
        return 1;
    }
    int16_t *d_s, *d_d;
    float* d_T;
    CK(hipMalloc(&d_s, src.size() * 2));
    CK(hipMalloc(&d_d, dst.size() * 2));
    CK(hipMalloc(&d_T, (size_t)n * 16 * 4));
    CK(hipMemcpy(d_s, src.data(), src.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_d, dst.data(), dst.size() * 2, hipMemcpyHostToDevice));
    for (int r = 0; r < 50; ++r)
        if (youth_icp_align_pairs_device(c, d_s, d_d, n, nullptr, d_T, nullptr)) return 1;
    CK(hipDeviceSynchronize());
    const int G = c->last_coop_G, npx = c->last_coop_px;
    if (!G) {
        fprintf(stderr, "coop path not taken for %d pairs\n", n);
        return 1;
    }
    const int blocks = G * n, iters = prm.iters;
    unsigned long long* d_ph;
    const size_t words = (size_t)blocks * 32 * 16;
    CK(hipMalloc(&d_ph, words * 8));
    CK(hipMemset(d_ph, 0, words * 8));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(coop_phase), &d_ph, sizeof(d_ph)));
    const int reps = 20;
    std::vector<double> ph[8], hop, spread, total, sol[3], wv[4], pro[6];
    std::vector<unsigned long long> h(words);
    for (int r = 0; r < reps; ++r) {
        if (youth_icp_align_pairs_device(c, d_s, d_d, n, nullptr, d_T, nullptr)) return 1;
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h.data(), d_ph, words * 8, hipMemcpyDeviceToHost));
        auto at = [&](int b, int k, int s) { return (double)h[((size_t)b * 32 + k) * 16 + s]; };
        for (int k = 1; k < iters; ++k) {
            for (int p = 0; p < n; ++p) {
                double last3 = 0, first4 = 1e300, mn0 = 1e300, mx0 = 0;
                for (int cc = 0; cc < G; ++cc) {
                    const int b = p * G + cc;
                    for (int s = 0; s < 7; ++s) ph[s].push_back((at(b, k, s + 1) - at(b, k, s)) * 10.0);
                    if (k + 1 < iters) ph[7].push_back((at(b, k + 1, 0) - at(b, k, 7)) * 10.0);
                    last3 = std::max(last3, at(b, k, 3));
                    first4 = std::min(first4, at(b, k, 6));  // last row stored -> first workgroup that summed them all
                    mn0 = std::min(mn0, at(b, k, 0));
                    mx0 = std::max(mx0, at(b, k, 0));
                }
                hop.push_back((first4 - last3) * 10.0);
                const int b0 = p * G;
                sol[0].push_back((at(b0, k, 8) - at(b0, k, 6)) * 10.0);
                sol[1].push_back((at(b0, k, 9) - at(b0, k, 8)) * 10.0);
                sol[2].push_back((at(b0, k, 10) - at(b0, k, 9)) * 10.0);
                for (int cc = 0; cc < G; ++cc) {
                    const int b = p * G + cc;
                    wv[0].push_back((at(b, k, 11) - at(b, k, 1)) * 10.0);  // wave 0 reduce-scatter
                    for (int w = 1; w < 4; ++w)                             // wave w loop end - wave 0's
                        wv[w].push_back((at(b, k, 11 + w) - at(b, k, 1)) * 10.0);
                }
                spread.push_back((mx0 - mn0) * 10.0);
            }
        }
        for (int p = 0; p < n; ++p)
            total.push_back((at(p * G, iters - 1, 7) - at(p * G, 1, 0)) * 10.0 / (iters - 1));
        double t0 = 1e300;
        for (int b = 0; b < blocks; ++b) t0 = std::min(t0, at(b, 3, 15));
        for (int b = 0; b < blocks; ++b) {
            pro[0].push_back((at(b, 3, 15) - t0) * 10.0);          // entry after first entry
            pro[1].push_back((at(b, 0, 15) - at(b, 3, 15)) * 10.0);  // prep tiles
            pro[2].push_back((at(b, 1, 15) - at(b, 0, 15)) * 10.0);  // source staging
            pro[3].push_back((at(b, 2, 15) - at(b, 1, 15)) * 10.0);  // prep wait + acquire
            pro[4].push_back((at(b, 0, 7) - at(b, 2, 15)) * 10.0);   // iteration 0
            pro[5].push_back((at(b, iters - 1, 7) - t0) * 10.0);     // first entry -> last solve
        }
    }
    const char* names[8] = {"pixel loop", "wg reduction", "publish", "(no counter poll)",
                            "(no barrier)", "poll rows + sum", "solve+barrier", "loop back"};
    printf("%dx%d pairs %d  G %d  px/lane %d  (ns, medians over workgroups x iterations 1..%d x %d reps)\n",
           W, H, n, G, npx, iters - 1, reps);
    double acc = 0;
    for (int s = 0; s < 8; ++s) {
        const double m = median(ph[s]);
        acc += m;
        printf("  %-22s %8.0f\n", names[s], m);
    }
    printf("  %-22s %8.0f\n", "sum of medians", acc);
    printf("  %-22s %8.0f\n", "iteration (chunk 0)", median(total));
    printf("  %-22s %8.0f\n", "hand-off hop", median(hop));
    printf("  %-22s %8.0f\n", "start spread", median(spread));
    printf("  wave 0 reduce-scatter %6.0f   pixel loop end of waves 1..3 - wave 0's: %6.0f %6.0f %6.0f\n",
           median(wv[0]), median(wv[1]), median(wv[2]), median(wv[3]));
    printf("  prologue: entry skew %6.0f  prep %6.0f  source %6.0f  prep wait %6.0f  iteration 0 %6.0f"
           "  entry->done %6.0f\n",
           median(pro[0]), median(pro[1]), median(pro[2]), median(pro[3]), median(pro[4]),
           median(pro[5]));
    printf("  chunk-0 lane 0: column sums -> solve %6.0f   solve + SE(3) update %6.0f   after %6.0f\n",
           median(sol[0]), median(sol[1]), median(sol[2]));
    youth_icp_destroy(c);
    return 0;
}
