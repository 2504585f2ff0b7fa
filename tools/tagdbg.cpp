// tagdbg — why k_icp_coop with the tagged partials (profiles/r03/
// k_icp_coop_tagged_partials_experiment.patch) times out.
// Developer probe, never shipped.  tools/make_tagdbg.sh generates
// tagdbg_kernel.hip = the product source + that patch + a short spin bound
// (20000 polls) + timeout records: every reader that gives up records the
// piece it was waiting for (row, value, the four words it last read, the
// iteration's tag) and re-reads it once at system scope.  After one C2 align
// this prints the status, the records, and the partial rows' tags as the
// host then reads them from memory.
#include "tagdbg_kernel.hip"

#include <algorithm>

#include "youth_synth.h"

int main(int argc, char** argv)
{
    const int W = 640, H = 480, N = W * H;
    const int reps = argc > 1 ? atoi(argv[1]) : 2;
    youth_intrinsics K = youth_default_intrinsics(W, H);
    youth_icp_params prm = youth_default_params();
    std::vector<int16_t> src(N), dst(N);
    std::vector<double> Tgt(16);
    youth_synth_pairs(YOUTH_SYNTH_PAIR_SEED, 0, 1, W, H, &K, YOUTH_SYNTH_NOISE | YOUTH_SYNTH_HOLES,
                      src.data(), dst.data(), Tgt.data());
    youth_icp_ctx* c = youth_icp_create(0, W, H, 2, &K, &prm);
    if (!c) return 1;
    int16_t *d_s, *d_d;
    unsigned* d_dbg;
    (void)hipMalloc(&d_s, N * 2);
    (void)hipMalloc(&d_d, N * 2);
    const size_t dbg_words = 64 + 256 * 64;
    (void)hipMalloc(&d_dbg, dbg_words * 4);
    (void)hipMemcpy(d_s, src.data(), N * 2, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_d, dst.data(), N * 2, hipMemcpyHostToDevice);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(tag_dbg), &d_dbg, sizeof(d_dbg));
    printf("poll loads: aux %d\n", POLL_AUX);
    for (int r = 0; r < reps; ++r) {
        (void)hipMemset(d_dbg, 0, dbg_words * 4);
        const int rc = youth_icp_align_pairs_device(c, d_s, d_d, 1, nullptr, nullptr, nullptr);
        (void)hipDeviceSynchronize();
        double T64[16];
        float T32[12];
        int32_t st = -1;
        youth_icp_get_poses(c, 1, T64, T32, &st);
        std::vector<unsigned> h(dbg_words);
        (void)hipMemcpy(h.data(), d_dbg, h.size() * 4, hipMemcpyDeviceToHost);
        const int G = c->last_coop_G;
        printf("rep %d: rc %d status %d  G %d px %d  timeout records %u\n", r, rc, st, G,
               c->last_coop_px, h[0]);
        unsigned waves[64] = {};
        int nw = 0;
        for (unsigned s2 = 0; s2 < std::min(h[0], 256u); ++s2) {
            const unsigned* q = &h[64 + s2 * 64];
            const unsigned wv = q[0] * 8 + q[1] / 64;
            bool seen = false;
            for (int k = 0; k < nw; ++k) seen |= waves[k] == wv;
            if (!seen && nw < 64) waves[nw++] = wv;
            if (s2 < 6 || !seen) {
                printf("  wg %4u thr %3u bb %3u v %2u tag %u spins %u badmask %04x\n    poll saw:", q[0],
                       q[1], q[2], q[3], q[4], q[5], q[6]);
                for (int i = 0; i < 16; ++i) printf(" %u", q[8 + i]);
                printf("\n    sys now: ");
                for (int i = 0; i < 16; ++i) printf(" %u", q[24 + i]);
                printf("\n    poll now:");
                for (int i = 0; i < 16; ++i) printf(" %u", q[40 + i]);
                printf("%s\n", q[63] == 0xabcd1234u ? "" : " (bad record)");
            }
        }
        printf("  waves with timeouts: %d:", nw);
        for (int k = 0; k < nw; ++k) printf(" wg%u.w%u", waves[k] / 8, waves[k] % 8);
        printf("\n");
        // the rows as they sit in memory now (both parity buffers)
        const size_t words = (size_t)2 * G * kPartStride * 4;
        std::vector<unsigned> part(words);
        (void)hipMemcpy(part.data(), c->d_partials, words * 4, hipMemcpyDeviceToHost);
        for (int par = 0; par < 2; ++par) {
            unsigned mn = ~0u, mx = 0;
            int zero = 0;
            for (int b = 0; b < G; ++b)
                for (int v = 0; v < kPartStride; ++v) {
                    const unsigned t = part[(((size_t)par * G + b) * kPartStride + v) * 4 + 1];
                    mn = std::min(mn, t);
                    mx = std::max(mx, t);
                    zero += t == 0;
                }
            printf("  partial buffer %d: tags min %u max %u, zero tags %d of %d\n", par, mn, mx, zero,
                   G * kPartStride);
        }
    }
    youth_icp_destroy(c);
    return 0;
}
