/*
 * batch_multi_demo.c — plain-C99 host aligning a batch of independent frame
 * pairs over every visible GPU (SURVEY §8e, config C4 from a C host like the
 * reference's main.c): youth_icp_align_batch_multi splits the batch into
 * contiguous shards, one host thread and context per device, and writes every
 * pose into the caller's array.  Prints the device count, the wall time and
 * pair 0's pose, and writes all poses as raw fp32 [n][16] to <out> (for the
 * test's oracle comparison).
 *
 * usage: batch_multi_demo <n_pairs> <out.f32> [W H]
 * exit 0 when every pair's status is 0.
 */
#define _POSIX_C_SOURCE 200809L
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "youth_icp.h"
#include "youth_synth.h"

int main(int argc, char** argv)
{
    const int n = argc > 1 ? atoi(argv[1]) : 8;
    const char* out = argc > 2 ? argv[2] : NULL;
    const int W = argc > 4 ? atoi(argv[3]) : 640, H = argc > 4 ? atoi(argv[4]) : 480;
    if (n <= 0 || W < 3 || H < 3) return 2;
    const youth_intrinsics K = youth_default_intrinsics(W, H);
    const size_t N = (size_t)W * H;
    int16_t* src = (int16_t*)malloc((size_t)n * N * sizeof(int16_t));
    int16_t* dst = (int16_t*)malloc((size_t)n * N * sizeof(int16_t));
    float* T = (float*)malloc((size_t)n * 16 * sizeof(float));
    int32_t* st = (int32_t*)malloc((size_t)n * sizeof(int32_t));
    if (!src || !dst || !T || !st) return 2;
    youth_synth_pairs(YOUTH_SYNTH_PAIR_SEED, 0, n, W, H, &K, YOUTH_SYNTH_NOISE | YOUTH_SYNTH_HOLES,
                      src, dst, NULL);
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    const int rc = youth_icp_align_batch_multi(src, dst, n, W, H, &K, 10, NULL, 0, T, st);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (rc != YOUTH_OK) {
        fprintf(stderr, "align_batch_multi: %d (%s)\n", rc, youth_icp_last_error());
        return 3;
    }
    int bad = 0;
    for (int p = 0; p < n; ++p) bad += st[p] != 0;
    const double s = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    printf("devices %d, pairs %d, %.3f ms (host buffers, incl. H2D), status nonzero %d\n",
           youth_icp_device_count(), n, s * 1e3, bad);
    printf("pair 0: t = (%.6f, %.6f, %.6f)\n", T[3], T[7], T[11]);
    if (out) {
        FILE* f = fopen(out, "wb");
        if (!f || fwrite(T, sizeof(float), (size_t)n * 16, f) != (size_t)n * 16) return 4;
        fclose(f);
    }
    free(src);
    free(dst);
    free(T);
    free(st);
    return bad ? 5 : 0;
}
