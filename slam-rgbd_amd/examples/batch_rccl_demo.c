/*
 * batch_rccl_demo.c — plain-C99, one process per GPU: every
 * process aligns its contiguous shard of one batch of synthetic pairs on its
 * GPU (youth_icp_align_batch_multi with one device) and the fp32 poses are
 * all-gathered over RCCL (youth_dist.h), so every rank ends up with all of
 * them.  Rank 0 creates the communicator id and publishes it through a file
 * (written then renamed, so readers never see a partial id); the other ranks
 * wait for the file.  A stale id file of an earlier run is never joined:
 * rank 0 removes it before anything else, and a reader accepts only a file
 * written at most 30 s before the reader itself started (the ranks of one
 * launch start together).  A rank whose align fails still joins the gather
 * (its rows NaN) so no peer blocks in the collective, then exits 6.
 *
 * usage: batch_rccl_demo <nranks> <rank> <id_file> <n_pairs> <out.f32> [W H]
 *   e.g. one shell per GPU:  batch_rccl_demo 8 $r /tmp/youth.id 512 /tmp/T$r.f32
 * Each rank writes the gathered [n_pairs][16] fp32 poses to <out.f32>;
 * exit 0 when every pair of the batch has status 0 on its rank.
 */
#define _POSIX_C_SOURCE 200809L
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include "youth_dist.h"
#include "youth_icp.h"
#include "youth_synth.h"

static int read_id(const char* path, unsigned char* id, time_t started)
{
    for (int k = 0; k < 6000; ++k) {  /* up to 60 s */
        struct stat sb;
        FILE* f = (stat(path, &sb) == 0 && sb.st_mtime + 30 >= started) ? fopen(path, "rb") : NULL;
        if (f) {
            const size_t n = fread(id, 1, YOUTH_DIST_ID_BYTES, f);
            fclose(f);
            if (n == YOUTH_DIST_ID_BYTES) return 0;
        }
        struct timespec ts = {0, 10 * 1000 * 1000};
        nanosleep(&ts, NULL);
    }
    return -1;
}

int main(int argc, char** argv)
{
    if (argc < 6) {
        fprintf(stderr, "usage: %s nranks rank id_file n_pairs out.f32 [W H]\n", argv[0]);
        return 2;
    }
    const int nranks = atoi(argv[1]), rank = atoi(argv[2]), n = atoi(argv[4]);
    const char* id_file = argv[3];
    const time_t started = time(NULL);
    if (atoi(argv[2]) == 0) (void)unlink(id_file);  /* never a stale id */
    const int W = argc > 7 ? atoi(argv[6]) : 640, H = argc > 7 ? atoi(argv[7]) : 480;
    if (nranks < 1 || rank < 0 || rank >= nranks || n < 1) return 2;
    const int ndev = youth_icp_device_count();
    if (ndev < 1) {
        fprintf(stderr, "no HIP device\n");
        return 3;
    }
    const int device = rank % ndev;
    unsigned char id[YOUTH_DIST_ID_BYTES];
    if (rank == 0) {
        char tmp[4096];
        snprintf(tmp, sizeof(tmp), "%s.tmp", id_file);
        FILE* f = fopen(tmp, "wb");
        if (youth_dist_unique_id(id) != YOUTH_OK || !f ||
            fwrite(id, 1, YOUTH_DIST_ID_BYTES, f) != YOUTH_DIST_ID_BYTES || fclose(f) != 0 ||
            rename(tmp, id_file) != 0) {
            fprintf(stderr, "rank 0: cannot publish the id: %s\n", youth_dist_last_error());
            return 4;
        }
    } else if (read_id(id_file, id, started) != 0) {
        fprintf(stderr, "rank %d: no id in %s\n", rank, id_file);
        return 4;
    }
    youth_dist* d = youth_dist_create(nranks, rank, device, id);
    if (!d) {
        fprintf(stderr, "rank %d: %s\n", rank, youth_dist_last_error());
        return 5;
    }
    int first = 0, count = 0;
    youth_icp_shard_range(n, nranks, rank, &first, &count);
    const youth_intrinsics K = youth_default_intrinsics(W, H);
    const size_t N = (size_t)W * H;
    int16_t* src = (int16_t*)malloc((size_t)(count ? count : 1) * N * sizeof(int16_t));
    int16_t* dst = (int16_t*)malloc((size_t)(count ? count : 1) * N * sizeof(int16_t));
    float* T = (float*)malloc((size_t)(count ? count : 1) * 16 * sizeof(float));
    int32_t* st = (int32_t*)malloc((size_t)(count ? count : 1) * sizeof(int32_t));
    float* all = (float*)malloc((size_t)n * 16 * sizeof(float));
    if (!src || !dst || !T || !st || !all) return 2;
    int bad = 0, align_failed = 0;
    if (count > 0) {
        youth_synth_pairs(YOUTH_SYNTH_PAIR_SEED, first, count, W, H, &K,
                          YOUTH_SYNTH_NOISE | YOUTH_SYNTH_HOLES, src, dst, NULL);
        if (youth_icp_align_batch_multi(src, dst, count, W, H, &K, 10, &device, 1, T, st) !=
            YOUTH_OK) {
            /* still join the collective (every peer is in it): NaN rows */
            fprintf(stderr, "rank %d: align: %s\n", rank, youth_icp_last_error());
            align_failed = 1;
            for (size_t i = 0; i < (size_t)count * 16; ++i) T[i] = NAN;
        }
        for (int p = 0; p < count && !align_failed; ++p) bad += st[p] != 0;
    }
    if (youth_dist_allgather_poses_host(d, T, n, all) != YOUTH_OK) {
        fprintf(stderr, "rank %d: gather: %s\n", rank, youth_dist_last_error());
        return 7;
    }
    if (align_failed) {
        youth_dist_destroy(d);
        return 6;
    }
    FILE* f = fopen(argv[5], "wb");
    if (!f || fwrite(all, sizeof(float), (size_t)n * 16, f) != (size_t)n * 16) return 8;
    fclose(f);
    printf("rank %d/%d on device %d: pairs [%d, %d) aligned, %d gathered, status nonzero %d\n",
           rank, nranks, device, first, first + count, n, bad);
    youth_dist_destroy(d);
    free(src);
    free(dst);
    free(T);
    free(st);
    free(all);
    return bad ? 9 : 0;
}
