/*
 * slam_rate.c — plain-C99 rate test of the SLAM.h drop-in: one producer
 * thread calling processSlamFrame as the reference's logger does at its
 * frame-complete point (loggingModule.c:354), the module's own worker
 * tracking (SLAM.cpp:32-63 semantics; micro-batches of the queued frames by
 * default).
 *
 *   backlogged: the producer pushes as fast as it can but never past the
 *               reference's drop threshold (it waits while 10 frames are
 *               queued, SLAM.cpp:163-168, so no frame is dropped); timed
 *               until the last frame's pose is in the trajectory;
 *   live:       one frame at a time, each waited for (a camera's per-frame
 *               latency).
 *
 * Prints one JSON object: frames/s per pass (backlogged), the median, the
 * producer's mean time inside processSlamFrame per pass (the frame copy), each
 * pass's CLOCK_MONOTONIC window, the
 * live latency median / p90 in microseconds, frames aligned in chained
 * launches, and a checksum of the last pass's world poses.
 *
 * With YOUTH_SLAM_TRACE=<file> set, the module's event trace
 * (youth_slam_trace_enable) covers the backlogged passes and is written to
 * <file> as "t_seconds kind arg" lines (tools/slam_trace.py reads it beside a
 * rocprofv3 kernel trace); the live frames' events go to <file>.live
 * (tools/slam_trace.py --live).
 *
 * usage: slam_rate <n_frames> <passes> [width height]
 */
#define _POSIX_C_SOURCE 200809L
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "youth_icp.h"
#include "youth_synth.h"

static double now_s(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static int cmp_d(const void* a, const void* b)
{
    const double x = *(const double*)a, y = *(const double*)b;
    return (x > y) - (x < y);
}

int main(int argc, char** argv)
{
    const int n = argc > 1 ? atoi(argv[1]) : 300;
    const int passes = argc > 2 ? atoi(argv[2]) : 5;
    const int W = argc > 4 ? atoi(argv[3]) : 640, H = argc > 4 ? atoi(argv[4]) : 480;
    if (n < 2 || passes < 1 || passes > 64 || W < 3 || H < 3) return 2;
    const size_t N = (size_t)W * H;
    youth_intrinsics K = youth_default_intrinsics(W, H);
    int16_t* frames = (int16_t*)malloc((size_t)n * N * sizeof(int16_t));
    double* lat = (double*)malloc((size_t)n * sizeof(double));
    double* T = (double*)malloc((size_t)n * 16 * sizeof(double));
    if (!frames || !lat || !T) return 3;
    youth_synth_sequence(YOUTH_SYNTH_SEQ_SEED, 0, n, W, H, &K,
                         YOUTH_SYNTH_NOISE | YOUTH_SYNTH_HOLES, frames, NULL);
    initSlamModule(NULL, NULL);
    if (!isSlamModuleRunning()) {
        fprintf(stderr, "slam_rate: module did not start (no HIP device?)\n");
        return 4;
    }
    /* warm: the worker's context, its plan and the page-locked queue pool;
     * SLAM_RATE_WARM_PASSES=k adds k untimed backlogged passes */
    for (int k = 0; k < n && k < 24; ++k) processSlamFrame(frames + (size_t)k * N, NULL, W, H, k);
    youth_slam_wait_idle(20000);
    const char* wp = getenv("SLAM_RATE_WARM_PASSES");
    for (int p = 0; wp && p < atoi(wp); ++p) {
        resetSlam();
        youth_slam_wait_idle(20000);
        for (int k = 0; k < n; ++k) {
            while (youth_slam_queue_size() >= 10) {
            }
            processSlamFrame(frames + (size_t)k * N, NULL, W, H, (uint32_t)k);
        }
        while (youth_slam_trajectory_length() < n) {
        }
    }
    double rate[64], push_us[64], win[64][2];
    long long batched = 0;
    const char* trace_path = getenv("YOUTH_SLAM_TRACE");
    const int trace_cap = 1 << 20;
    if (trace_path && youth_slam_trace_enable(trace_cap) != 0) return 7;
    for (int p = 0; p < passes; ++p) {
        resetSlam();
        youth_slam_wait_idle(20000);
        const long long b0 = youth_slam_batched_frames();
        const double t0 = now_s();
        double in_push = 0.0;
        for (int k = 0; k < n; ++k) {
            while (youth_slam_queue_size() >= 10) {
            }
            const double tp = now_s();
            if (processSlamFrame(frames + (size_t)k * N, NULL, W, H, (uint32_t)k) != 1) return 5;
            in_push += now_s() - tp;
        }
        while (youth_slam_trajectory_length() < n) {
        }
        win[p][0] = t0;
        win[p][1] = now_s();
        rate[p] = n / (win[p][1] - t0);
        push_us[p] = in_push * 1e6 / n;
        batched += youth_slam_batched_frames() - b0;
    }
    if (trace_path) {
        double* tt = (double*)malloc(trace_cap * sizeof(double));
        int* tk = (int*)malloc(trace_cap * sizeof(int));
        int* ta = (int*)malloc(trace_cap * sizeof(int));
        if (!tt || !tk || !ta) return 3;
        int ne = youth_slam_trace_read(trace_cap, tt, tk, ta);
        if (ne > trace_cap) ne = trace_cap;
        youth_slam_trace_enable(0);
        FILE* f = fopen(trace_path, "w");
        if (!f) return 8;
        for (int p = 0; p < passes; ++p) fprintf(f, "# pass %d %.9f %.9f\n", p, win[p][0], win[p][1]);
        for (int i = 0; i < ne; ++i) fprintf(f, "%.9f %d %d\n", tt[i], tk[i], ta[i]);
        fclose(f);
        free(tt);
        free(tk);
        free(ta);
    }
    const int got = youth_slam_get_trajectory(n, NULL, T);
    double sum = 0.0;
    for (int i = 0; i < got * 16; ++i) sum += T[i];
    resetSlam();
    youth_slam_wait_idle(20000);
    const int nl = n < 60 ? n : 60;
    double* lt0 = (double*)malloc((size_t)nl * 2 * sizeof(double));
    if (!lt0) return 3;
    if (trace_path && youth_slam_trace_enable(trace_cap) != 0) return 7;
    for (int k = 0; k < nl; ++k) {
        const double t0 = now_s();
        processSlamFrame(frames + (size_t)k * N, NULL, W, H, (uint32_t)k);
        while (youth_slam_trajectory_length() < k + 1) {
        }
        const double t1 = now_s();
        lat[k] = (t1 - t0) * 1e6;
        lt0[2 * k] = t0;
        lt0[2 * k + 1] = t1;
    }
    if (trace_path) {
        // the live frames' events: <file>.live, one "# live k t0 t1" line per frame
        double* tt = (double*)malloc(trace_cap * sizeof(double));
        int* tk = (int*)malloc(trace_cap * sizeof(int));
        int* ta = (int*)malloc(trace_cap * sizeof(int));
        if (!tt || !tk || !ta) return 3;
        int ne = youth_slam_trace_read(trace_cap, tt, tk, ta);
        if (ne > trace_cap) ne = trace_cap;
        youth_slam_trace_enable(0);
        char lp[4096];
        snprintf(lp, sizeof(lp), "%s.live", trace_path);
        FILE* f = fopen(lp, "w");
        if (!f) return 8;
        for (int k = 0; k < nl; ++k) fprintf(f, "# live %d %.9f %.9f\n", k, lt0[2 * k], lt0[2 * k + 1]);
        for (int i = 0; i < ne; ++i) fprintf(f, "%.9f %d %d\n", tt[i], tk[i], ta[i]);
        fclose(f);
        free(tt);
        free(tk);
        free(ta);
    }
    free(lt0);
    stopSlamModule();
    double sorted[64];
    memcpy(sorted, rate, (size_t)passes * sizeof(double));
    qsort(sorted, (size_t)passes, sizeof(double), cmp_d);
    qsort(lat + 1, (size_t)(nl - 1), sizeof(double), cmp_d);
    printf("{\"frames\": %d, \"width\": %d, \"height\": %d, \"value\": %.1f, \"unit\": \"frames/s\", "
           "\"pass_values\": [",
           n, W, H, sorted[passes / 2]);
    for (int p = 0; p < passes; ++p) printf("%s%.1f", p ? ", " : "", rate[p]);
    printf("], \"push_us_per_frame\": [");
    for (int p = 0; p < passes; ++p) printf("%s%.1f", p ? ", " : "", push_us[p]);
    printf("], \"pass_windows_s\": [");
    for (int p = 0; p < passes; ++p) printf("%s[%.6f, %.6f]", p ? ", " : "", win[p][0], win[p][1]);
    printf("], \"batched_frames\": %lld, \"frames_recorded\": %d, \"pose_checksum\": %.17g, "
           "\"live_latency_us_median\": %.1f, \"live_latency_us_p90\": %.1f, "
           "\"producer\": \"one C thread, processSlamFrame\"}\n",
           batched, got, sum, lat[1 + (nl - 1) / 2], lat[1 + (int)(0.9 * (nl - 2))]);
    free(frames);
    free(lat);
    free(T);
    return got == n ? 0 : 6;
}
