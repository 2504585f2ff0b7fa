/*
 * icp_stub.c — TEST INFRASTRUCTURE ONLY: a CPU stand-in for the
 * libyouth_icp device entry points the host-side threading code calls
 * (slam_api.cpp's worker: create / destroy / track_submit / track_collect /
 * track_frame / track_reset / track_submit_batch / track_set_batch /
 * track_chained / track_chained_frames / track_submit_pinned /
 * host_alloc / host_free / device_count / last_error / track_realign /
 * track_realigned, plus youth_default_intrinsics), so the SLAM.h
 * queue + worker, the AlgorithmModule frame loop and the POSIX-queue
 * transport can run under ThreadSanitizer / AddressSanitizer on a machine
 * without a GPU (SURVEY §5 "Race detection").  It is linked only into the
 * sanitizer driver (tests/tsan/Makefile), never into libyouth_icp.so, and
 * computes no ICP: the "relative pose" is a translation derived from the
 * frame's depth sum, enough for the driver to check that every frame reached
 * the trajectory in order.  YOUTH_STUB_TIMEOUT_EVERY=k (read at create)
 * makes every k-th frame with a reference come back YOUTH_STATUS_TIMEOUT with
 * a wrong pose, as a timed-out cooperative align does, so the worker's
 * realign path runs too; youth_icp_track_realign recomputes the pose from the
 * two frames it is given.
 */
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "youth_icp.h"

struct youth_icp_ctx {
    int W, H, has_ref;
    long long ref_sum;
    /* submitted frames' results, oldest first */
    double T[YOUTH_TRACK_MAX_IN_FLIGHT][16];
    int has[YOUTH_TRACK_MAX_IN_FLIGHT], n, head, batch;
    long long chained, chained_frames;
    /* in-place (pinned) submissions: the caller's buffer and its depth sum at
     * submit time, re-read at collect (a buffer reused while its frame is in
     * flight fails the run) */
    const int16_t* src[YOUTH_TRACK_MAX_IN_FLIGHT];
    long long src_sum[YOUTH_TRACK_MAX_IN_FLIGHT];
    int status[YOUTH_TRACK_MAX_IN_FLIGHT];
    int timeout_every, tracked;
    long long realigned;
};

static long long depth_sum(const youth_icp_ctx* c, const int16_t* d)
{
    long long s = 0;
    for (int i = 0; i < c->W * c->H; ++i) s += d[i];
    return s;
}

int16_t* youth_icp_host_alloc(size_t values)
{
    return values ? (int16_t*)malloc(values * sizeof(int16_t)) : NULL;
}

void youth_icp_host_free(int16_t* p) { free(p); }

int youth_icp_device_count(void) { return 1; }
const char* youth_icp_last_error(void) { return "stub"; }

youth_intrinsics youth_default_intrinsics(int width, int height)
{
    youth_intrinsics K = {570.3f, 570.3f, (float)(width / 2), (float)(height / 2), 1000.0f};
    return K;
}

youth_icp_ctx* youth_icp_create(int device, int W, int H, int max_frames,
                                const youth_intrinsics* K, const youth_icp_params* P)
{
    (void)device, (void)max_frames, (void)K, (void)P;
    youth_icp_ctx* c = (youth_icp_ctx*)calloc(1, sizeof(*c));
    if (c) c->W = W, c->H = H;
    const char* e = getenv("YOUTH_STUB_TIMEOUT_EVERY");
    if (c && e) c->timeout_every = atoi(e);
    return c;
}

void youth_icp_destroy(youth_icp_ctx* c) { free(c); }
void youth_icp_track_reset(youth_icp_ctx* c) { c->has_ref = 0; }

static int stub_track(youth_icp_ctx* c, const int16_t* depth, double* T_rel, int* has_ref);

int youth_icp_track_submit(youth_icp_ctx* c, const int16_t* depth, const double* T_init)
{
    (void)T_init;
    if (c->n >= YOUTH_TRACK_MAX_IN_FLIGHT) return YOUTH_EINVAL;
    const int j = (c->head + c->n) % YOUTH_TRACK_MAX_IN_FLIGHT;
    stub_track(c, depth, c->T[j], &c->has[j]);
    c->status[j] = 0;
    if (c->has[j] && c->timeout_every > 0 && ++c->tracked % c->timeout_every == 0) {
        c->status[j] = YOUTH_STATUS_TIMEOUT;
        c->T[j][3] = 1e9; /* a partly iterated pose: must never reach the trajectory */
    }
    c->src[j] = NULL;
    ++c->n;
    return 0;
}

int youth_icp_track_realign(youth_icp_ctx* c, const int16_t* ref_depth, const int16_t* depth,
                            const double* T_init, double* T_rel)
{
    (void)T_init;
    memset(T_rel, 0, 16 * sizeof(double));
    T_rel[0] = T_rel[5] = T_rel[10] = T_rel[15] = 1.0;
    T_rel[3] = (double)(depth_sum(c, depth) - depth_sum(c, ref_depth)) * 1e-6;
    ++c->realigned;
    return 0;
}

long long youth_icp_track_realigned(const youth_icp_ctx* c, long long* persistent, long long* failed)
{
    if (persistent) *persistent = 0;
    if (failed) *failed = 0;
    return c->realigned;
}

int youth_icp_track_collect(youth_icp_ctx* c, double* T_rel, int* has_ref)
{
    if (c->n == 0) return YOUTH_EINVAL;
    struct timespec ts = {0, 200 * 1000}; /* a GPU align takes ~100 us */
    nanosleep(&ts, NULL);
    if (c->src[c->head] && depth_sum(c, c->src[c->head]) != c->src_sum[c->head]) abort();
    memcpy(T_rel, c->T[c->head], 16 * sizeof(double));
    if (has_ref) *has_ref = c->has[c->head];
    const int st = c->status[c->head];
    c->head = (c->head + 1) % YOUTH_TRACK_MAX_IN_FLIGHT;
    --c->n;
    return st;
}

int youth_icp_track_pending(const youth_icp_ctx* c) { return c->n; }

int youth_icp_track_set_batch(youth_icp_ctx* c, int frames)
{
    const int old = c->batch ? c->batch : 1;
    c->batch = frames;
    return old;
}

long long youth_icp_track_chained(const youth_icp_ctx* c) { return c->chained; }
long long youth_icp_track_chained_frames(const youth_icp_ctx* c) { return c->chained_frames; }

/* as the library: a sequence's first frame alone, then one "launch" */
int youth_icp_track_submit_batch(youth_icp_ctx* c, const int16_t* depth, int n_frames)
{
    if (n_frames < 1 || n_frames > YOUTH_TRACK_MAX_BATCH ||
        c->n + n_frames > YOUTH_TRACK_MAX_IN_FLIGHT)
        return YOUTH_EINVAL;
    const int first_alone = !c->has_ref;
    const int chain = n_frames - first_alone > 1;
    for (int i = 0; i < n_frames; ++i)
        youth_icp_track_submit(c, depth + (size_t)i * c->W * c->H, NULL);
    c->chained += chain;
    c->chained_frames += chain ? n_frames - first_alone : 0;
    return 0;
}

int youth_icp_track_submit_pinned(youth_icp_ctx* c, const int16_t* const* frames, int n_frames)
{
    if (n_frames < 1 || n_frames > YOUTH_TRACK_MAX_BATCH ||
        c->n + n_frames > YOUTH_TRACK_MAX_IN_FLIGHT)
        return YOUTH_EINVAL;
    const int first_alone = !c->has_ref;
    const int chain = n_frames - first_alone > 1;
    for (int i = 0; i < n_frames; ++i) {
        const int j = (c->head + c->n) % YOUTH_TRACK_MAX_IN_FLIGHT;
        youth_icp_track_submit(c, frames[i], NULL);
        c->src[j] = frames[i];
        c->src_sum[j] = depth_sum(c, frames[i]);
    }
    c->chained += chain;
    c->chained_frames += chain ? n_frames - first_alone : 0;
    return 0;
}

int youth_icp_track_frame(youth_icp_ctx* c, const int16_t* depth, const double* T_init,
                          double* T_rel, int* has_ref)
{
    (void)T_init;
    struct timespec ts = {0, 200 * 1000};
    nanosleep(&ts, NULL);
    return stub_track(c, depth, T_rel, has_ref);
}

static int stub_track(youth_icp_ctx* c, const int16_t* depth, double* T_rel, int* has_ref)
{
    long long s = 0;
    for (int i = 0; i < c->W * c->H; ++i) s += depth[i];
    memset(T_rel, 0, 16 * sizeof(double));
    T_rel[0] = T_rel[5] = T_rel[10] = T_rel[15] = 1.0;
    if (has_ref) *has_ref = c->has_ref;
    if (c->has_ref) T_rel[3] = (double)(s - c->ref_sum) * 1e-6;
    c->has_ref = 1;
    c->ref_sum = s;
    return 0;
}
