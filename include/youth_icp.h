/*
 * youth_icp.h — C-ABI of the MI355X-native RGBD frame-to-frame ICP path.
 *
 * This library drops in behind the reference's AlgorithmModule slot
 * (SeunghwanByun/SLAM-RGBD, Youth.Source/AlgorithmModule/).  Two groups of
 * entry points:
 *
 *   1. The reference's own C API, same names / argument meaning / return
 *      convention, so existing callers link unchanged:
 *        - SLAM.h:11-38        initSlamModule .. resetSlam
 *        - algorithmModule.h:6 algorithmModule (pthread start routine)
 *      Return convention (SLAM.h:21,26,30; SLAM.cpp:127-129,178-181):
 *      int 1 = success, 0 = failure / not running.  Nothing throws across
 *      this boundary; errors are logged to stderr.
 *
 *   2. An additive batch / device API (build-only; SURVEY §8b last row) used
 *      by the multi-pair configs and the benchmark.  These return
 *      YOUTH_OK (0) or a negative YOUTH_E* code.
 *
 * Plain C99: no torch types, no HIP types (streams travel as void*).
 * Caller-owned host buffers are borrowed for the duration of the call only
 * (SLAM.cpp:133-148 copies before returning); the library owns all device
 * memory it allocates.
 */
#ifndef YOUTH_ICP_H
#define YOUTH_ICP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------ */
/* Types                                                                     */
/* ------------------------------------------------------------------------ */

/* Pinhole intrinsics + depth scale.  Defaults follow
 * AlgorithmModule/config/astra_orb_slam3_rgbd.yaml:9-12,35 (fx=fy=570.3,
 * cx=320, cy=240, DepthMapFactor=1000) and, for any W x H, the viewer's
 * convention viewerModule.c:343-345 (f = 570.3, c = (W/2, H/2) integer). */
typedef struct youth_intrinsics {
    float fx, fy, cx, cy;
    float depth_scale; /* depth units per metre (1000 = millimetres) */
} youth_intrinsics;

/* ICP parameters (this build's spec; the reference has no ICP). */
typedef struct youth_icp_params {
    int   iters;        /* fixed Gauss-Newton iterations, no early exit */
    float dist_thresh;  /* correspondence gate |P' - P_t| < dist_thresh (m) */
} youth_icp_params;

/* Per-pair status bits returned by the batch API. */
#define YOUTH_STATUS_OK          0
#define YOUTH_STATUS_DEGENERATE  1 /* an iteration's 6x6 system was singular: update skipped */
#define YOUTH_STATUS_FEW_MATCHES 2 /* an iteration had < 6 correspondences: update skipped */
#define YOUTH_STATUS_TIMEOUT     4 /* an align kernel hit its spin bound (never expected) */

/* Return codes of the additive API. */
#define YOUTH_OK        0
#define YOUTH_EINVAL   -1 /* bad argument */
#define YOUTH_ENOMEM   -2 /* device / host allocation failed */
#define YOUTH_EHIP     -3 /* a HIP runtime call failed (see youth_icp_last_error) */
#define YOUTH_ENODEV   -4 /* no HIP device visible */

/* Number of fp64 values in one normal-equation record:
 * [0..20] upper triangle of J^T J (row-major, i<=j), [21..26] J^T r,
 * [27] sum r^2, [28] correspondence count. */
#define YOUTH_NEQ 29

typedef struct youth_icp_ctx youth_icp_ctx;

/* ------------------------------------------------------------------------ */
/* 1. Reference API (drop-in)                                                */
/* ------------------------------------------------------------------------ */

/* Replaces SLAM.h:11 / SLAM.cpp:67-95.  Parses Camera.fx/fy/cx/cy/width/height
 * and DepthMapFactor from the YAML at config_file (NULL or unreadable file:
 * viewer defaults).  vocabulary_file is accepted and ignored (no ORB
 * vocabulary in an ICP tracker).  Starts the private worker thread. */
void initSlamModule(const char* config_file, const char* vocabulary_file);

/* Replaces SLAM.h:14 / SLAM.cpp:97-124: stop the worker, drop the queue. */
void stopSlamModule(void);

/* Replaces SLAM.h:22 / SLAM.cpp:126-175.  Copies depth (int16 mm, 0 =
 * invalid) into the bounded ingest queue (size > 10 -> drop oldest down to 5,
 * SLAM.cpp:163-168) and returns 1; 0 when not running or on bad arguments.
 * color_data may be NULL (ICP does not use colour). */
int processSlamFrame(const int16_t* depth_data, const uint8_t* color_data,
                     int width, int height, uint32_t timestamp);

/* Replaces SLAM.h:27 / SLAM.cpp:177-198: writes "<map_file>_trajectory.txt"
 * (TUM: ts tx ty tz qx qy qz qw).  ts is the caller's timestamp in ms
 * printed as-is (the reference passes ms as "seconds", SLAM.cpp:151). */
int saveSlamMap(const char* map_file);

/* Replaces SLAM.h:31. */
int isSlamModuleRunning(void);

/* Replaces SLAM.h:35: number of valid 3-D points in the latest tracked frame. */
int getSlamMapPoints(void);

/* Replaces SLAM.h:38: clear the trajectory and the reference frame. */
void resetSlam(void);

/* Replaces algorithmModule.h:6 (algorithmModule.c:3-5 calls an undefined
 * SLAM()).  pthread start routine: starts the module if it is not running
 * (arg, if non-NULL, is a const char* config path), then blocks until
 * stopSlamModule() and returns NULL. */
void* algorithmModule(void* id);

/* ------------------------------------------------------------------------ */
/* 2. Additive API                                                           */
/* ------------------------------------------------------------------------ */

/* Viewer-convention intrinsics for W x H (f = 570.3, c = (W/2, H/2)). */
youth_intrinsics youth_default_intrinsics(int width, int height);
youth_icp_params youth_default_params(void);

/* Human-readable text of the last error on this thread ("" if none). */
const char* youth_icp_last_error(void);

/* Number of visible HIP devices (0 when none; never fails). */
int youth_icp_device_count(void);

/* 1 when this context's back-projection divides use the 2-instruction
 * sequence (proven equal to IEEE division on the whole pixel x depth domain
 * by an on-device exhaustive check at creation), 0 for the IEEE path.
 * Environment YOUTH_ICP_NO_FASTDIV=1 forces the IEEE path. */
int youth_icp_fastdiv_enabled(youth_icp_ctx* ctx);

/* Arithmetic of spec a7/a8 (association, residual, Jacobian):
 *   YOUTH_SPEC_SURVEY (default) SURVEY.md §8a a7/a8 + §7 word for word:
 *                     products and sums rounded separately in a fixed order
 *                     (no FMA), the projection quotient fx P'x / P'z an IEEE
 *                     division;
 *   YOUTH_SPEC_FMA    opt-in: fma chains and one correctly rounded
 *                     reciprocal 1/P'z (~6 % faster k_icp; poses move by up
 *                     to ~1e-5 against the survey spec).
 * Both are bit-exact (indices) against the oracle run in the same spec
 * (oracle_set_spec).  youth_icp_set_spec selects one for the context's later
 * aligns and returns the previous spec (EINVAL for another value); the
 * environment YOUTH_ICP_SPEC=survey|fma sets a new context's (and therefore
 * the SLAM.h worker's and the host batch API's) initial spec. */
#define YOUTH_SPEC_FMA    0
#define YOUTH_SPEC_SURVEY 1
int youth_icp_set_spec(youth_icp_ctx* ctx, int spec);
int youth_icp_get_spec(const youth_icp_ctx* ctx);

/* Reduction of spec a9 (the 28 sums of J J^T, J r, r^2):
 *   YOUTH_REDUCE_EXACT (default) every product of two fp32 values exact in
 *                     fp64 (one fp64 fma per product), accumulated in fp64.
 *                     Launch-independent: the same pair aligned in any batch
 *                     size, shard, chunking or kernel path gives the same pose
 *                     up to fp64 summation order (~1e-16 relative), within
 *                     1e-5 of the CPU oracle at SURVEY §8d noise;
 *   YOUTH_REDUCE_LANE32 opt-in: each GPU lane sums its matched pixels' 28
 *                     products with one fp32 fma each over its whole share of
 *                     an iteration, converts them to fp64 once, and the lanes
 *                     are added in fp64 (fixed order); ~10 % faster k_icp.
 *                     Its results depend on the launch's lane partition (pairs
 *                     per launch, chunking, shard count, YOUTH_ICP_BATCH_CHUNK,
 *                     persistent vs cooperative kernel): they are
 *                     bit-reproducible only for the same launch shape, and
 *                     at SURVEY §8d noise a pose can move by up to ~5e-5.
 * youth_icp_set_reduce returns the previous mode (EINVAL for another value);
 * the environment YOUTH_ICP_REDUCE=lane32|exact sets a new context's initial
 * mode.  youth_icp_get_lanes reports how the last align partitioned each
 * iteration's source pixels into lanes (the oracle's oracle_set_reduce
 * restates a LANE32 iteration exactly given that partition); it returns
 * YOUTH_EINVAL when the last call ran launches of more than one partition
 * (a pipelined youth_icp_align_batch whose chunks took different kernels):
 *   YOUTH_LANES_STRIDED   workgroups of `threads` lanes own chunks of `chunk`
 *                         pixels; in each step of 4 threads pixels, lane l
 *                         takes pixels 4l .. 4l+3 (k_icp, k_reduce);
 *   YOUTH_LANES_COOP      workgroup c owns [c npx threads, (c+1) npx threads),
 *                         lane t the pixels c npx threads + s threads + t;
 *   YOUTH_LANES_COOP_TILE workgroup c owns target tile c (64 x npx threads/64
 *                         pixels, raster order), lane t the tile pixels
 *                         k = s threads + t. */
#define YOUTH_REDUCE_EXACT  0
#define YOUTH_REDUCE_LANE32 1
#define YOUTH_LANES_STRIDED   0
#define YOUTH_LANES_COOP      1
#define YOUTH_LANES_COOP_TILE 2
typedef struct youth_lanes {
    int kind, chunk, threads, npx;
} youth_lanes;
int youth_icp_set_reduce(youth_icp_ctx* ctx, int mode);
int youth_icp_get_reduce(const youth_icp_ctx* ctx);
int youth_icp_get_lanes(const youth_icp_ctx* ctx, youth_lanes* out);

/* Concurrent batch aligns on one device (build-only; no SLAM.h counterpart).
 * A caller that keeps `contexts` contexts' persistent aligns in flight at
 * once on the same GPU (e.g. two steps of small batches on two streams)
 * declares it on each of them: the persistent k_icp then runs on
 * 1/contexts of the resident workgroup slots with 1/contexts of the work
 * chunks, so the launches run side by side instead of each waiting for the
 * other's slots (DESIGN.md §5 "Small shards").  Results are unchanged
 * except in the last bits of the sums (their chunking differs).  1 (default)
 * .. YOUTH_ICP_MAX_CONCURRENCY; returns the previous value, EINVAL
 * otherwise.  The small-batch cooperative kernel is not affected. */
#define YOUTH_ICP_MAX_CONCURRENCY 4
int youth_icp_set_concurrency(youth_icp_ctx* ctx, int contexts);

/* One-shot host API:  aligns n_pairs independent pairs; src and
 * dst are [n_pairs][H][W] int16 host arrays.  T_out: [n_pairs][16] row-major
 * fp32 4x4 with P_dst = T * P_src.  assoc_out: nullable [n_pairs][H*W] int32
 * final-iteration correspondence index (v'*W+u') or -1.  Uses device 0 and a
 * cached context; batches of >= 32 pairs are pipelined in 16-pair chunks
 * (H2D of chunk k overlaps the align of chunk k-1).  Returns YOUTH_OK even
 * when a pair's solve was skipped: per-pair status (YOUTH_STATUS_*) is
 * reported by youth_icp_align_batch_multi's status_out.  A chunk whose
 * cooperative launch timed out (a GPU shared with another process: the grid
 * was not co-resident) is aligned again on the persistent kernel before the
 * call returns, so neither call hands out a TIMEOUT pose (stderr says so). */
int youth_icp_align_batch(const int16_t* src, const int16_t* dst, int n_pairs,
                          int W, int H, const youth_intrinsics* K, int iters,
                          float* T_out, int32_t* assoc_out);

/* Multi-GPU host API (SURVEY §8e, C4 from a plain-C host such as main.c): the
 * n_pairs pairs are split into contiguous shards, one per device
 * (youth_icp_shard_range: the first n_pairs % k shards get one pair more),
 * each aligned by its own host thread on its own cached context and stream
 * (pipelined as youth_icp_align_batch), and every shard's poses land in its
 * rows of T_out: the pose gather is the per-device D2H into the caller's
 * buffer, no collective.  devices: nullable list of n_devices distinct device
 * ids (NULL or n_devices <= 0: every visible device); at most n_pairs devices
 * are used.  status_out: nullable [n_pairs] int32 YOUTH_STATUS_* per pair
 * (TIMEOUT folded in).  Blocks until every shard is done; on error returns
 * the first failing shard's code, youth_icp_last_error naming its device.
 * Multi-process (one process per GPU, RCCL gather): see INTEGRATION.md. */
int youth_icp_align_batch_multi(const int16_t* src, const int16_t* dst, int n_pairs,
                                int W, int H, const youth_intrinsics* K, int iters,
                                const int* devices, int n_devices, float* T_out,
                                int32_t* status_out);

/* Shard `part` of n_pairs split over n_parts: *first and *count (the split
 * youth_icp_align_batch_multi and the bench's ranks use). */
int youth_icp_shard_range(int n_pairs, int n_parts, int part, int* first, int* count);

/* Context: device workspace sized for max_frames frames of W x H (target
 * records + depth staging); 3 <= W, H <= 16384 and W*H <= 2^26 (EINVAL
 * otherwise).  The pair API needs n_pairs <= max_frames, the
 * sequence API n_frames - 1 <= max_frames, the one-shot host API stages
 * 2 * n_pairs depth frames. */
youth_icp_ctx* youth_icp_create(int device, int W, int H, int max_frames,
                                const youth_intrinsics* K,
                                const youth_icp_params* P);
void youth_icp_destroy(youth_icp_ctx* ctx);

/* Device-resident align of n_pairs pairs.  d_src / d_dst: device pointers to
 * [n_pairs][H][W] int16 (d_src is read by every iteration: keep it alive and
 * unmodified until the align has completed on `stream`).  T_init: nullable HOST [n_pairs][16] fp64 (identity
 * if NULL; every entry must be finite, else YOUTH_EINVAL).  d_T_out: nullable DEVICE [n_pairs][16] fp32.  stream: a
 * hipStream_t as void* (NULL = the context's own stream).  Asynchronous:
 * returns after enqueueing; use youth_icp_sync / youth_icp_get_poses.  One
 * context's aligns must execute in order (one stream, or ordered by the
 * caller): they share its workspace and per-call hand-off state.  Small
 * batches run as one cooperative launch (youth_icp_get_plan): its
 * workgroups wait on each other, so the whole grid must be co-resident.  It
 * is launched as a plain kernel sized to an idle device, with every such
 * launch of the process ordered per device; that assumes this process owns
 * the GPU (no other process's kernels holding CUs meanwhile).  On a shared
 * GPU set YOUTH_ICP_COOP_LAUNCH=runtime (hipLaunchCooperativeKernel: the
 * runtime admits the grid or refuses it, and a refusal falls back to the
 * persistent kernel) or YOUTH_ICP_NO_COOP=1; a grid that is not co-resident
 * ends at the spin bound with YOUTH_STATUS_TIMEOUT, never a hang.  The
 * first cooperative launch of the process from a second stream on a device
 * waits once for that device to drain (hipDeviceSynchronize, without
 * holding any lock: other threads' cooperative launches on the device wait
 * for it, nothing else does); it fails (YOUTH_EHIP) if a stream on the
 * device is being captured at that moment.  Later stream switches only
 * order the launches through an event. */
int youth_icp_align_pairs_device(youth_icp_ctx* ctx, const int16_t* d_src,
                                 const int16_t* d_dst, int n_pairs,
                                 const double* T_init, float* d_T_out,
                                 void* stream);

/* Streamed-sequence align (config C5): d_frames [n_frames][H][W] int16 on
 * device; computes the n_frames-1 relative poses T_k (P_k = T_k P_{k+1});
 * every frame is back-projected and normal-estimated once. */
int youth_icp_align_sequence_device(youth_icp_ctx* ctx, const int16_t* d_frames,
                                    int n_frames, float* d_T_out, void* stream);

/* Block until the context's last enqueued work on `stream` is done. */
int youth_icp_sync(youth_icp_ctx* ctx, void* stream);

/* Copy results of the last align to host (synchronises).  T64: [n][16] fp64
 * (nullable), T32: [n][16] fp32 (nullable), status: [n] int32 (nullable). */
int youth_icp_get_poses(youth_icp_ctx* ctx, int n, double* T64, float* T32,
                        int32_t* status);

/* Per-iteration diagnostics of the last align: [n][iters] correspondence
 * counts and sums of squared residuals (nullable). */
int youth_icp_get_stats(youth_icp_ctx* ctx, int n, int iters, double* count,
                        double* sum_r2);

/* Kernel timing (HIP events on the launch stream; for bench.py's roofline).
 * enable=1: around every iteration-kernel launch (kind 0), solve (1) and prep
 * (2) launch; enable=2: around the iteration kernel only (fewer markers in a
 * timed region); 0: off.  Any call resets the counters. */
int youth_icp_set_timing(youth_icp_ctx* ctx, int enable);
/* total_ms / launches of reduction (kind 0), solve (1), frame-prep (2). */
int youth_icp_get_timing(youth_icp_ctx* ctx, int kind, double* total_ms,
                         int* launches);

/* Scheduler telemetry of the LAST persistent align on this context: total
 * epoch polls (each followed by s_sleep 8) and the number of work items that
 * had to wait for their pair's previous-iteration pose.  Synchronises the
 * context stream.  Zero for the per-iteration (non-persistent) path. */
int youth_icp_get_sched_stats(youth_icp_ctx* ctx, unsigned* spins,
                              unsigned* waited_items);

/* Kernel path of the last align on this context (build-only, reporting):
 * returns 1 when it ran the small-batch cooperative kernel (k_icp_coop:
 * *workgroups_per_pair x 512 threads, *px_per_lane source pixels per lane,
 * target prep fused), 0 for the persistent batch kernel (k_prep + k_icp),
 * 2 for the per-iteration fallback (YOUTH_ICP_NO_PERSISTENT=1: k_prep, k_init,
 * then one k_reduce with the fused last-workgroup solve per iteration),
 * negative on error.  Either pointer may be NULL. */
int youth_icp_get_plan(youth_icp_ctx* ctx, int* workgroups_per_pair, int* px_per_lane);

/* Validation of the projection reciprocal rz = RN(1 / z') the kernels form
 * from v_rcp_f32 plus correction steps: *bit_mismatches counts bitwise
 * differences from IEEE 1.0f / den over EVERY fp32 den in the guarded range
 * [2^-60, 2^60] (must be 0); *proj_mismatches counts differences of the
 * projected pixel floor(fma(num, rz, c + 0.5)) or its in-range test against
 * the IEEE reciprocal's on n pseudo-random (seeded) cases (must be 0). */
int youth_icp_selftest_projdiv(int device, long long n, unsigned long long seed,
                               long long* bit_mismatches, long long* proj_mismatches);

/* Validation of YOUTH_SPEC_SURVEY's projection (the correctly rounded
 * reciprocal plus ONE correction step for the quotient, one
 * v_cvt_flr_i32_f32 for the floor) against IEEE num / den and floorf:
 * *quot_mismatches bitwise on n seeded cases with den in [2^-60, 2^60], half
 * of them next to a rounding midpoint; *proj_mismatches of the projected
 * pixel floor((q + c) + 0.5) or its in-range test on n cases, den over the
 * whole positive range; *floor_mismatches of the one-instruction floor over
 * all 2^32 bit patterns (NaN and denormals excluded: the projection never
 * forms them).  All must be 0. */
int youth_icp_selftest_projquot(int device, long long n, unsigned long long seed,
                                long long* quot_mismatches, long long* proj_mismatches,
                                long long* floor_mismatches);

/* Self-test of the target-normal normalisation's fast path (correctly rounded
 * sqrt without rescaling, three quotients sharing one reciprocal) against
 * IEEE sqrtf and division: *sqrt_mismatches over every fp32 in [2^-96, 2^118]
 * (must be 0), *quot_mismatches bitwise over n random vectors that take the
 * fast path (must be 0), *fast_cases = how many did. */
int youth_icp_selftest_normalize(int device, long long n, unsigned long long seed,
                                 long long* sqrt_mismatches, long long* quot_mismatches,
                                 long long* fast_cases);

/* --- Stage-level entry points (validation / parity tests) --------------- */

/* Depth -> XYZ planes (+ normals when want_normals) for n_frames host frames.
 * Outputs are HOST arrays [n_frames][H*W] each (any may be NULL).  With X, Y
 * and Z all NULL the records come from the align path's record kernel (no
 * planes stored), else from the same kernel storing the planes too. */
int youth_icp_prepare_host(youth_icp_ctx* ctx, const int16_t* depth,
                           int n_frames, int want_normals, float* X, float* Y,
                           float* Z, float* NX, float* NY, float* NZ);

/* One association + reduction pass for one pair at a GIVEN fp32 pose
 * T12 (3x4 row-major).  src/dst host depth frames.  assoc: nullable
 * [H*W] int32; neq: nullable [YOUTH_NEQ] fp64. */
int youth_icp_reduce_host(youth_icp_ctx* ctx, const int16_t* src,
                          const int16_t* dst, const float* T12, int32_t* assoc,
                          double* neq);

/* Solve one normal-equation record on the device and apply the SE(3)
 * update to T64 (4x4 row-major fp64, in/out).  Returns status bits >= 0 or
 * a negative YOUTH_E* code. */
int youth_icp_solve_host(youth_icp_ctx* ctx, const double* neq, double* T64);

/* --- Frame-to-frame tracking (the SLAM API's worker uses this) ----------- */

/* Upload one host depth frame into the context's 2-slot ring, back-project
 * it with normals and, when a reference frame is held, align it (source) to
 * the reference (target) with T_init (nullable host fp64 4x4; identity if
 * NULL; finite, else YOUTH_EINVAL and the frame is dropped).  The new frame
 * then becomes the reference.  T_rel (host fp64 4x4):
 * P_ref = T_rel * P_new, identity for the first frame (*has_ref = 0).
 * Returns status bits (>= 0) or a negative YOUTH_E* code.  Synchronous. */
int youth_icp_track_frame(youth_icp_ctx* ctx, const int16_t* depth,
                          const double* T_init, double* T_rel, int* has_ref);

/* Pipelined form of youth_icp_track_frame (the SLAM API's worker uses it):
 * youth_icp_track_submit copies the host frame into a pinned staging buffer
 * (the caller's buffer is free on return), enqueues its H2D on a transfer
 * stream and its align (against the frame submitted before it) on the
 * context's stream, and returns without waiting, so the next frame's copy
 * overlaps the aligns in flight.  At most YOUTH_TRACK_MAX_IN_FLIGHT frames
 * may be in flight (YOUTH_EINVAL otherwise): two suffice one frame at a
 * time; two micro-batches (youth_icp_track_submit_batch) use up to 16.
 * youth_icp_track_collect waits for the OLDEST
 * submitted frame and returns exactly what youth_icp_track_frame would have
 * returned for it (status bits or a negative code, T_rel, *has_ref).
 * youth_icp_track_frame = submit + collect, with nothing in flight.
 * collect polls the frame's completion event for up to 2 ms, then blocks in
 * the runtime (YOUTH_ICP_TRACK_WAIT=sync: block at once).
 * Each frame in flight pins one staging frame of host memory (W x H x 2
 * bytes: 614 KB at 640x480), allocated the first time the ring needs that
 * many and freed by youth_icp_destroy. */
#define YOUTH_TRACK_MAX_IN_FLIGHT 16
int youth_icp_track_submit(youth_icp_ctx* ctx, const int16_t* depth,
                           const double* T_init);
int youth_icp_track_collect(youth_icp_ctx* ctx, double* T_rel, int* has_ref);
/* Frames submitted and not yet collected (0 .. YOUTH_TRACK_MAX_IN_FLIGHT). */
int youth_icp_track_pending(const youth_icp_ctx* ctx);

/* What a tracked frame's status bits mean for its pose, and what to do:
 *   YOUTH_STATUS_TIMEOUT      the align's cooperative grid was not co-resident
 *                             (another process held CUs; k_icp_coop is launched
 *                             as a plain kernel sized to an idle device) and its
 *                             waits hit their spin bound: T_rel is a partly
 *                             iterated pose and MUST NOT be used.  The frame's
 *                             records (the next reference) are complete
 *                             nevertheless: every workgroup preps its tiles
 *                             before it waits, so the frames after it are
 *                             unaffected.  Re-align it with
 *                             youth_icp_track_realign (the SLAM worker and
 *                             youth_icp_track_host_sequence do).
 *   YOUTH_STATUS_FEW_MATCHES  some iteration had < 6 correspondences, or
 *   YOUTH_STATUS_DEGENERATE   its 6x6 system was singular: that iteration's
 *                             update was skipped, the others were applied.
 *                             T_rel is the pose the remaining updates reached
 *                             (identity when none was applied: the "no motion"
 *                             estimate).  It is a valid, if weak, estimate: the
 *                             SLAM worker composes it into the trajectory and
 *                             records the status beside the pose
 *                             (youth_slam_get_status).
 *
 * youth_icp_track_realign aligns depth (source, the timed-out frame) to
 * ref_depth (target, the frame tracked before it), host int16 frames of the
 * context's size, synchronously, and returns the status bits (>= 0) with
 * T_rel (fp64 4x4, P_ref = T_rel P_new) or a negative YOUTH_E* code.  It
 * first waits for everything the tracker has in flight (their results stay
 * collectable), then runs the context's single-pair cooperative plan, which
 * reproduces the undisturbed tracker's pose bit for bit; if that times out
 * too, the persistent kernel, which needs no co-residency (the same pose up to
 * fp64 summation order, ~1e-16 relative).  The tracker's reference and its
 * frames in flight are not disturbed.  youth_icp_track_realigned counts the
 * successful realigns on the cooperative plan (returned), on the persistent
 * kernel (*persistent) and realigns that still timed out (*failed). */
int youth_icp_track_realign(youth_icp_ctx* ctx, const int16_t* ref_depth,
                            const int16_t* depth, const double* T_init, double* T_rel);
long long youth_icp_track_realigned(const youth_icp_ctx* ctx, long long* persistent,
                                    long long* failed);

/* Micro-batch of n_frames consecutive host frames ([n_frames][H][W]) for a
 * backlogged stream: the same as n_frames youth_icp_track_submit calls
 * (T_init identity), each frame collected by its own youth_icp_track_collect
 * with exactly the result youth_icp_track_frame gives, bit for bit.  When the
 * context holds a reference and has room (max_frames >= 2 m for a chain of
 * m frames), consecutive frames are aligned by ONE cooperative launch in
 * which pair i (frame i against frame i - 1, frame -1 = the reference) runs
 * on the single-pair plan and waits for the pair before it to have prepped
 * its target, as many frames per launch as that plan's grids fit on the
 * chip (youth_icp_track_set_batch(ctx, m) plans for m; the default plan at
 * 640x480 holds one pair); the rest one launch per frame.
 * 1 <= n_frames <= YOUTH_TRACK_MAX_BATCH, and at most
 * YOUTH_TRACK_MAX_IN_FLIGHT frames in flight afterwards (EINVAL).
 * The frames are copied into page-locked staging before the call returns;
 * from 1 MiB per call the copy is split over the calling thread and the
 * context's helper threads (3, started by the first such call;
 * YOUTH_ICP_COPY_THREADS=k sets k, 0 copies on the calling thread only). */
#define YOUTH_TRACK_MAX_BATCH 8
int youth_icp_track_submit_batch(youth_icp_ctx* ctx, const int16_t* depth, int n_frames);

/* youth_icp_track_submit_batch without the staging copy: frames[i] (n_frames
 * pointers) are page-locked host frames the caller allocated with
 * youth_icp_host_alloc and keeps unchanged until frame i has been collected;
 * their H2D copies read them in place.  The SLAM worker submits the ingest
 * queue's buffers this way, so a frame is copied once on the host (in
 * processSlamFrame).  Same results and limits as youth_icp_track_submit_batch. */
int youth_icp_track_submit_pinned(youth_icp_ctx* ctx, const int16_t* const* frames,
                                  int n_frames);
/* Page-locked host memory for `values` int16 values (NULL on failure or 0),
 * and its release (NULL is ignored). */
int16_t* youth_icp_host_alloc(size_t values);
void youth_icp_host_free(int16_t* p);

/* Frames per submission youth_icp_track_host_sequence uses (1, default: one
 * launch per frame; up to YOUTH_TRACK_MAX_BATCH: micro-batches).  Batch mode
 * (> 1) plans the context's cooperative launches with the fewest source
 * pixels per lane that let that many pairs share one grid on the chip less
 * 32 CUs (kept free for the next micro-batch's frame pull, k_pull_frames;
 * YOUTH_ICP_PULL_RESERVE_CU overrides; 640x480: 6, 9, 11 and 22 px per lane
 * for 2, 3, 4 and 8 frames), so results stay bit-identical between
 * batched and per-frame submission on that context (and within 1e-13 of the
 * oracle, like the default plan).
 * Returns the previous value or YOUTH_EINVAL. */
int youth_icp_track_set_batch(youth_icp_ctx* ctx, int frames);
/* Micro-batch launches this context has run (a batch that did not fit one
 * grid runs as per-frame launches and is not counted). */
long long youth_icp_track_chained(const youth_icp_ctx* ctx);
/* Frames those micro-batch launches aligned (the first frame of a sequence,
 * prepped alone, and frames that ran one launch each are not counted). */
long long youth_icp_track_chained_frames(const youth_icp_ctx* ctx);

/* A recorded host sequence (frames [n_frames][H][W], e.g. a .bin playback)
 * through the tracker, two frames in flight (with youth_icp_track_set_batch(m):
 * two micro-batches of m): the same results as
 * youth_icp_track_frame on each frame in order (continuing from the
 * reference the context holds).  T_rel [n][16] and status [n] (nullable)
 * receive the frames that had a reference, in order; returns how many, or a
 * negative YOUTH_E* code (nothing left in flight either way).  A frame
 * k >= 1 whose align timed out is realigned against frame k - 1
 * (youth_icp_track_realign), so its entry is the undisturbed result. */
int youth_icp_track_host_sequence(youth_icp_ctx* ctx, const int16_t* frames, int n_frames,
                                  double* T_rel, int32_t* status);

/* Forget the reference frame (next tracked frame starts a new sequence). */
void youth_icp_track_reset(youth_icp_ctx* ctx);

/* --- Host utilities (no device needed) ----------------------------------- */

/* Reads Camera.fx/fy/cx/cy/width/height and DepthMapFactor from an
 * ORB-SLAM3-style YAML (astra_orb_slam3_rgbd.yaml:9-20,35).  Missing keys keep
 * the values already in *K / *W / *H.  Returns 1 if the file was read, 0 if
 * it could not be opened. */
int youth_parse_camera_yaml(const char* path, youth_intrinsics* K, int* W, int* H);

/* Bounded frame-ingest queue with the reference's overflow policy
 * (SLAM.cpp:159-169: after a push, if size > high_water, drop the oldest until
 * size == low_water; reference values 10 / 5).  Thread-safe.  Frames are
 * copied in and out. */
typedef struct youth_frame_queue youth_frame_queue;
youth_frame_queue* youth_queue_create(int high_water, int low_water);
void youth_queue_destroy(youth_frame_queue* q);
/* Returns the number of frames dropped by this push (>= 0), or YOUTH_E*. */
int youth_queue_push(youth_frame_queue* q, const int16_t* depth, int width,
                     int height, uint32_t timestamp);
/* Pops the oldest frame into depth_out (capacity `cap` int16 values).
 * Returns 1 when a frame was popped, 0 when empty, YOUTH_EINVAL when the
 * frame does not fit (it stays queued). */
int youth_queue_pop(youth_frame_queue* q, int16_t* depth_out, size_t cap,
                    int* width, int* height, uint32_t* timestamp);
int youth_queue_size(youth_frame_queue* q);
void youth_queue_clear(youth_frame_queue* q);

/* --- SLAM-module introspection (additive) ------------------------------- */

/* Number of poses in the trajectory (1 per tracked frame). */
int youth_slam_trajectory_length(void);
/* Copy up to n trajectory entries: timestamps [n] and world poses [n][16]
 * (fp64 row-major, first frame = identity).  Returns the count copied. */
int youth_slam_get_trajectory(int n, uint32_t* timestamps, double* T_wc);
/* Entry `index` of the trajectory: 1 with *timestamp / T_wc[16] filled, 0 if
 * index is out of range. */
int youth_slam_get_pose(int index, uint32_t* timestamp, double* T_wc);
/* Block until the ingest queue is empty and the worker is idle, or
 * timeout_ms elapses.  Returns 1 when drained, 0 on timeout / not running. */
int youth_slam_wait_idle(int timeout_ms);
/* Frames the worker has aligned in chained micro-batch launches since the
 * module started (youth_icp_track_chained_frames of its context: frames of
 * a backlogged queue; 0 when every frame arrived alone or with
 * YOUTH_SLAM_TRACK_BATCH=1). */
long long youth_slam_batched_frames(void);
/* Aligns the worker found timed out (YOUTH_STATUS_TIMEOUT) and realigned
 * (youth_icp_track_realign): returns those the cooperative plan completed
 * (bit-identical to an undisturbed run), *persistent those the persistent
 * kernel completed, *lost those that still timed out.  A timed-out pose is
 * never composed into the trajectory: a lost frame is left out of it, and the
 * next frame composes onto the last recorded pose (no motion across the lost
 * frame).  Counted since the module started. */
long long youth_slam_realigned(long long* persistent, long long* lost);
/* Status bits (YOUTH_STATUS_FEW_MATCHES / _DEGENERATE, never TIMEOUT) of the
 * first n trajectory entries into status[n] (nullable), and the number of
 * recorded frames with each bit since the module started (nullable).  Such a
 * frame's pose is composed: it is the pose its applied updates reached
 * (youth_icp_track_realign's comment).  Returns the count copied. */
int youth_slam_get_status(int n, int32_t* status, long long* few_matches,
                          long long* degenerate);
/* Frames waiting in the module's ingest queue (processSlamFrame drops the
 * oldest down to 5 when it passes 10, SLAM.cpp:163-168): a producer that
 * must not lose frames waits while this is 10. */
int youth_slam_queue_size(void);
/* Block until the module stops (used by algorithmModule). */
void youth_slam_wait_stopped(void);

/* Event trace of the ingest path (diagnostic, additive): with a capacity > 0
 * the producer (processSlamFrame) and the worker record timestamped events
 * (CLOCK_MONOTONIC seconds, the clock rocprofv3 traces use) into a
 * fixed-size buffer, lock-free; events past the capacity are dropped.
 * youth_slam_trace_enable(0) stops recording and frees the buffer.  Enable
 * or disable at any time (a buffer is freed only after every writer that may
 * hold it has finished).  youth_slam_trace_read copies up to n events (t[n]
 * seconds, kind[n], arg[n]) and returns how many were recorded and finished,
 * in order (at most the capacity; may exceed n).  Kinds and their arg: */
#define YOUTH_SLAM_EV_PUSH_BEGIN    1  /* queue depth before the push */
#define YOUTH_SLAM_EV_PUSH_END      2  /* buffer: 0 pooled, 2 new pageable (1 unused: the
                                          producer never allocates page-locked memory) */
#define YOUTH_SLAM_EV_TAKE          3  /* frames in the micro-batch being formed */
#define YOUTH_SLAM_EV_SUBMIT_BEGIN  4  /* frames submitted */
#define YOUTH_SLAM_EV_SUBMIT_END    5  /* return code */
#define YOUTH_SLAM_EV_COLLECT_BEGIN 6  /* frames in flight */
#define YOUTH_SLAM_EV_COLLECT_END   7  /* 1 the last frame of its submission */
#define YOUTH_SLAM_EV_IDLE_BEGIN    8  /* worker waits for a frame (queue empty) */
#define YOUTH_SLAM_EV_IDLE_END      9  /* queue depth */
#define YOUTH_SLAM_EV_POOL          10 /* worker: page-locked buffers allocated (+) / freed (-) */
#define YOUTH_SLAM_EV_DROP          11 /* frames dropped by the >10 -> 5 policy */
#define YOUTH_SLAM_EV_SUBMIT_STEP   12 /* inside a tracker submission: 1 slots ready, 2 waits
                                          enqueued, 3 H2D copies enqueued, 4 H2D event, 5 launch */
#define YOUTH_SLAM_EV_REALIGN       13 /* a timed-out align realigned: 0 cooperative plan,
                                          1 persistent kernel, 2 lost */
int youth_slam_trace_enable(int capacity);
int youth_slam_trace_read(int n, double* t, int* kind, int* arg);

#ifdef __cplusplus
}
#endif

#endif /* YOUTH_ICP_H */
