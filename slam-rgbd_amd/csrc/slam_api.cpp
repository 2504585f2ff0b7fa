// slam_api.cpp — drop-in implementation of the reference's SLAM.h C API.
//
// Reference: Youth.Source/AlgorithmModule/SLAM.h:11-38 and SLAM.cpp:15-230.
// Same entry points, argument meaning, 1/0 return convention and threading
// model (caller threads enqueue; ONE private worker thread tracks), but the
// ORB-SLAM3 TrackRGBD call (SLAM.cpp:54) is replaced by HIP frame-to-frame
// point-to-plane ICP (youth_icp_track_submit / _collect, two frames in
// flight).  Host-only C++: no HIP types.
//
// Differences from the reference that are deliberate:
//  - processSlamFrame keeps depth as int16 millimetres (the GPU converts with
//    the viewer's /1000.0f rule, viewerModule.c:343) instead of
//    convertTo(CV_32F, 1/1000) (SLAM.cpp:154-155); colour is ignored (ICP).
//  - every frame path returns a value (SLAM.cpp:172-174 falls off the end).
//  - the running flags are atomics (the reference shares plain bools).

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "host_copy.h"
#include "youth_icp.h"

// ----------------------------------------------------------- event trace --
// youth_slam_trace_enable / _read (youth_icp.h): timestamped events of the
// producer and the worker in a fixed buffer, one fetch_add per event.
// The buffer and its capacity are published together (one pointer), and a
// buffer is freed only once no thread can still be writing into it: a writer
// announces itself in g_tr_active before it loads the pointer it writes
// through, and enable waits for the announced writers after swapping the
// pointer (the worker traces on its own, e.g. idle wake-ups, so "no frame
// being pushed" does not mean "no writer").  A slot is readable
// once its writer has set `ready`.
namespace {

struct TraceEv {
    double t;
    int kind, arg;
    std::atomic<int> ready{0};
};
struct TraceBuf {
    explicit TraceBuf(int n) : cap(n), ev(new TraceEv[n]) {}
    ~TraceBuf() { delete[] ev; }
    const int cap;
    TraceEv* const ev;
    std::atomic<int> claimed{0};  // slots handed out (may pass cap: the buffer is full)
};
std::atomic<TraceBuf*> g_tr{nullptr};
std::atomic<int> g_tr_active{0};  // writers between their announcement and their last store

double mono_s()
{
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

void trace(int kind, int arg)
{
    if (!g_tr.load(std::memory_order_relaxed)) return;  // tracing off: no shared write
    g_tr_active.fetch_add(1);                            // seq_cst: before the load below
    TraceBuf* b = g_tr.load();
    if (b && b->claimed.load(std::memory_order_relaxed) < b->cap) {
        const int i = b->claimed.fetch_add(1, std::memory_order_relaxed);
        if (i < b->cap) {
            TraceEv& e = b->ev[i];
            e.t = mono_s();
            e.kind = kind;
            e.arg = arg;
            e.ready.store(1, std::memory_order_release);
        }
    }
    g_tr_active.fetch_sub(1);
}

}  // namespace

// ------------------------------------------------------- ingest queue -----
// Frames live in reusable buffers: a push copies the caller's frame into a
// free buffer of the queue's pool (the one host copy of a frame on the SLAM
// path), the drop policy and pops hand buffers back to the pool.  The SLAM
// module's queue uses page-locked buffers (youth_icp_host_alloc, up to
// kPinnedBytes of them), which the worker takes out of the queue and submits
// to the tracker in place (youth_icp_track_submit_pinned), returning each to
// the pool once its frame has been collected.
// Page-locked buffers are allocated and freed only off the producer's path
// (initSlamModule and the worker: queue_prefill / queue_release): a
// hipHostMalloc or hipHostFree can take milliseconds and synchronise the
// device, which a camera callback must not wait for.  A producer that finds
// no pooled buffer of the frame's size takes a pageable one (malloc); the
// worker frees it after use and adds a page-locked one to the pool.  Pooled
// page-locked buffers are never freed on a full pool: the page-locked budget
// bounds how many exist.
struct youth_frame_queue {
    struct Item {
        int16_t* buf = nullptr;
        size_t cap = 0;      // values the buffer holds
        bool pinned = false;
        int w = 0, h = 0;
        uint32_t ts = 0;
    };
    static constexpr size_t kPinnedBytes = (size_t)256 << 20;
    static constexpr size_t kPoolMax = 48;  // pageable buffers kept
    std::mutex mu;
    std::deque<Item> q;
    // q.size(), stored under mu after every change: youth_queue_size reads
    // it without the lock, so a producer polling the depth (the reference's
    // logger waits on it) never contends with the worker's takes
    std::atomic<int> depth{0};
    std::vector<Item> pool;
    int high = 10, low = 5;
    bool pinned = false;      // page-locked buffers (SLAM module queue), allocated off the producer path
    // the producer's copy (youth_queue_push): 1 streaming stores
    // (youth::stream_copy; YOUTH_SLAM_PUSH_COPY=nt), 0 memcpy (=memcpy)
    int copy_mode = 1;
    // YOUTH_SLAM_PUSH_THREADS=k (k >= 1): a frame of >= 256 KB is copied by
    // the producer and k helper threads (host_copy.h; one producer at a time,
    // a concurrent producer copies alone); 0 (default): the producer alone
    std::unique_ptr<youth::HostCopyPool> copier;
    std::mutex copier_mu;
    size_t pinned_bytes = 0;  // page-locked bytes allocated and not freed
    int pinned_count = 0;     // page-locked buffers allocated and not freed
};

namespace {

void buf_free(youth_frame_queue* q, youth_frame_queue::Item& it)
{
    if (!it.buf) return;
    if (it.pinned) {
        youth_icp_host_free(it.buf);
        std::lock_guard<std::mutex> lk(q->mu);
        q->pinned_bytes -= it.cap * sizeof(int16_t);
        --q->pinned_count;
    } else {
        free(it.buf);
    }
    it.buf = nullptr;
    it.cap = 0;
}

// A buffer of >= n values for the producer: a pooled one, else (no pooled
// buffer fits) a new pageable one.  *kind: 0 pooled, 2 new pageable (this
// path never allocates page-locked memory: the worker and init do).
bool buf_get(youth_frame_queue* q, size_t n, youth_frame_queue::Item& it, int* kind)
{
    {
        std::lock_guard<std::mutex> lk(q->mu);
        for (size_t k = q->pool.size(); k-- > 0;) {
            if (q->pool[k].cap < n) continue;
            it.buf = q->pool[k].buf;
            it.cap = q->pool[k].cap;
            it.pinned = q->pool[k].pinned;
            q->pool.erase(q->pool.begin() + (long)k);
            *kind = 0;
            return true;
        }
    }
    *kind = 2;
    it.buf = static_cast<int16_t*>(malloc(n * sizeof(int16_t)));
    it.pinned = false;
    it.cap = it.buf ? n : 0;
    return it.buf != nullptr;
}

// A new page-locked buffer of n values while the budget lasts (worker / init).
bool buf_new_pinned(youth_frame_queue* q, size_t n, youth_frame_queue::Item& it)
{
    {
        std::lock_guard<std::mutex> lk(q->mu);
        if (q->pinned_bytes + n * sizeof(int16_t) > q->kPinnedBytes) return false;
        q->pinned_bytes += n * sizeof(int16_t);
        ++q->pinned_count;
    }
    it.buf = youth_icp_host_alloc(n);
    if (!it.buf) {
        std::lock_guard<std::mutex> lk(q->mu);
        q->pinned_bytes -= n * sizeof(int16_t);
        --q->pinned_count;
        return false;
    }
    it.pinned = true;
    it.cap = n;
    return true;
}

// back to the pool (q->mu held): page-locked buffers always (the budget
// bounds them), pageable ones up to kPoolMax (else freed by the caller, which
// is plain free())
void pool_put_locked(youth_frame_queue* q, youth_frame_queue::Item& it,
                     std::vector<youth_frame_queue::Item>& to_free)
{
    if (!it.buf) return;
    if (it.pinned || (!q->pinned && q->pool.size() < q->kPoolMax))
        q->pool.push_back(it);
    else
        to_free.push_back(it);
    it.buf = nullptr;
}

void free_all(youth_frame_queue* q, std::vector<youth_frame_queue::Item>& v)
{
    for (auto& it : v) buf_free(q, it);
    v.clear();
}

// The oldest frame, buffer and all (1), or 0 when empty.
int queue_take(youth_frame_queue* q, youth_frame_queue::Item& out)
{
    std::lock_guard<std::mutex> lk(q->mu);
    if (q->q.empty()) return 0;
    out = q->q.front();
    q->q.pop_front();
    q->depth.store((int)q->q.size(), std::memory_order_release);
    return 1;
}

// Page-locked buffers of n values until `count` exist (worker / init; pooled
// buffers smaller than n are freed first: a resolution change).  Returns the
// number allocated minus the number freed.
int queue_prefill(youth_frame_queue* q, size_t n, int count)
{
    std::vector<youth_frame_queue::Item> to_free;
    {
        std::lock_guard<std::mutex> lk(q->mu);
        std::vector<youth_frame_queue::Item> keep;
        for (auto& it : q->pool) (it.cap >= n ? keep : to_free).push_back(it);
        q->pool.swap(keep);
    }
    const int freed = (int)to_free.size();
    free_all(q, to_free);
    int added = 0;
    for (;;) {
        {
            std::lock_guard<std::mutex> lk(q->mu);
            if (q->pinned_count >= count) break;
        }
        youth_frame_queue::Item it;
        if (!buf_new_pinned(q, n, it)) break;
        std::lock_guard<std::mutex> lk(q->mu);
        q->pool.push_back(it);
        ++added;
    }
    return added - freed;
}

// The worker's pass over a returned buffer: page-locked ones of at least n
// values go back to the pool; a pageable one (the producer found the pool
// empty), or a page-locked one smaller than the worker's frame size n (in
// flight across a resolution change: pooled, it would count toward the
// page-locked target forever and keep new-size buffers out), is
// freed and, while fewer than `target` page-locked buffers exist, replaced
// by a page-locked one of n values.  Returns 1 when it allocated one.
int queue_release(youth_frame_queue* q, youth_frame_queue::Item& it, size_t n = 0, int target = 0)
{
    const bool replace = it.buf && (!it.pinned || (n > 0 && it.cap < n));
    std::vector<youth_frame_queue::Item> to_free;
    {
        std::lock_guard<std::mutex> lk(q->mu);
        if (it.buf && it.pinned && n > 0 && it.cap < n) {
            to_free.push_back(it);
            it.buf = nullptr;
        } else {
            pool_put_locked(q, it, to_free);
        }
    }
    free_all(q, to_free);
    if (!replace || !q->pinned || n == 0) return 0;
    {
        std::lock_guard<std::mutex> lk(q->mu);
        if (q->pinned_count >= target) return 0;
    }
    youth_frame_queue::Item fresh;
    if (!buf_new_pinned(q, n, fresh)) return 0;
    std::lock_guard<std::mutex> lk(q->mu);
    q->pool.push_back(fresh);
    return 1;
}

}  // namespace

extern "C" {

youth_frame_queue* youth_queue_create(int high_water, int low_water)
{
    if (high_water < 1 || low_water < 0 || low_water > high_water) return nullptr;
    auto* q = new youth_frame_queue();
    q->high = high_water;
    q->low = low_water;
    if (const char* e = getenv("YOUTH_SLAM_PUSH_COPY")) q->copy_mode = strcmp(e, "memcpy") == 0 ? 0 : 1;
    if (const char* e = getenv("YOUTH_SLAM_PUSH_THREADS"))
        if (atoi(e) > 0) q->copier.reset(new youth::HostCopyPool(std::min(atoi(e), 7), q->copy_mode == 1));
    return q;
}

void youth_queue_destroy(youth_frame_queue* q)
{
    if (!q) return;
    std::vector<youth_frame_queue::Item> all(q->q.begin(), q->q.end());
    all.insert(all.end(), q->pool.begin(), q->pool.end());
    q->q.clear();
    q->pool.clear();
    free_all(q, all);
    delete q;
}

int youth_queue_push(youth_frame_queue* q, const int16_t* depth, int width, int height,
                     uint32_t timestamp)
{
    if (!q || !depth || width <= 0 || height <= 0) return YOUTH_EINVAL;
    const size_t n = (size_t)width * (size_t)height;
    youth_frame_queue::Item it;
    int kind = 0;
    trace(YOUTH_SLAM_EV_PUSH_BEGIN, youth_queue_size(q));
    if (!buf_get(q, n, it, &kind)) return YOUTH_ENOMEM;
    bool copied = false;
    if (q->copier && n * sizeof(int16_t) >= ((size_t)256 << 10)) {
        std::unique_lock<std::mutex> lk(q->copier_mu, std::try_to_lock);
        if (lk.owns_lock()) {
            const youth::HostCopyPool::Seg seg{it.buf, depth, n * sizeof(int16_t)};
            q->copier->run(&seg, 1, n * sizeof(int16_t) / (2 * (q->copier->helpers() + 1)));
            copied = true;
        }
    }
    if (copied)
        ;
    else if (q->copy_mode == 1)
        youth::stream_copy(it.buf, depth, n * sizeof(int16_t));
    else
        memcpy(it.buf, depth, n * sizeof(int16_t));
    it.w = width;
    it.h = height;
    it.ts = timestamp;
    std::vector<youth_frame_queue::Item> to_free;
    int dropped = 0;
    {
        std::lock_guard<std::mutex> lk(q->mu);
        q->q.push_back(it);
        // SLAM.cpp:163-168: size > 10 -> pop the oldest down to 5
        if ((int)q->q.size() > q->high) {
            fprintf(stderr, "youth_icp: frame queue is getting large (%zu), dropping to %d\n",
                    q->q.size(), q->low);
            while ((int)q->q.size() > q->low) {
                pool_put_locked(q, q->q.front(), to_free);
                q->q.pop_front();
                ++dropped;
            }
        }
        q->depth.store((int)q->q.size(), std::memory_order_release);
    }
    free_all(q, to_free);
    if (dropped) trace(YOUTH_SLAM_EV_DROP, dropped);
    trace(YOUTH_SLAM_EV_PUSH_END, kind);
    return dropped;
}

int youth_queue_pop(youth_frame_queue* q, int16_t* depth_out, size_t cap, int* width,
                    int* height, uint32_t* timestamp)
{
    if (!q) return YOUTH_EINVAL;
    youth_frame_queue::Item it;
    {
        std::lock_guard<std::mutex> lk(q->mu);
        if (q->q.empty()) return 0;
        const auto& f = q->q.front();
        if ((size_t)f.w * (size_t)f.h > cap || !depth_out) return YOUTH_EINVAL;
        it = f;
        q->q.pop_front();
        q->depth.store((int)q->q.size(), std::memory_order_release);
    }
    memcpy(depth_out, it.buf, (size_t)it.w * it.h * sizeof(int16_t));
    if (width) *width = it.w;
    if (height) *height = it.h;
    if (timestamp) *timestamp = it.ts;
    queue_release(q, it);
    return 1;
}

int youth_queue_size(youth_frame_queue* q)
{
    if (!q) return 0;
    return q->depth.load(std::memory_order_acquire);
}

void youth_queue_clear(youth_frame_queue* q)
{
    if (!q) return;
    std::vector<youth_frame_queue::Item> to_free;
    {
        std::lock_guard<std::mutex> lk(q->mu);
        for (auto& it : q->q) pool_put_locked(q, it, to_free);
        q->q.clear();
        q->depth.store(0, std::memory_order_release);
    }
    free_all(q, to_free);
}

// ---------------------------------------------------------- YAML config ---
int youth_parse_camera_yaml(const char* path, youth_intrinsics* K, int* W, int* H)
{
    if (!path || !K) return 0;
    FILE* f = fopen(path, "r");
    if (!f) return 0;
    char line[512];
    while (fgets(line, sizeof(line), f)) {
        char* p = line;
        while (*p == ' ' || *p == '\t') ++p;
        if (*p == '#' || *p == '\0' || *p == '\n') continue;
        char* colon = strchr(p, ':');
        if (!colon) continue;
        std::string key(p, colon - p);
        while (!key.empty() && (key.back() == ' ' || key.back() == '\t')) key.pop_back();
        char* end = nullptr;
        const double val = strtod(colon + 1, &end);
        if (end == colon + 1) continue;  // not a number (e.g. Camera.type: "PinHole")
        if (key == "Camera.fx") K->fx = (float)val;
        else if (key == "Camera.fy") K->fy = (float)val;
        else if (key == "Camera.cx") K->cx = (float)val;
        else if (key == "Camera.cy") K->cy = (float)val;
        else if (key == "DepthMapFactor") K->depth_scale = (float)val;
        else if (key == "Camera.width" && W) *W = (int)val;
        else if (key == "Camera.height" && H) *H = (int)val;
    }
    fclose(f);
    return 1;
}

}  // extern "C"

// ------------------------------------------------------------ SLAM state --
namespace {

struct PoseRec {
    uint32_t ts;
    int32_t status;  // the frame's YOUTH_STATUS_* bits (never TIMEOUT: such a frame is realigned or skipped)
    double T[16];
};

std::mutex g_slam_mu;  // SLAM.cpp:16 slam_mutex: tracker + trajectory
std::mutex g_life_mu;  // initSlamModule / stopSlamModule against each other
std::atomic<bool> g_running{false};
std::atomic<bool> g_process{false};  // SLAM.cpp:29 process_frames
std::atomic<bool> g_busy{false};
std::atomic<bool> g_reset{false};
std::atomic<long long> g_batched{0};  // frames tracked in micro-batches
// timed-out aligns (YOUTH_STATUS_TIMEOUT): realigned on the cooperative plan,
// on the persistent kernel, and lost (still timed out: not recorded)
std::atomic<long long> g_realigned[3] = {};
// recorded frames with YOUTH_STATUS_FEW_MATCHES / _DEGENERATE set
std::atomic<long long> g_weak[2] = {};
std::thread g_worker;
youth_frame_queue* g_queue = nullptr;

std::mutex g_state_mu;  // run/stop hand-off for algorithmModule
std::condition_variable g_state_cv;

// processSlamFrame wakes the idle worker (no polling interval between a
// camera frame's arrival and its upload)
std::mutex g_wake_mu;
std::condition_variable g_wake_cv;

// configuration from initSlamModule
youth_intrinsics g_cfg_K;
int g_cfg_W = 0, g_cfg_H = 0;
bool g_cfg_has_yaml = false;

// tracker state (worker thread owns ctx; trajectory guarded by g_slam_mu)
std::vector<PoseRec> g_traj;
// g_traj.size(), stored under g_slam_mu after every change: a host polling
// for its pose (youth_slam_trajectory_length) does not take the lock the
// worker records every pose under
std::atomic<int> g_traj_len{0};
int g_last_points = 0;

void mat_mul4(const double* A, const double* B, double* C)
{
    double O[16];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            double s = 0.0;
            for (int k = 0; k < 4; ++k) s += A[i * 4 + k] * B[k * 4 + j];
            O[i * 4 + j] = s;
        }
    memcpy(C, O, sizeof(O));
}

youth_intrinsics intrinsics_for(int w, int h)
{
    if (g_cfg_has_yaml && (g_cfg_W == 0 || g_cfg_W == w) && (g_cfg_H == 0 || g_cfg_H == h))
        return g_cfg_K;
    return youth_default_intrinsics(w, h);
}

// Frames per micro-batch of the worker (YOUTH_SLAM_TRACK_BATCH, default
// YOUTH_TRACK_MAX_BATCH) and the page-locked buffers its queue keeps: a
// backlog holds about queue (11) + in flight (2 batch) + one batch of frames,
// plus the held reference frame (the target of a realign).
int slam_batch()
{
    const char* eb = getenv("YOUTH_SLAM_TRACK_BATCH");
    return eb ? std::max(1, std::min(atoi(eb), YOUTH_TRACK_MAX_BATCH)) : YOUTH_TRACK_MAX_BATCH;
}
int pool_target(int batch) { return 12 + 3 * batch; }

// SLAM.cpp:32-63 processFramesThread, with TrackRGBD replaced by HIP ICP.
// The worker takes every frame of the current size already queued behind
// the one it pops, up to `batch` (YOUTH_TRACK_MAX_BATCH by default;
// YOUTH_SLAM_TRACK_BATCH=m overrides, 1 = one frame per launch), and
// submits them as ONE micro-batch (youth_icp_track_submit_pinned: the queue's
// page-locked buffers are copied to the device in place), two submissions in
// flight.  The context is planned for `batch` (youth_icp_track_set_batch), so
// every frame runs on that plan whether it arrived alone (a live camera) or
// in a backlog (a .bin replay, a burst): a frame's pose does not depend on
// the queue's timing.  A frame's pose reaches the trajectory when the
// submission after its own is made or the queue runs empty (the worker stays
// busy until then: youth_slam_wait_idle).
void worker_main(int device)
{
    using Item = youth_frame_queue::Item;
    fprintf(stderr, "youth_icp: SLAM processing thread started\n");
    youth_icp_ctx* ctx = nullptr;
    int cw = 0, ch = 0;
    const int batch = slam_batch();
    std::vector<int16_t> packed;  // pageable frames of a micro-batch, packed (rare)
    bool held = false;            // a taken frame of another size (or sequence), next round
    Item held_item;
    double T_w_ref[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    struct Pending {
        uint32_t ts;
        int npts;   // valid pixels (counted for the last frame of a submission, else -1)
        bool last;  // the last frame of its submission
        Item item;  // its buffer, in use by the H2D until the frame is collected
    };
    std::deque<Pending> pend;  // submitted, not yet collected (oldest first)
    int subs = 0;              // submissions in pend
    // The last collected frame's buffer stays out of the pool until the next
    // frame has been collected: it is the target a timed-out align of that
    // frame is realigned against (youth_icp_track_realign).
    Item ref_hold;
    bool ref_valid = false;  // ref_hold is the tracker's reference of the next collected frame
    auto drop_ref = [&]() {
        if (ref_hold.buf && queue_release(g_queue, ref_hold, (size_t)cw * ch, pool_target(batch)))
            trace(YOUTH_SLAM_EV_POOL, 1);
        ref_hold = Item();
        ref_valid = false;
    };
    // collect the oldest submitted frame; record its pose unless a reset
    // arrived since it was submitted; it becomes the held reference and the
    // previous one's buffer goes back to the pool
    auto finish_one = [&](bool record) {
        Pending pr0 = pend.front();
        pend.pop_front();
        subs -= pr0.last;
        double T_rel[16];
        int has_ref = 0;
        trace(YOUTH_SLAM_EV_COLLECT_BEGIN, (int)pend.size() + 1);
        int st = youth_icp_track_collect(ctx, T_rel, &has_ref);
        trace(YOUTH_SLAM_EV_COLLECT_END, pr0.last ? 1 : 0);
        // (a frame of a sequence that a reset ended is not recorded: no retry)
        const bool keep = record && !g_reset.load();
        if (st >= 0 && has_ref && (st & YOUTH_STATUS_TIMEOUT) && keep) {
            // never composed: aligned again from the two frames' host buffers
            // (the cooperative plan, bit-identical when it completes; else the
            // persistent kernel); still timed out = lost
            int how = 2;
            if (ref_valid) {
                long long p0 = 0, p1 = 0;
                const long long c0 = youth_icp_track_realigned(ctx, &p0, nullptr);
                const int st2 = youth_icp_track_realign(ctx, ref_hold.buf, pr0.item.buf, nullptr, T_rel);
                const long long c1 = youth_icp_track_realigned(ctx, &p1, nullptr);
                if (st2 < 0)
                    fprintf(stderr, "youth_icp: realign failed: %s\n", youth_icp_last_error());
                else
                    st = st2;
                how = c1 > c0 ? 0 : p1 > p0 ? 1 : 2;
            }
            g_realigned[how].fetch_add(1);
            trace(YOUTH_SLAM_EV_REALIGN, how);
        }
        drop_ref();
        if (st < 0) {
            if (queue_release(g_queue, pr0.item, (size_t)cw * ch, pool_target(batch)))
                trace(YOUTH_SLAM_EV_POOL, 1);
            fprintf(stderr, "youth_icp: tracking failed: %s\n", youth_icp_last_error());
            return;
        }
        ref_hold = pr0.item;
        ref_valid = true;
        if (!keep) return;
        if (st & YOUTH_STATUS_TIMEOUT) {
            // no pose for this frame: it is left out of the trajectory and the
            // next frame composes onto the last recorded pose (no motion
            // across the lost frame)
            fprintf(stderr, "youth_icp: frame %u lost (align timed out twice)\n", pr0.ts);
            return;
        }
        std::lock_guard<std::mutex> lk(g_slam_mu);
        // resetSlam raises g_reset under this lock before it clears the
        // trajectory: a frame of the old sequence that passed the check
        // above sees the flag here and is not taken as the new origin
        if (g_reset.load()) return;
        if (!has_ref || g_traj.empty()) {
            // new sequence: this frame is the world origin
            double I[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
            memcpy(T_w_ref, I, sizeof(I));
            g_traj.clear();
            g_traj_len.store(0, std::memory_order_release);
        } else {
            // P_ref = T_rel P_new  =>  T_w_new = T_w_ref * T_rel
            mat_mul4(T_w_ref, T_rel, T_w_ref);
        }
        // FEW_MATCHES / DEGENERATE: some iteration skipped its update; the pose
        // the others reached is composed (identity motion if none applied)
        // and the bits are kept with it (youth_slam_get_status)
        if (st & YOUTH_STATUS_FEW_MATCHES) g_weak[0].fetch_add(1);
        if (st & YOUTH_STATUS_DEGENERATE) g_weak[1].fetch_add(1);
        PoseRec pr;
        pr.ts = pr0.ts;
        pr.status = st;
        memcpy(pr.T, T_w_ref, sizeof(pr.T));
        g_traj.push_back(pr);
        g_traj_len.store((int)g_traj.size(), std::memory_order_release);
        if (pr0.npts >= 0) g_last_points = pr0.npts;
    };
    while (g_process.load()) {
        Item items[YOUTH_TRACK_MAX_BATCH];
        g_busy.store(true);
        int got = 1;
        if (held) {
            items[0] = held_item;
            held = false;
        } else {
            got = queue_take(g_queue, items[0]);
        }
        if (got != 1) {
            if (!pend.empty()) {  // nothing new: finish what is in flight
                finish_one(true);
                continue;
            }
            g_busy.store(false);
            trace(YOUTH_SLAM_EV_IDLE_BEGIN, 0);
            {
                // the predicate re-checks the queue under g_wake_mu, which
                // processSlamFrame takes before notifying: no lost wake-up
                // (system_clock: pthread_cond_timedwait, which ThreadSanitizer
                // intercepts; a steady_clock wait_for is pthread_cond_clockwait)
                std::unique_lock<std::mutex> lk(g_wake_mu);
                g_wake_cv.wait_until(lk, std::chrono::system_clock::now() + std::chrono::milliseconds(20),
                                     [] { return !g_process.load() || youth_queue_size(g_queue) > 0; });
            }
            trace(YOUTH_SLAM_EV_IDLE_END, youth_queue_size(g_queue));
            continue;
        }
        const int w = items[0].w, h = items[0].h;
        if (g_reset.exchange(false)) {
            while (!pend.empty()) finish_one(false);  // frames of the old sequence
            drop_ref();
            if (ctx) youth_icp_track_reset(ctx);
        }
        if (!ctx || w != cw || h != ch) {
            while (!pend.empty()) finish_one(true);
            drop_ref();
            if (ctx) youth_icp_destroy(ctx);
            const youth_intrinsics K = intrinsics_for(w, h);
            ctx = youth_icp_create(device, w, h, 2 * batch, &K, nullptr);
            cw = w;
            ch = h;
            if (!ctx) {
                fprintf(stderr, "youth_icp: context creation failed: %s\n",
                        youth_icp_last_error());
                cw = ch = 0;
                queue_release(g_queue, items[0]);
                g_busy.store(false);
                continue;
            }
            if (batch > 1) youth_icp_track_set_batch(ctx, batch);
            // page-locked buffers for this size up front (initSlamModule made
            // them for the configured size already)
            trace(YOUTH_SLAM_EV_POOL, queue_prefill(g_queue, (size_t)w * h, pool_target(batch)));
        }
        const size_t N = (size_t)w * h;
        // two submissions in flight: with two queued, finish the oldest
        // before gathering the batch (the queue fills meanwhile, so a backlog
        // goes out in full micro-batches rather than as many small launches
        // each costing a full one)
        if (subs >= 2)
            while (!pend.empty()) {
                const bool last = pend.front().last;
                finish_one(true);
                if (last) break;
            }
        // the micro-batch: frames of this size already waiting, up to `batch`
        // in all (one of another size, or taken after a reset, is held for
        // the next round)
        int m = 1;
        while (m < batch && !held) {
            Item it;
            if (queue_take(g_queue, it) != 1) break;
            if (it.w == w && it.h == h && !g_reset.load()) {
                items[m++] = it;
            } else {
                held_item = it;
                held = true;
            }
        }
        trace(YOUTH_SLAM_EV_TAKE, m);
        // the tracker holds 2 batch frames in flight
        while (!pend.empty() && (int)pend.size() + m > 2 * batch) finish_one(true);
        const long long chained0 = youth_icp_track_chained_frames(ctx);
        bool pinned = true;
        for (int i = 0; i < m; ++i) pinned &= items[i].pinned;
        int rc;
        trace(YOUTH_SLAM_EV_SUBMIT_BEGIN, m);
        if (pinned) {
            const int16_t* fr[YOUTH_TRACK_MAX_BATCH];
            for (int i = 0; i < m; ++i) fr[i] = items[i].buf;
            rc = youth_icp_track_submit_pinned(ctx, fr, m);
        } else if (m == 1) {
            rc = youth_icp_track_submit(ctx, items[0].buf, nullptr);
        } else {
            packed.resize((size_t)m * N);
            for (int i = 0; i < m; ++i)
                memcpy(packed.data() + (size_t)i * N, items[i].buf, N * sizeof(int16_t));
            rc = youth_icp_track_submit_batch(ctx, packed.data(), m);
        }
        trace(YOUTH_SLAM_EV_SUBMIT_END, rc);
        // frames of this submission that ran in chained (micro-batch) launches
        g_batched.fetch_add(youth_icp_track_chained_frames(ctx) - chained0);
        // getSlamMapPoints reports the newest recorded frame: only the last
        // frame of a submission is counted
        int npts = 0;
        for (size_t i = 0; i < N; ++i) npts += items[m - 1].buf[i] > 0;
        // a failed micro-batch may have submitted its first frames
        const int sent = rc < 0 ? youth_icp_track_pending(ctx) - (int)pend.size() : m;
        if (rc < 0) fprintf(stderr, "youth_icp: tracking failed: %s\n", youth_icp_last_error());
        for (int i = 0; i < m; ++i) {
            if (i < sent)
                pend.push_back(Pending{items[i].ts, i == m - 1 ? npts : -1, i == sent - 1, items[i]});
            else
                queue_release(g_queue, items[i], N, pool_target(batch));
        }
        subs += sent > 0;
        if (batch == 1 && pend.size() == 2) finish_one(true);
    }
    while (ctx && !pend.empty()) finish_one(true);
    drop_ref();
    if (held) queue_release(g_queue, held_item);
    if (ctx) youth_icp_destroy(ctx);
    fprintf(stderr, "youth_icp: SLAM processing thread stopped\n");
}

// Rotation matrix -> unit quaternion (x, y, z, w), Shepperd's method.
void rot_to_quat(const double* T, double q[4])
{
    const double m00 = T[0], m01 = T[1], m02 = T[2];
    const double m10 = T[4], m11 = T[5], m12 = T[6];
    const double m20 = T[8], m21 = T[9], m22 = T[10];
    const double tr = m00 + m11 + m22;
    double x, y, z, w;
    if (tr > 0.0) {
        const double s = std::sqrt(tr + 1.0) * 2.0;
        w = 0.25 * s;
        x = (m21 - m12) / s;
        y = (m02 - m20) / s;
        z = (m10 - m01) / s;
    } else if (m00 > m11 && m00 > m22) {
        const double s = std::sqrt(1.0 + m00 - m11 - m22) * 2.0;
        w = (m21 - m12) / s;
        x = 0.25 * s;
        y = (m01 + m10) / s;
        z = (m02 + m20) / s;
    } else if (m11 > m22) {
        const double s = std::sqrt(1.0 + m11 - m00 - m22) * 2.0;
        w = (m02 - m20) / s;
        x = (m01 + m10) / s;
        y = 0.25 * s;
        z = (m12 + m21) / s;
    } else {
        const double s = std::sqrt(1.0 + m22 - m00 - m11) * 2.0;
        w = (m10 - m01) / s;
        x = (m02 + m20) / s;
        y = (m12 + m21) / s;
        z = 0.25 * s;
    }
    const double n = std::sqrt(x * x + y * y + z * z + w * w);
    q[0] = x / n;
    q[1] = y / n;
    q[2] = z / n;
    q[3] = w / n;
}

int write_tum(const std::string& path, const std::vector<PoseRec>& traj)
{
    FILE* f = fopen(path.c_str(), "w");
    if (!f) return 0;
    for (const auto& p : traj) {
        double q[4];
        rot_to_quat(p.T, q);
        // the reference hands TrackRGBD the ms timestamp as "seconds"
        // (SLAM.cpp:151), so the TUM time column carries ms as-is.
        fprintf(f, "%.6f %.9f %.9f %.9f %.9f %.9f %.9f %.9f\n", (double)p.ts, p.T[3], p.T[7],
                p.T[11], q[0], q[1], q[2], q[3]);
    }
    const int ok = ferror(f) == 0;
    fclose(f);
    return ok;
}

}  // namespace

extern "C" {

// SLAM.cpp:67-95
void initSlamModule(const char* config_file, const char* vocabulary_file)
{
    (void)vocabulary_file;  // no ORB vocabulary in an ICP tracker
    fprintf(stderr, "youth_icp: initializing HIP ICP module...\n");
    // g_life_mu serialises init/stop (SLAM.cpp:69 takes slam_mutex): two
    // concurrent inits must not both start a worker
    std::lock_guard<std::mutex> life(g_life_mu);
    if (g_running.load()) {
        fprintf(stderr, "youth_icp: SLAM module is already running\n");
        return;
    }
    std::lock_guard<std::mutex> lk(g_slam_mu);
    const int ndev = youth_icp_device_count();
    if (ndev <= 0) {
        // the product path never falls back to a CPU tracker
        fprintf(stderr, "youth_icp: no HIP device visible; module NOT started\n");
        return;
    }
    g_cfg_K = youth_default_intrinsics(640, 480);
    g_cfg_W = 0;
    g_cfg_H = 0;
    g_cfg_has_yaml = false;
    if (config_file && youth_parse_camera_yaml(config_file, &g_cfg_K, &g_cfg_W, &g_cfg_H))
        g_cfg_has_yaml = true;
    else if (config_file)
        fprintf(stderr, "youth_icp: cannot read %s; using viewer intrinsics\n", config_file);
    int device = 0;
    if (const char* e = getenv("YOUTH_ICP_DEVICE")) device = atoi(e);
    if (device < 0 || device >= ndev) device = 0;
    if (!g_queue) {
        g_queue = youth_queue_create(10, 5);
        g_queue->pinned = true;  // buffers the tracker copies to the device in place
    }
    youth_queue_clear(g_queue);
    // page-locked buffers for the configured frame size (the YAML's, else
    // 640x480) before the first frame: the producer never allocates them
    {
        const int pw = g_cfg_W > 0 ? g_cfg_W : 640, ph = g_cfg_H > 0 ? g_cfg_H : 480;
        queue_prefill(g_queue, (size_t)pw * ph, pool_target(slam_batch()));
    }
    g_traj.clear();
    g_traj_len.store(0, std::memory_order_release);
    g_last_points = 0;
    g_process.store(true);
    g_batched.store(0);
    for (auto& r : g_realigned) r.store(0);
    for (auto& r : g_weak) r.store(0);
    try {
        g_worker = std::thread(worker_main, device);
    } catch (const std::exception& ex) {
        fprintf(stderr, "youth_icp: failed to start worker: %s\n", ex.what());
        g_process.store(false);
        return;
    }
    {
        std::lock_guard<std::mutex> sl(g_state_mu);
        g_running.store(true);
    }
    g_state_cv.notify_all();
    fprintf(stderr, "youth_icp: HIP ICP module initialized (device %d)\n", device);
}

// SLAM.cpp:97-124
void stopSlamModule(void)
{
    fprintf(stderr, "youth_icp: stopping HIP ICP module...\n");
    std::lock_guard<std::mutex> life(g_life_mu);
    g_process.store(false);
    if (g_worker.joinable()) g_worker.join();
    if (g_queue) youth_queue_clear(g_queue);
    {
        std::lock_guard<std::mutex> sl(g_state_mu);
        g_running.store(false);
    }
    g_state_cv.notify_all();
    fprintf(stderr, "youth_icp: HIP ICP module stopped\n");
}

// SLAM.cpp:126-175
int processSlamFrame(const int16_t* depth_data, const uint8_t* color_data, int width,
                     int height, uint32_t timestamp)
{
    (void)color_data;
    if (!g_running.load() || !g_queue) return 0;
    if (!depth_data || width < 3 || height < 3 || width > 4096 || height > 4096) {
        fprintf(stderr, "youth_icp: processSlamFrame: bad frame %dx%d\n", width, height);
        return 0;
    }
    const int rc = youth_queue_push(g_queue, depth_data, width, height, timestamp);
    if (rc >= 0) {
        std::lock_guard<std::mutex> lk(g_wake_mu);
        g_wake_cv.notify_one();
    }
    if (rc < 0) {
        fprintf(stderr, "youth_icp: processSlamFrame: enqueue failed (%d)\n", rc);
        return 0;
    }
    return 1;
}

// SLAM.cpp:177-198
int saveSlamMap(const char* map_file)
{
    if (!g_running.load() || !map_file) {
        fprintf(stderr, "youth_icp: SLAM system is not running\n");
        return 0;
    }
    std::vector<PoseRec> traj;
    {
        std::lock_guard<std::mutex> lk(g_slam_mu);
        traj = g_traj;
    }
    const std::string base(map_file);
    // every frame is tracked frame-to-frame, so the keyframe file equals the
    // trajectory (SLAM.cpp:188 writes both)
    const int ok = write_tum(base + "_trajectory.txt", traj) &&
                   write_tum(base + "_keyframes.txt", traj);
    if (ok)
        fprintf(stderr, "youth_icp: map saved to %s\n", map_file);
    else
        fprintf(stderr, "youth_icp: error saving map to %s\n", map_file);
    return ok ? 1 : 0;
}

int isSlamModuleRunning(void) { return g_running.load() ? 1 : 0; }

int getSlamMapPoints(void)
{
    if (!g_running.load()) return 0;
    std::lock_guard<std::mutex> lk(g_slam_mu);
    return g_last_points;
}

void resetSlam(void)
{
    if (!g_running.load()) return;
    {
        // the flag first, under the trajectory lock: finish_one re-checks it
        // under the same lock, so no pre-reset frame is recorded after the
        // clear
        std::lock_guard<std::mutex> lk(g_slam_mu);
        g_reset.store(true);
        g_traj.clear();
        g_traj_len.store(0, std::memory_order_release);
        g_last_points = 0;
    }
    fprintf(stderr, "youth_icp: SLAM system reset\n");
}

int youth_slam_trajectory_length(void) { return g_traj_len.load(std::memory_order_acquire); }

int youth_slam_get_trajectory(int n, uint32_t* timestamps, double* T_wc)
{
    std::lock_guard<std::mutex> lk(g_slam_mu);
    int m = (int)g_traj.size();
    if (n < m) m = n;
    for (int i = 0; i < m; ++i) {
        if (timestamps) timestamps[i] = g_traj[i].ts;
        if (T_wc) memcpy(T_wc + (size_t)i * 16, g_traj[i].T, sizeof(g_traj[i].T));
    }
    return m;
}

int youth_slam_get_pose(int index, uint32_t* timestamp, double* T_wc)
{
    std::lock_guard<std::mutex> lk(g_slam_mu);
    if (index < 0 || index >= (int)g_traj.size()) return 0;
    if (timestamp) *timestamp = g_traj[index].ts;
    if (T_wc) memcpy(T_wc, g_traj[index].T, sizeof(g_traj[index].T));
    return 1;
}

long long youth_slam_batched_frames(void) { return g_batched.load(); }

long long youth_slam_realigned(long long* persistent, long long* lost)
{
    if (persistent) *persistent = g_realigned[1].load();
    if (lost) *lost = g_realigned[2].load();
    return g_realigned[0].load();
}

int youth_slam_get_status(int n, int32_t* status, long long* few_matches, long long* degenerate)
{
    if (few_matches) *few_matches = g_weak[0].load();
    if (degenerate) *degenerate = g_weak[1].load();
    std::lock_guard<std::mutex> lk(g_slam_mu);
    int m = (int)g_traj.size();
    if (n < m) m = n;
    for (int i = 0; i < m && status; ++i) status[i] = g_traj[i].status;
    return m;
}

int youth_slam_queue_size(void) { return g_queue ? youth_queue_size(g_queue) : 0; }

int youth_slam_wait_idle(int timeout_ms)
{
    const auto t0 = std::chrono::steady_clock::now();
    while (g_running.load()) {
        if (youth_queue_size(g_queue) == 0 && !g_busy.load()) {
            // re-check after a short pause: the worker may be between pop and busy
            std::this_thread::sleep_for(std::chrono::milliseconds(2));
            if (youth_queue_size(g_queue) == 0 && !g_busy.load()) return 1;
        }
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms))
            return 0;
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    return 0;
}

// recorded from inside the tracker (icp_kernels.hip: a submission's steps)
void youth_slam_trace_hook(int kind, int arg) { trace(kind, arg); }

// enable / read are serialised against each other (the writers never take it)
std::mutex g_tr_mu;

int youth_slam_trace_enable(int capacity)
{
    if (capacity < 0) return YOUTH_EINVAL;
    TraceBuf* b = nullptr;
    if (capacity > 0) {
        b = new (std::nothrow) TraceBuf(capacity);
        if (!b) return YOUTH_ENOMEM;
    }
    std::lock_guard<std::mutex> lk(g_tr_mu);
    TraceBuf* old = g_tr.exchange(b);  // seq_cst: after it, new writers see b
    // a writer that may still hold `old` has announced itself before loading it
    while (g_tr_active.load() != 0) std::this_thread::yield();
    delete old;
    return YOUTH_OK;
}

int youth_slam_trace_read(int n, double* t, int* kind, int* arg)
{
    std::lock_guard<std::mutex> lk(g_tr_mu);  // the buffer is not swapped meanwhile
    TraceBuf* b = g_tr.load();
    if (!b) return 0;
    const int claimed = std::min(b->claimed.load(std::memory_order_relaxed), b->cap);
    // the events whose writers have finished, up to the first unfinished one
    int done = 0;
    while (done < claimed && b->ev[done].ready.load(std::memory_order_acquire)) ++done;
    const int m = std::min(n, done);
    for (int i = 0; i < m; ++i) {
        if (t) t[i] = b->ev[i].t;
        if (kind) kind[i] = b->ev[i].kind;
        if (arg) arg[i] = b->ev[i].arg;
    }
    return done;
}

void youth_slam_wait_stopped(void)
{
    std::unique_lock<std::mutex> lk(g_state_mu);
    g_state_cv.wait(lk, [] { return !g_running.load(); });
}

}  // extern "C"
