// driver.cpp — sanitizer driver for the host-side threading code (SURVEY §5
// "Race detection"; built by tests/tsan/Makefile with -fsanitize=thread and
// with -fsanitize=address,undefined, linked with the CPU stand-in
// icp_stub.c).  Every scenario calls the product's real entry points from
// several threads at once:
//   1. concurrent initSlamModule (SLAM.cpp:67-95: one worker must start);
//   2. producers calling processSlamFrame (SLAM.cpp:126-175) while readers
//      poll the map, save it and reset it (SLAM.h:27-38);
//   3. the ingest queue API hammered by pushers and poppers (>10 -> 5 policy);
//   4. the AlgorithmModule frame loop over an in-process transport, stopped
//      from another thread;
//   5. the same loop over POSIX queues (youth_algorithm_loop), when the
//      machine allows them;
//   6. stopSlamModule while producers are still pushing;
//   7. timed-out aligns (the stub's YOUTH_STUB_TIMEOUT_EVERY) realigned by
//      the worker, with the event trace enabled, read and disabled from
//      another thread while the worker records (a freed trace
//      buffer must never be written).
// Exit 0 when every check holds; the sanitizers abort (exit 66 / non-zero)
// on a report.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <mqueue.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "youth_icp.h"
#include "youth_wire.h"

static void check(bool ok, const char* what)
{
    if (!ok) {
        fprintf(stderr, "FAIL: %s\n", what);
        exit(1);
    }
}

static const int W = 32, H = 24;

static std::vector<int16_t> frame(int value)
{
    return std::vector<int16_t>((size_t)W * H, (int16_t)value);
}

static void scenario_init_and_producers()
{
    std::thread a([] { initSlamModule(nullptr, nullptr); });
    std::thread b([] { initSlamModule(nullptr, nullptr); });
    a.join();
    b.join();
    check(isSlamModuleRunning() == 1, "module running after concurrent init");

    std::atomic<bool> done{false};
    std::vector<std::thread> prod;
    for (int t = 0; t < 4; ++t)
        prod.emplace_back([t] {
            for (int k = 0; k < 40; ++k) {
                auto f = frame(1000 + 100 * t + k);
                check(processSlamFrame(f.data(), nullptr, W, H, (uint32_t)(t * 1000 + k)) == 1,
                      "processSlamFrame accepted");
                if (k % 8 == 0) std::this_thread::sleep_for(std::chrono::microseconds(300));
            }
        });
    const std::string base = "/tmp/youth_tsan_map_" + std::to_string(getpid());
    std::thread reader([&] {
        int n = 0;
        while (!done.load()) {
            (void)getSlamMapPoints();
            const int len = youth_slam_trajectory_length();
            std::vector<uint32_t> ts(len > 0 ? len : 1);
            std::vector<double> T((size_t)(len > 0 ? len : 1) * 16);
            (void)youth_slam_get_trajectory(len, ts.data(), T.data());
            if (++n % 16 == 0) check(saveSlamMap(base.c_str()) == 1, "saveSlamMap");
            if (n == 40) resetSlam();
            std::this_thread::sleep_for(std::chrono::microseconds(200));
        }
    });
    for (auto& p : prod) p.join();
    check(youth_slam_wait_idle(20000) == 1, "worker idle");
    if (getenv("YOUTH_SLAM_TRACK_BATCH"))
        check(youth_slam_batched_frames() > 0, "worker tracked micro-batches");
    done.store(true);
    reader.join();
    // one more frame after the reader's reset (which may have come after the
    // last producer frame was tracked): the trajectory is not empty
    auto last = frame(4242);
    check(processSlamFrame(last.data(), nullptr, W, H, 99999) == 1, "processSlamFrame accepted");
    check(youth_slam_wait_idle(20000) == 1, "worker idle");
    const int len = youth_slam_trajectory_length();
    check(len > 0 && len <= 161, "trajectory length bounded by frames pushed");
    unlink((base + "_trajectory.txt").c_str());
    unlink((base + "_keyframes.txt").c_str());
}

static void scenario_queue()
{
    youth_frame_queue* q = youth_queue_create(10, 5);
    std::atomic<int> popped{0};
    std::atomic<bool> stop{false};
    std::vector<std::thread> th;
    for (int t = 0; t < 4; ++t)
        th.emplace_back([&, t] {
            for (int k = 0; k < 200; ++k) {
                auto f = frame(t * 1000 + k);
                check(youth_queue_push(q, f.data(), W, H, (uint32_t)k) >= 0, "queue push");
                check(youth_queue_size(q) <= 10, "queue bounded");
            }
        });
    for (int t = 0; t < 2; ++t)
        th.emplace_back([&] {
            std::vector<int16_t> buf((size_t)W * H);
            while (!stop.load()) {
                int w = 0, h = 0;
                uint32_t ts = 0;
                if (youth_queue_pop(q, buf.data(), buf.size(), &w, &h, &ts) == 1) {
                    check(w == W && h == H, "popped frame size");
                    popped.fetch_add(1);
                }
            }
        });
    for (int t = 0; t < 4; ++t) th[t].join();
    while (youth_queue_size(q) > 0) std::this_thread::yield();
    stop.store(true);
    th[4].join();
    th[5].join();
    check(popped.load() > 0 && popped.load() <= 800, "popped count");
    youth_queue_destroy(q);
}

struct InProc {
    std::mutex mu;
    std::deque<std::vector<unsigned char>> q;
    std::vector<youth_pose_msg> poses;
};

static int inproc_send(void* user, const void* msg, size_t len)
{
    auto* ip = (InProc*)user;
    std::lock_guard<std::mutex> lk(ip->mu);
    ip->q.emplace_back((const unsigned char*)msg, (const unsigned char*)msg + len);
    return 0;
}

static int inproc_recv(void* user, void* buf, size_t cap, int timeout_ms)
{
    auto* ip = (InProc*)user;
    for (int waited = 0; waited <= timeout_ms; ++waited) {
        {
            std::lock_guard<std::mutex> lk(ip->mu);
            if (!ip->q.empty()) {
                auto m = std::move(ip->q.front());
                ip->q.pop_front();
                if (m.size() > cap) return -1;
                memcpy(buf, m.data(), m.size());
                return (int)m.size();
            }
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    return 0;
}

static int inproc_publish(void* user, const void* msg, size_t len)
{
    auto* ip = (InProc*)user;
    if (len != sizeof(youth_msg_header) + sizeof(youth_pose_msg)) return 1;
    youth_pose_msg p;
    memcpy(&p, (const unsigned char*)msg + sizeof(youth_msg_header), sizeof(p));
    std::lock_guard<std::mutex> lk(ip->mu);
    ip->poses.push_back(p);
    return 0;
}

static void scenario_frame_loop()
{
    stopSlamModule();
    initSlamModule(nullptr, nullptr);
    InProc ip;
    int stop = 0;
    int frames = -1;
    std::thread loop([&] {
        frames = youth_algorithm_run(inproc_recv, &ip, inproc_publish, &ip, &stop);
    });
    for (int k = 0; k < 12; ++k) {
        auto f = frame(2000 + k);
        check(youth_wire_send_frame(inproc_send, &ip, (uint32_t)(500 + k), (uint32_t)(40 * k), W,
                                    H, f.data(), nullptr) == 2,
              "send_frame messages");
        std::this_thread::sleep_for(std::chrono::milliseconds(3));
    }
    for (int i = 0; i < 5000; ++i) {
        {
            std::lock_guard<std::mutex> lk(ip.mu);
            if (ip.q.empty() && (int)ip.poses.size() == youth_slam_trajectory_length() &&
                youth_slam_wait_idle(0) == 1)
                break;
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    __atomic_store_n(&stop, 1, __ATOMIC_RELEASE);
    loop.join();
    check(frames == 12, "frame loop handed every frame to processSlamFrame");
    std::lock_guard<std::mutex> lk(ip.mu);
    check(!ip.poses.empty(), "poses published");
    for (size_t i = 0; i < ip.poses.size(); ++i)
        check(ip.poses[i].index == (int)i, "pose indices consecutive");
}

static void scenario_mq_loop()
{
    const std::string fq = "/youth_tsan_f_" + std::to_string(getpid());
    const std::string pq = "/youth_tsan_p_" + std::to_string(getpid());
    stopSlamModule();  // a fresh trajectory: pose k is frame k's
    initSlamModule(nullptr, nullptr);
    int stop = 0;
    int frames = -2;
    std::thread loop([&] { frames = youth_algorithm_loop(fq.c_str(), pq.c_str(), &stop); });
    int sent = 0;
    for (int k = 0; k < 4; ++k) {
        auto f = frame(3000 + k);
        if (youth_wire_mq_send_frame(fq.c_str(), (uint32_t)(900 + k), (uint32_t)(33 * k), W, H,
                                     f.data(), nullptr) != 2)
            break;
        ++sent;
        youth_msg_header h;
        youth_pose_msg p;
        check(youth_wire_mq_recv_pose(pq.c_str(), 10000, &h, &p) == 1, "pose over mq");
        check(p.index == k && h.frameId == 900 + k, "mq pose k belongs to frame k");
    }
    __atomic_store_n(&stop, 1, __ATOMIC_RELEASE);
    loop.join();
    mq_unlink(fq.c_str());
    mq_unlink(pq.c_str());
    if (sent == 0) {
        fprintf(stderr, "note: POSIX queues unavailable here; mq scenario skipped\n");
        return;
    }
    if (frames != sent) fprintf(stderr, "mq loop: frames %d sent %d\n", frames, sent);
    check(frames == sent, "mq loop frames");
}

static void scenario_stop_under_load()
{
    std::atomic<bool> go{true};
    std::vector<std::thread> prod;
    for (int t = 0; t < 3; ++t)
        prod.emplace_back([&, t] {
            int k = 0;
            while (go.load()) {
                auto f = frame(4000 + t * 10 + (k++ % 10));
                (void)processSlamFrame(f.data(), nullptr, W, H, (uint32_t)k);  // 0 once stopped
            }
        });
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    stopSlamModule();
    check(isSlamModuleRunning() == 0, "stopped");
    go.store(false);
    for (auto& p : prod) p.join();
}

static void scenario_realign_and_trace()
{
    stopSlamModule();
    setenv("YOUTH_STUB_TIMEOUT_EVERY", "3", 1);
    initSlamModule(nullptr, nullptr);
    std::atomic<bool> done{false};
    std::thread tracer([&] {
        std::vector<double> t(256);
        std::vector<int> k(256), a(256);
        for (int i = 0; !done.load(); ++i) {
            check(youth_slam_trace_enable(i % 3 == 2 ? 0 : 64 + 32 * (i % 5)) == 0, "trace enable");
            (void)youth_slam_trace_read(256, t.data(), k.data(), a.data());
            std::this_thread::sleep_for(std::chrono::microseconds(150));
        }
    });
    const int F = 40;
    long long want = 0;
    for (int k = 0; k < F; ++k) {
        auto f = frame(100 + 7 * k);
        while (youth_slam_queue_size() >= 10) std::this_thread::yield();
        check(processSlamFrame(f.data(), nullptr, W, H, (uint32_t)k) == 1, "processSlamFrame accepted");
        if (k % 5 == 0) std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    check(youth_slam_wait_idle(20000) == 1, "worker idle");
    done.store(true);
    tracer.join();
    check(youth_slam_trace_enable(0) == 0, "trace off");
    long long persistent = -1, lost = -1;
    const long long realigned = youth_slam_realigned(&persistent, &lost);
    check(realigned >= F / 3 - 1 && persistent == 0 && lost == 0, "timed-out aligns realigned");
    // every frame recorded, the last pose the sum of the stub's translations
    // (7 mm steps x W x H values x 1e-6 per frame): no timed-out pose composed
    const int len = youth_slam_trajectory_length();
    check(len == F, "every frame recorded");
    std::vector<uint32_t> ts(F);
    std::vector<double> T((size_t)F * 16);
    check(youth_slam_get_trajectory(F, ts.data(), T.data()) == F, "trajectory");
    want = (long long)(F - 1) * 7 * W * H;
    check(T[(size_t)(F - 1) * 16 + 3] > 0.999999 * want * 1e-6 &&
              T[(size_t)(F - 1) * 16 + 3] < 1.000001 * want * 1e-6,
          "trajectory composed from realigned poses");
    std::vector<int32_t> st(F, -1);
    check(youth_slam_get_status(F, st.data(), nullptr, nullptr) == F, "status");
    for (int i = 0; i < F; ++i) check(st[i] == 0, "no TIMEOUT bit recorded");
    stopSlamModule();
    unsetenv("YOUTH_STUB_TIMEOUT_EVERY");
    initSlamModule(nullptr, nullptr);  // scenario_stop_under_load stops it
}

int main()
{
    scenario_init_and_producers();
    scenario_queue();
    scenario_frame_loop();
    scenario_mq_loop();
    scenario_realign_and_trace();
    scenario_stop_under_load();
    printf("sanitizer driver: all scenarios passed\n");
    return 0;
}
