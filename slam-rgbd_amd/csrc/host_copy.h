// host_copy.h — host-side parallel copy of caller frames into page-locked
// staging (the tracker's youth_icp_track_submit_batch /
// youth_icp_track_host_sequence path).
//
// A micro-batch of 8 640x480 frames is 4.9 MB.  One thread copies it in
// ~245 us on the GPU box's host (profiles/r05/bench_r5ac.json: 31 us per
// frame), longer than the GPU's ~200 us for the micro-batch, so a streamed
// sequence ran at the host copy's rate.  The pool splits the copy into
// pieces claimed from one atomic counter by the calling thread and `helpers`
// persistent threads.  The caller always copies too, so a helper that wakes
// late only means fewer hands; run() returns when every piece is done and
// no helper still holds the job (a late helper can never see the next one).
#pragma once

#include <emmintrin.h>
#include <stdint.h>

#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

namespace youth {

// memcpy with non-temporal (streaming) 16-byte stores for the destination:
// a frame copied into a page-locked queue buffer is next read by the GPU
// (k_pull_frames / the H2D), not by this CPU, so the stores skip the
// read-for-ownership of each destination line and leave the bytes in memory
// rather than in this core's caches.  The sfence orders the streaming stores
// before anything the caller publishes after it (the queue push under its
// mutex).  SSE2 only (every x86-64).
inline void stream_copy(void* dst, const void* src, size_t bytes)
{
    char* d = static_cast<char*>(dst);
    const char* s = static_cast<const char*>(src);
    size_t head = (16 - ((uintptr_t)d & 15)) & 15;
    if (head > bytes) head = bytes;
    memcpy(d, s, head);
    d += head;
    s += head;
    bytes -= head;
    size_t i = 0;
    for (; i + 128 <= bytes; i += 128) {
        __m128i v[8];
        for (int k = 0; k < 8; ++k) v[k] = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s + i + 16 * k));
        for (int k = 0; k < 8; ++k) _mm_stream_si128(reinterpret_cast<__m128i*>(d + i + 16 * k), v[k]);
    }
    memcpy(d + i, s + i, bytes - i);
    _mm_sfence();
}

class HostCopyPool {
public:
    struct Seg {
        void* dst;
        const void* src;
        size_t bytes;
    };

    // stream: pieces copied with youth::stream_copy (a destination no CPU
    // reads next), else memcpy
    explicit HostCopyPool(int helpers, bool stream = false) : stream_(stream)
    {
        for (int i = 0; i < helpers; ++i) th_.emplace_back([this] { loop(); });
    }
    ~HostCopyPool()
    {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    HostCopyPool(const HostCopyPool&) = delete;
    HostCopyPool& operator=(const HostCopyPool&) = delete;

    int helpers() const { return (int)th_.size(); }

    // Copy every segment; each is cut into pieces of about `piece` bytes
    // (multiples of 4 KB).  One caller at a time per pool.
    void run(const Seg* seg, int n_seg, size_t piece)
    {
        piece = piece < 4096 ? 4096 : (piece + 4095) / 4096 * 4096;
        int total = 0;
        for (int i = 0; i < n_seg; ++i) total += (int)((seg[i].bytes + piece - 1) / piece);
        if (total == 0) return;
        {
            std::lock_guard<std::mutex> lk(mu_);
            seg_ = seg;
            n_seg_ = n_seg;
            piece_ = piece;
            total_ = total;
            next_.store(0, std::memory_order_relaxed);
            open_ = true;
            ++gen_;
        }
        if (total > 1) cv_.notify_all();
        work(seg, n_seg, piece, total);
        std::unique_lock<std::mutex> lk(mu_);
        open_ = false;  // no helper joins from here on
        idle_.wait(lk, [this] { return active_ == 0; });
    }

private:
    // claim pieces until none is left; piece k = the k-th piece in segment
    // order
    void work(const Seg* seg, int n_seg, size_t piece, int total)
    {
        for (int k; (k = next_.fetch_add(1, std::memory_order_relaxed)) < total;) {
            int s = 0;
            size_t off = (size_t)k * piece;
            for (; s < n_seg; ++s) {
                const size_t np = (seg[s].bytes + piece - 1) / piece;
                if (off < np * piece) break;
                off -= np * piece;
            }
            const size_t len = seg[s].bytes - off < piece ? seg[s].bytes - off : piece;
            if (stream_)
                stream_copy(static_cast<char*>(seg[s].dst) + off,
                            static_cast<const char*>(seg[s].src) + off, len);
            else
                memcpy(static_cast<char*>(seg[s].dst) + off,
                       static_cast<const char*>(seg[s].src) + off, len);
        }
    }

    void loop()
    {
        unsigned seen = 0;
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            cv_.wait(lk, [&] { return stop_ || (open_ && gen_ != seen); });
            if (stop_) return;
            seen = gen_;
            const Seg* seg = seg_;
            const int n_seg = n_seg_, total = total_;
            const size_t piece = piece_;
            ++active_;
            lk.unlock();
            work(seg, n_seg, piece, total);
            lk.lock();
            if (--active_ == 0) idle_.notify_all();
        }
    }

    std::mutex mu_;
    std::condition_variable cv_, idle_;
    std::vector<std::thread> th_;
    const Seg* seg_ = nullptr;
    int n_seg_ = 0, total_ = 0, active_ = 0;
    size_t piece_ = 0;
    std::atomic<int> next_{0};
    unsigned gen_ = 0;
    bool open_ = false, stop_ = false;
    const bool stream_;
};

}  // namespace youth
