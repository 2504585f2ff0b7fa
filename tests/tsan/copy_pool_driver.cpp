// Sanitizer driver for slam-rgbd_amd/csrc/host_copy.h (the tracker's
// parallel staging copy): many jobs of random segment counts and sizes on
// pools of 0-4 helpers, checked byte for byte; several pools used from
// several threads at once; pools destroyed right after a job and with helpers
// that never saw one.  Built with -fsanitize=thread and with
// -fsanitize=address,undefined (tests/test_sanitizers.py).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "host_copy.h"

static int check_jobs(int helpers, int jobs, unsigned seed, bool stream = false)
{
    youth::HostCopyPool pool(helpers, stream);
    std::mt19937 rng(seed);
    for (int j = 0; j < jobs; ++j) {
        const int n = 1 + (int)(rng() % 8);
        std::vector<std::vector<unsigned char>> src(n), dst(n);
        std::vector<youth::HostCopyPool::Seg> seg(n);
        for (int i = 0; i < n; ++i) {
            const size_t bytes = rng() % 3 == 0 ? rng() % 64 : 1 + rng() % 300000;
            src[i].resize(bytes);
            dst[i].assign(bytes, 0xAB);
            for (size_t b = 0; b < bytes; ++b) src[i][b] = (unsigned char)(rng() >> 7);
            seg[i] = {dst[i].data(), src[i].data(), bytes};
        }
        const size_t piece = (size_t)1 << (12 + rng() % 6);
        pool.run(seg.data(), n, piece);
        for (int i = 0; i < n; ++i)
            if (src[i] != dst[i]) {
                fprintf(stderr, "copy mismatch: helpers %d job %d segment %d\n", helpers, j, i);
                return 1;
            }
    }
    return 0;
}

int main()
{
    int bad = 0;
    for (int h = 0; h <= 4; ++h) bad |= check_jobs(h, 60, 1234u + h);
    // streaming stores (the SLAM producer's copy, youth::stream_copy): odd
    // sizes and unaligned segments included
    for (int h = 0; h <= 2; ++h) bad |= check_jobs(h, 40, 777u + h, true);
    // pools used concurrently from four threads (one caller per pool)
    std::vector<std::thread> th;
    std::vector<int> rc(4, 0);
    for (int t = 0; t < 4; ++t)
        th.emplace_back([t, &rc] { rc[t] = check_jobs(1 + t % 3, 40, 99u + t); });
    for (auto& x : th) x.join();
    for (int r : rc) bad |= r;
    // destroyed without a job, and right after one
    for (int k = 0; k < 20; ++k) {
        youth::HostCopyPool idle(3);
        (void)idle;
        bad |= check_jobs(2, 1, 7u + k);
    }
    if (bad) return 1;
    printf("copy pool: all scenarios passed\n");
    return 0;
}
