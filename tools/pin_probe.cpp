// Probe: does the first DMA from a freshly hipHostMalloc'd
// buffer cost more than later ones?  N page-locked 640x480 int16 buffers, each
// copied H2D twice (async + stream sync), first-use and second-use times; then
// the same for a buffer allocated on another host thread.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>

static double now_ms()
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main()
{
    const size_t bytes = 640 * 480 * 2;
    const int n = 48;
    void* d = nullptr;
    hipStream_t s;
    if (hipMalloc(&d, bytes) != hipSuccess || hipStreamCreate(&s) != hipSuccess) return 1;
    std::vector<void*> h(n);
    double t0 = now_ms();
    for (int i = 0; i < n; ++i)
        if (hipHostMalloc(&h[i], bytes, hipHostMallocDefault) != hipSuccess) return 2;
    printf("hipHostMalloc x%d: %.3f ms total\n", n, now_ms() - t0);
    for (int pass = 0; pass < 2; ++pass) {
        double worst = 0, sum = 0;
        int worst_i = -1;
        for (int i = 0; i < n; ++i) {
            const double a = now_ms();
            if (hipMemcpyAsync(d, h[i], bytes, hipMemcpyHostToDevice, s) != hipSuccess) return 3;
            const double b = now_ms();
            if (hipStreamSynchronize(s) != hipSuccess) return 4;
            const double c = now_ms();
            sum += c - a;
            if (c - a > worst) {
                worst = c - a;
                worst_i = i;
            }
            if (pass == 0 && i < 4) printf("  buffer %d first use: enqueue %.3f ms, total %.3f ms\n", i, b - a, c - a);
        }
        printf("pass %d: mean %.3f ms per copy, worst %.3f ms (buffer %d)\n", pass, sum / n, worst, worst_i);
    }
    // a buffer allocated by another thread, first used here
    void* other = nullptr;
    std::thread th([&] { (void)hipHostMalloc(&other, bytes, hipHostMallocDefault); });
    th.join();
    const double a = now_ms();
    (void)hipMemcpyAsync(d, other, bytes, hipMemcpyHostToDevice, s);
    (void)hipStreamSynchronize(s);
    printf("other-thread buffer first use: %.3f ms\n", now_ms() - a);
    // many small coherent result slots, as the tracker allocates lazily
    double tm = 0;
    for (int i = 0; i < 16; ++i) {
        void* r = nullptr;
        const double q = now_ms();
        (void)hipHostMalloc(&r, 17 * sizeof(double), hipHostMallocCoherent);
        tm = std::max(tm, now_ms() - q);
    }
    printf("hipHostMalloc coherent 136 B: worst %.3f ms\n", tm);
    return 0;
}
