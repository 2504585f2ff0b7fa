// Probe: the SLAM worker's hipMemcpyAsync of a micro-batch
// sometimes blocks the host for ~8 ms (profiles/r05/slamtrace*).  This mimics
// the tracker's pattern -- a transfer stream that waits for the compute
// stream's last event, 8 H2D copies of 614,400 B from page-locked buffers
// (rotating over 35), an event the compute stream waits for, a ~150 us kernel
// -- and reports every enqueue that takes > 1 ms: the iteration, the buffer,
// and whether an idle pause (every 40 iterations, like the gap between bench
// passes) preceded it.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>

__global__ void spin(long long cycles, int* out)
{
    const long long t0 = clock64();
    while (clock64() - t0 < cycles) {
    }
    if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = 1;
}

static double now_ms()
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv)
{
    const int iters = argc > 1 ? atoi(argv[1]) : 2000;
    const int pause_every = argc > 2 ? atoi(argv[2]) : 40;
    const double pause_ms = argc > 3 ? atof(argv[3]) : 5.0;
    const size_t bytes = 640 * 480 * 2;
    const int nbuf = 35, m = 8;
    hipStream_t comp, xfer;
    if (hipStreamCreateWithFlags(&comp, hipStreamNonBlocking) != hipSuccess) return 1;
    if (hipStreamCreateWithFlags(&xfer, hipStreamNonBlocking) != hipSuccess) return 1;
    std::vector<void*> h(nbuf);
    for (auto& p : h)
        if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) return 2;
    char* d = nullptr;
    int* flag = nullptr;
    if (hipMalloc(&d, 16 * bytes) != hipSuccess || hipMalloc(&flag, 4) != hipSuccess) return 3;
    hipEvent_t ec[2], ex[2];
    for (int i = 0; i < 2; ++i) {
        (void)hipEventCreateWithFlags(&ec[i], hipEventDisableTiming);
        (void)hipEventCreateWithFlags(&ex[i], hipEventDisableTiming);
    }
    int b = 0, slow = 0;
    double worst = 0;
    bool paused = false;
    const double T0 = now_ms();
    for (int it = 0; it < iters; ++it) {
        if (pause_every > 0 && it % pause_every == 0 && it) {
            (void)hipStreamSynchronize(comp);
            std::this_thread::sleep_for(std::chrono::microseconds((long)(pause_ms * 1000)));
            paused = true;
        }
        const int half = it & 1;
        if (it >= 2) (void)hipStreamWaitEvent(xfer, ec[half], 0);
        for (int i = 0; i < m; ++i) {
            const double a = now_ms();
            (void)hipMemcpyAsync(d + (size_t)(half * m + i) * bytes, h[b], bytes, hipMemcpyHostToDevice, xfer);
            const double e = now_ms() - a;
            worst = std::max(worst, e);
            if (e > 1.0) {
                ++slow;
                printf("slow enqueue %.3f ms: iteration %d copy %d buffer %d, t = %.1f ms%s\n", e, it, i, b,
                       a - T0, paused ? " (first iteration after a pause)" : "");
            }
            b = (b + 1) % nbuf;
        }
        paused = false;
        (void)hipEventRecord(ex[half], xfer);
        (void)hipStreamWaitEvent(comp, ex[half], 0);
        hipLaunchKernelGGL(spin, dim3(256), dim3(64), 0, comp, 300000LL, flag);
        (void)hipEventRecord(ec[half], comp);
        if (it >= 1) (void)hipEventSynchronize(ec[half ^ 1]);
    }
    (void)hipDeviceSynchronize();
    printf("%d iterations, %d slow enqueues (> 1 ms), worst %.3f ms, %.1f ms total\n", iters, slow, worst,
           now_ms() - T0);
    return 0;
}
