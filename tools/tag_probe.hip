// tag_probe.hip — developer probe (not shipped): the tagged-partials hand-off
// of profiles/r03/k_icp_coop_tagged_partials_experiment.patch in isolation,
// to find why its readers never saw the tags.
//
// G workgroups of 512 threads, `iters` iterations.  Per iteration wave 0 of
// workgroup c publishes row c: 30 values, each as a tagged piece; then every
// thread of every workgroup reads every row's pieces (as sum_pair_rows_tagged
// does: thread e reads column e / 30 of value e % 30) until each piece
// carries the iteration's tag, and checks the value.  Rows double-buffered by
// iteration parity.  Spins bounded (kSpin polls): a piece not seen by then is
// counted as a timeout, nothing waits longer.
//
// Forms (argv[1]):
//   0  the patch: ONE 16-B buffer_store sc1 {lo, tag, hi, tag} per value,
//      readers buffer_load_dwordx4 sc1 (aux 16);
//   1  the guide's R2 (cdna_hip_programming.md Guideline 16): 8-B granules
//      {value32, tag} by __hip_atomic_store relaxed agent (one sc1 store each),
//      readers __hip_atomic_load relaxed agent (global_load_dwordx2 sc1);
//   2  form 0 with readers at system scope (aux 17: sc0 sc1);
//   3  form 0, but readers first wait for an agent-scope arrival counter of
//      the iteration (the product's counter hand-off), then read once.
// Output: one line per form: timeouts, wrong values, µs per iteration.
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>

typedef unsigned u4v __attribute__((ext_vector_type(4)));
constexpr int kThreads = 512, kVals = 30, kCols = 16;
constexpr unsigned kSpin = 20000;

__device__ __forceinline__ unsigned lo32(double d) { return (unsigned)__double_as_longlong(d); }
__device__ __forceinline__ unsigned hi32(double d)
{
    return (unsigned)((unsigned long long)__double_as_longlong(d) >> 32);
}

__device__ __forceinline__ double value_of(int row, int v, int k)
{
    return (double)(row * 1000 + v) + 0.25 * (double)k;
}

template <int kForm>
__global__ __launch_bounds__(kThreads, 1) void k_probe(u4v* part, unsigned long long* gran,
                                                       unsigned* arrive, int G, int iters,
                                                       unsigned* timeouts, unsigned* wrong)
{
    const int c = blockIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    unsigned my_to = 0, my_wrong = 0;
    for (int k = 0; k < iters; ++k) {
        const unsigned tag = (unsigned)k + 1u;
        const size_t base = (size_t)(k & 1) * G * kVals;
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
            part + base, (short)0, G * kVals * 16, 0x00020000);
        if (wave == 0 && lane < kVals) {
            const double val = value_of(c, lane, k);
            if (kForm == 1) {
                unsigned long long* g = gran + 2 * (base + (size_t)c * kVals + lane);
                __hip_atomic_store(g, ((unsigned long long)tag << 32) | lo32(val), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(g + 1, ((unsigned long long)tag << 32) | hi32(val),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                const u4v pc = {lo32(val), tag, hi32(val), tag};
                __builtin_amdgcn_raw_buffer_store_b128(pc, r, (c * kVals + lane) * 16, 0, 16);
            }
            if (kForm == 3) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (lane == 0)
                    __hip_atomic_fetch_add(arrive + k, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (kForm == 3) {
            if (threadIdx.x == 0) {
                unsigned s = 0;
                while (__hip_atomic_load(arrive + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
                           (unsigned)G &&
                       ++s < kSpin)
                    __builtin_amdgcn_s_sleep(1);
                if (s >= kSpin) ++my_to;
            }
            __syncthreads();
        }
        for (int e = threadIdx.x; e < kCols * kVals; e += kThreads) {
            const int j = e / kVals, v = e - j * kVals;
            for (int b = j; b < G; b += kCols) {
                unsigned spins = 0;
                double got;
                for (;;) {
                    bool ok;
                    if (kForm == 1) {
                        const unsigned long long* g = gran + 2 * (base + (size_t)b * kVals + v);
                        const unsigned long long a = __hip_atomic_load(g, __ATOMIC_RELAXED,
                                                                       __HIP_MEMORY_SCOPE_AGENT);
                        const unsigned long long h = __hip_atomic_load(g + 1, __ATOMIC_RELAXED,
                                                                       __HIP_MEMORY_SCOPE_AGENT);
                        ok = (unsigned)(a >> 32) == tag && (unsigned)(h >> 32) == tag;
                        got = __hiloint2double((int)(unsigned)h, (int)(unsigned)a);
                    } else {
                        const u4v x = __builtin_bit_cast(
                            u4v, __builtin_amdgcn_raw_buffer_load_b128(r, (b * kVals + v) * 16, 0,
                                                                       kForm == 2 ? 17 : 16));
                        ok = x.y == tag && x.w == tag;
                        got = __hiloint2double((int)x.z, (int)x.x);
                    }
                    if (ok || kForm == 3) {
                        if (!ok) ++my_wrong;
                        break;
                    }
                    if (++spins > kSpin) {
                        ++my_to;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                if (spins <= kSpin && got != value_of(b, v, k)) ++my_wrong;
            }
        }
        __syncthreads();
    }
    if (my_to) atomicAdd(timeouts, my_to);
    if (my_wrong) atomicAdd(wrong, my_wrong);
}

template <int kForm>
static void run(int G, int iters, int reps)
{
    u4v* part;
    unsigned long long* gran;
    unsigned *arrive, *cnt;
    const size_t pieces = (size_t)2 * G * kVals;
    hipMalloc(&part, pieces * 16);
    hipMalloc(&gran, pieces * 16);
    hipMalloc(&arrive, (size_t)iters * reps * sizeof(unsigned));
    hipMalloc(&cnt, 2 * sizeof(unsigned));
    unsigned tot_to = 0, tot_wrong = 0;
    float ms_tot = 0;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int r = 0; r < reps; ++r) {
        hipMemset(part, 0, pieces * 16);
        hipMemset(gran, 0, pieces * 16);
        hipMemset(arrive, 0, (size_t)iters * reps * sizeof(unsigned));
        hipMemset(cnt, 0, 2 * sizeof(unsigned));
        hipEventRecord(e0);
        hipLaunchKernelGGL(k_probe<kForm>, dim3(G), dim3(kThreads), 0, 0, part, gran, arrive, G,
                           iters, cnt, cnt + 1);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        ms_tot += ms;
        unsigned h[2];
        hipMemcpy(h, cnt, sizeof(h), hipMemcpyDeviceToHost);
        tot_to += h[0];
        tot_wrong += h[1];
    }
    printf("form %d: G %d iters %d reps %d  timeouts %u  wrong %u  %.2f us/iteration  (%s)\n", kForm,
           G, iters, reps, tot_to, tot_wrong, ms_tot * 1e3 / (reps * iters),
           hipGetErrorString(hipGetLastError()));
    fflush(stdout);
    hipFree(part);
    hipFree(gran);
    hipFree(arrive);
    hipFree(cnt);
}

int main(int argc, char** argv)
{
    const int form = argc > 1 ? atoi(argv[1]) : -1;
    const int G = argc > 2 ? atoi(argv[2]) : 200;
    const int iters = argc > 3 ? atoi(argv[3]) : 10;
    const int reps = argc > 4 ? atoi(argv[4]) : 5;
    if (G < 1 || G > 256) return 2;  // one workgroup per CU at most: all resident
    if (form < 0 || form == 3) run<3>(G, iters, reps);
    if (form < 0 || form == 1) run<1>(G, iters, reps);
    if (form < 0 || form == 0) run<0>(G, iters, reps);
    if (form < 0 || form == 2) run<2>(G, iters, reps);
    return 0;
}
