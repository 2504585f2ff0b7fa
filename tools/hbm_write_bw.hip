// HBM ceilings for k_prep's traffic shape on one MI355X (tools only, not the
// product): 512 frames x 640 x 480 px; per pixel k_prep reads 2 B of depth
// and writes one 16-byte record.  Kernels (grid-stride, 256 threads, 4096
// workgroups):
//   write16   16 B/px of non-temporal stores, no reads;
//   write16p  the same with plain stores;
//   read16    16 B/px of loads over the 2.52 GB record buffer (the read
//             ceiling k_icp's 18 B/px-iteration stream is measured against);
//   read2     2 B/px of loads (8 B per lane: 4 px), summed so nothing is dead;
//   mix       read 2 B + write 16 B per px (k_prep's bytes, no arithmetic),
//             one lane-contiguous store per px.
// Prints GB/s of algorithmic bytes per kernel (median of 20 after 3 warm-ups).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

typedef unsigned int u4v __attribute__((ext_vector_type(4)));

__global__ void k_write16(u4v* out, long long n, int nt)
{
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        const u4v v = {(unsigned)i, 1u, 2u, 3u};
        if (nt)
            __builtin_nontemporal_store(v, out + i);
        else
            out[i] = v;
    }
}

__global__ void k_read2(const short4* in, int n4, unsigned* sink)
{
    unsigned acc = 0;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
        const short4 d = in[i];
        acc += (unsigned)(d.x + d.y + d.z + d.w);
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void k_mix(const short4* in, u4v* out, int n4)
{
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
        const short4 d = in[i];
        u4v* o = out + 4 * i;
        __builtin_nontemporal_store((u4v){(unsigned)d.x, 0u, 0u, 0u}, o + 0);
        __builtin_nontemporal_store((u4v){(unsigned)d.y, 0u, 0u, 0u}, o + 1);
        __builtin_nontemporal_store((u4v){(unsigned)d.z, 0u, 0u, 0u}, o + 2);
        __builtin_nontemporal_store((u4v){(unsigned)d.w, 0u, 0u, 0u}, o + 3);
    }
}

__global__ void k_read16(const u4v* in, long long n, unsigned* sink)
{
    unsigned acc = 0;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        const u4v v = in[i];
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void k_mix2(const short* in, u4v* out, long long n)
{
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        __builtin_nontemporal_store((u4v){(unsigned)in[i], 0u, 0u, 0u}, out + i);
}

int main()
{
    const long long px = 512LL * 640 * 480;  // 157,286,400
    float4* out;
    short4* in;
    unsigned* sink;
    if (hipMalloc(&out, px * 16) || hipMalloc(&in, px * 2) || hipMalloc(&sink, 4)) return 1;
    hipMemset(in, 1, px * 2);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto run = [&](const char* name, double bytes, auto launch) {
        std::vector<float> ms;
        for (int r = 0; r < 23; ++r) {
            hipEventRecord(a);
            launch();
            hipEventRecord(b);
            hipEventSynchronize(b);
            float t;
            hipEventElapsedTime(&t, a, b);
            if (r >= 3) ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        const float med = ms[ms.size() / 2];
        printf("%-22s %8.3f ms  %7.0f GB/s\n", name, med, bytes / (med * 1e-3) / 1e9);
    };
    char name[64];
    for (int blk : {256, 512}) {
        for (int grid : {1024, 4096, 16384, 65536}) {
            snprintf(name, sizeof name, "write16 g%d b%d", grid, blk);
            run(name, px * 16.0, [&] { hipLaunchKernelGGL(k_write16, dim3(grid), dim3(blk), 0, 0, (u4v*)out, px, 1); });
        }
    }
    // the read side: 16-B loads over the same 2.52 GB (the records buffer),
    // several shapes (k_icp streams 18 B/px-iteration of reads)
    for (int blk : {256, 512}) {
        for (int grid : {1024, 4096, 16384, 65536}) {
            snprintf(name, sizeof name, "read16 g%d b%d", grid, blk);
            run(name, px * 16.0, [&] { hipLaunchKernelGGL(k_read16, dim3(grid), dim3(blk), 0, 0, (const u4v*)out, px, sink); });
        }
    }
    run("write16p", px * 16.0, [&] { hipLaunchKernelGGL(k_write16, dim3(16384), dim3(256), 0, 0, (u4v*)out, px, 0); });
    run("read2", px * 2.0, [&] { hipLaunchKernelGGL(k_read2, dim3(4096), dim3(256), 0, 0, in, (int)(px / 4), sink); });
    // one store per px (lane-contiguous), the 2 B read alongside
    run("mix", px * 18.0, [&] { hipLaunchKernelGGL(k_mix2, dim3(16384), dim3(256), 0, 0, (const short*)in, (u4v*)out, px); });
    return 0;
}
