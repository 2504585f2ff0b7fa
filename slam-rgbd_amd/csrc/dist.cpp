// dist.cpp — youth_dist.h: the multi-process RCCL pose gather.
//
// The C4 exchange is one all-gather of fp32 3x4-in-4x4 poses, 64 B per pair
// (<= 64 x 64 B per rank at 8 GPUs): latency-bound over xGMI, so it is ONE
// ncclAllGather of the padded largest shard into a per-communicator scratch
// buffer, then one small kernel (k_compact) that drops the padding and lands
// every rank's rows at its shard's offset.  Both on the caller's stream.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <string>

#include "youth_dist.h"
#include "youth_icp.h"

struct youth_dist {
    ncclComm_t comm = nullptr;
    int nranks = 0, rank = 0, device = 0;
    float* scratch = nullptr;  // [nranks][max_count][16]
    size_t scratch_rows = 0;
    float* staging = nullptr;  // host variant: [max_count + n_pairs][16]
    size_t staging_rows = 0;
    hipStream_t stream = nullptr;  // host variant's stream
    // every gather stages through `scratch`: calls are ordered across streams
    // (`order` is recorded on a gather's stream right after it; a call from
    // another stream waits on it), so double-buffering callers on two streams
    // cannot mix batches in the scratch rows
    hipStream_t last = nullptr;
    bool any = false;
    hipEvent_t order = nullptr;
};

static thread_local std::string g_err;

// Row r of a batch of n pairs split over k ranks (youth_icp_shard_range: the
// first n % k shards hold one row more) is row i of rank q's shard.
__host__ __device__ static inline void row_source(int n, int k, int r, int* q, int* i)
{
    const int Q = n / k, m = n % k;
    if (r < m * (Q + 1)) {
        *q = r / (Q + 1);
        *i = r - *q * (Q + 1);
    } else {
        const int rr = r - m * (Q + 1);
        *q = m + rr / Q;
        *i = rr - (*q - m) * Q;
    }
}

// out row r (16 floats = four float4) <- scratch slot of its rank, row i
__global__ void k_compact(const float4* __restrict__ scratch, int max_count, int n, int k,
                          float4* __restrict__ out)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * 4) return;
    int q, i;
    row_source(n, k, t >> 2, &q, &i);
    out[t] = scratch[((size_t)q * max_count + i) * 4 + (t & 3)];
}

__attribute__((format(printf, 2, 3))) static int fail(int code, const char* fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

extern "C" {

const char* youth_dist_last_error(void) { return g_err.c_str(); }

int youth_dist_unique_id(unsigned char id[YOUTH_DIST_ID_BYTES])
{
    static_assert(YOUTH_DIST_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "id size");
    if (!id) return fail(YOUTH_EINVAL, "unique_id: null");
    ncclUniqueId u;
    const ncclResult_t r = ncclGetUniqueId(&u);
    if (r != ncclSuccess) return fail(YOUTH_EHIP, "ncclGetUniqueId: %s", ncclGetErrorString(r));
    memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
    return YOUTH_OK;
}

youth_dist* youth_dist_create(int nranks, int rank, int device,
                              const unsigned char id[YOUTH_DIST_ID_BYTES])
{
    if (nranks < 1 || rank < 0 || rank >= nranks || !id) {
        fail(YOUTH_EINVAL, "dist_create: bad arguments (nranks %d, rank %d)", nranks, rank);
        return nullptr;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
        fail(YOUTH_ENODEV, "dist_create: no HIP device %d", device);
        return nullptr;
    }
    if (hipSetDevice(device) != hipSuccess) {
        fail(YOUTH_EHIP, "dist_create: hipSetDevice(%d)", device);
        return nullptr;
    }
    ncclUniqueId u;
    memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
    auto* d = new youth_dist();
    d->nranks = nranks;
    d->rank = rank;
    d->device = device;
    const ncclResult_t r = ncclCommInitRank(&d->comm, nranks, u, rank);
    if (r != ncclSuccess) {
        fail(YOUTH_EHIP, "ncclCommInitRank: %s", ncclGetErrorString(r));
        delete d;
        return nullptr;
    }
    return d;
}

int youth_dist_allgather_poses(youth_dist* d, const float* d_local, int n_pairs, float* d_all,
                               void* stream)
{
    if (!d || !d_all || n_pairs < 0) return fail(YOUTH_EINVAL, "allgather_poses: bad arguments");
    if (n_pairs == 0) return YOUTH_OK;
    int first = 0, count = 0;
    youth_icp_shard_range(n_pairs, d->nranks, d->rank, &first, &count);
    const int max_count = (n_pairs + d->nranks - 1) / d->nranks;  // rank 0's shard
    if (count > 0 && !d_local) return fail(YOUTH_EINVAL, "allgather_poses: null d_local");
    if (hipSetDevice(d->device) != hipSuccess) return fail(YOUTH_EHIP, "hipSetDevice");
    const hipStream_t s = (hipStream_t)stream;
    if (!d->order && hipEventCreateWithFlags(&d->order, hipEventDisableTiming) != hipSuccess)
        return fail(YOUTH_EHIP, "hipEventCreate");
    // stream switch: wait for the previous gather through the event recorded
    // on ITS stream right after it (below); the previous stream's handle is
    // never used again (the caller may have destroyed it)
    if (d->any && d->last != s && hipStreamWaitEvent(s, d->order, 0) != hipSuccess)
        return fail(YOUTH_EHIP, "hipStreamWaitEvent");
    d->last = s;
    const size_t rows = (size_t)d->nranks * max_count;
    if (rows > d->scratch_rows) {
        // a previous gather may still read the old scratch on some stream
        if (d->scratch && (hipDeviceSynchronize() != hipSuccess || hipFree(d->scratch) != hipSuccess))
            return fail(YOUTH_EHIP, "hipFree scratch");
        d->scratch = nullptr;
        d->scratch_rows = 0;
        if (hipMalloc(&d->scratch, rows * 16 * sizeof(float)) != hipSuccess)
            return fail(YOUTH_EHIP, "hipMalloc scratch (%zu rows)", rows);
        d->scratch_rows = rows;
    }
    // this rank's rows (padded to max_count) into its slot: the all-gather
    // sends from the slot in place (sendbuff == recvbuff + rank * count)
    float* mine = d->scratch + (size_t)d->rank * max_count * 16;
    if (count > 0 &&
        hipMemcpyAsync(mine, d_local, (size_t)count * 16 * sizeof(float), hipMemcpyDeviceToDevice,
                       s) != hipSuccess)
        return fail(YOUTH_EHIP, "hipMemcpyAsync local rows");
    const ncclResult_t r = ncclAllGather(mine, d->scratch, (size_t)max_count * 16, ncclFloat32,
                                         d->comm, s);
    if (r != ncclSuccess) return fail(YOUTH_EHIP, "ncclAllGather: %s", ncclGetErrorString(r));
    hipLaunchKernelGGL(k_compact, dim3((n_pairs * 4 + 255) / 256), dim3(256), 0, s,
                       (const float4*)d->scratch, max_count, n_pairs, d->nranks, (float4*)d_all);
    if (hipGetLastError() != hipSuccess) return fail(YOUTH_EHIP, "k_compact launch");
    if (hipEventRecord(d->order, s) != hipSuccess) return fail(YOUTH_EHIP, "hipEventRecord");
    d->any = true;
    return YOUTH_OK;
}

int youth_dist_allgather_poses_host(youth_dist* d, const float* h_local, int n_pairs,
                                    float* h_all)
{
    if (!d || !h_all || n_pairs < 0) return fail(YOUTH_EINVAL, "allgather_poses_host: bad arguments");
    if (n_pairs == 0) return YOUTH_OK;
    int first = 0, count = 0;
    youth_icp_shard_range(n_pairs, d->nranks, d->rank, &first, &count);
    if (count > 0 && !h_local) return fail(YOUTH_EINVAL, "allgather_poses_host: null h_local");
    if (hipSetDevice(d->device) != hipSuccess) return fail(YOUTH_EHIP, "hipSetDevice");
    if (!d->stream && hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking) != hipSuccess)
        return fail(YOUTH_EHIP, "hipStreamCreate");
    const size_t rows = (size_t)count + n_pairs;
    if (rows > d->staging_rows) {
        if (d->staging && (hipStreamSynchronize(d->stream) != hipSuccess ||
                           hipFree(d->staging) != hipSuccess))
            return fail(YOUTH_EHIP, "hipFree staging");
        d->staging = nullptr;
        d->staging_rows = 0;
        if (hipMalloc(&d->staging, rows * 16 * sizeof(float)) != hipSuccess)
            return fail(YOUTH_EHIP, "hipMalloc staging (%zu rows)", rows);
        d->staging_rows = rows;
    }
    float* d_local = d->staging;
    float* d_all = d->staging + (size_t)count * 16;
    if (count > 0 && hipMemcpyAsync(d_local, h_local, (size_t)count * 16 * sizeof(float),
                                    hipMemcpyHostToDevice, d->stream) != hipSuccess)
        return fail(YOUTH_EHIP, "hipMemcpyAsync H2D");
    const int rc = youth_dist_allgather_poses(d, d_local, n_pairs, d_all, d->stream);
    if (rc) {
        (void)hipStreamSynchronize(d->stream);
        return rc;
    }
    if (hipMemcpyAsync(h_all, d_all, (size_t)n_pairs * 16 * sizeof(float), hipMemcpyDeviceToHost,
                       d->stream) != hipSuccess ||
        hipStreamSynchronize(d->stream) != hipSuccess)
        return fail(YOUTH_EHIP, "D2H / sync");
    return YOUTH_OK;
}

int youth_dist_row_source(int n_pairs, int nranks, int row, int* rank, int* index)
{
    if (n_pairs < 1 || nranks < 1 || row < 0 || row >= n_pairs || !rank || !index)
        return fail(YOUTH_EINVAL, "row_source: bad arguments");
    row_source(n_pairs, nranks, row, rank, index);
    return YOUTH_OK;
}

int youth_dist_nranks(const youth_dist* d) { return d ? d->nranks : 0; }
int youth_dist_rank(const youth_dist* d) { return d ? d->rank : -1; }

void youth_dist_destroy(youth_dist* d)
{
    if (!d) return;
    (void)hipSetDevice(d->device);
    // the last gather (on whichever stream) completes before the
    // communicator and the scratch it uses go away
    if (d->stream) (void)hipStreamSynchronize(d->stream);
    if (d->any && d->order) (void)hipEventSynchronize(d->order);
    if (d->comm) (void)ncclCommDestroy(d->comm);
    if (d->order) (void)hipEventDestroy(d->order);
    if (d->scratch) (void)hipFree(d->scratch);
    if (d->staging) (void)hipFree(d->staging);
    if (d->stream) (void)hipStreamDestroy(d->stream);
    delete d;
}

}  // extern "C"
