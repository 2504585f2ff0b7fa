/*
 * youth_dist.h — multi-process pose gather over RCCL for a plain-C host that
 * runs one process per GPU ("batch of 512 independent
 * pairs sharded across 8 MI355X, RCCL pose gather over xGMI").  Library:
 * libyouth_dist.so (links RCCL; libyouth_icp.so itself does not).
 *
 * Each process aligns its contiguous shard of ONE batch of n_pairs
 * (youth_icp_shard_range(n_pairs, nranks, rank, ...), the split the bench's
 * ranks and youth_icp_align_batch_multi use) and then calls
 * youth_dist_allgather_poses: afterwards every rank holds all n_pairs fp32
 * poses in pair order.  One ncclAllGather of the (padded) largest shard —
 * 64 B per pair, latency-bound over xGMI — plus one compaction kernel.
 * No collective touches the data path (depth frames never cross GPUs).
 *
 * Bootstrap: rank 0 calls youth_dist_unique_id and hands the 128 bytes to
 * every rank out of band (a file, a socket, an environment variable, MPI),
 * as ncclGetUniqueId / ncclCommInitRank require.  Plain C99, no HIP or RCCL
 * types: streams travel as void*.  Return codes are youth_icp.h's YOUTH_*.
 */
#ifndef YOUTH_DIST_H
#define YOUTH_DIST_H

#ifdef __cplusplus
extern "C" {
#endif

#define YOUTH_DIST_ID_BYTES 128 /* NCCL_UNIQUE_ID_BYTES */

typedef struct youth_dist youth_dist;

/* A fresh communicator id (rank 0 only).  YOUTH_OK or a negative code. */
int youth_dist_unique_id(unsigned char id[YOUTH_DIST_ID_BYTES]);

/* Join the communicator of nranks processes as `rank`, on HIP device
 * `device` (collective: every rank calls it with the same id).  NULL on
 * failure (youth_dist_last_error). */
youth_dist* youth_dist_create(int nranks, int rank, int device,
                              const unsigned char id[YOUTH_DIST_ID_BYTES]);

/* Gather every rank's shard of a batch of n_pairs poses.  d_local: DEVICE
 * [count][16] fp32, this rank's rows (count from youth_icp_shard_range);
 * d_all: DEVICE [n_pairs][16] fp32, receives all rows in pair order (may not
 * overlap d_local).  Enqueued on `stream` (hipStream_t as void*, NULL = the
 * default stream) and asynchronous, like any RCCL collective: every rank
 * must call it with the same n_pairs, in the same order.  Calls of one
 * communicator share its scratch rows, so they are ordered across streams:
 * a call from a stream other than the previous call's first waits for all
 * work enqueued on that previous stream (one event, only at a switch), so
 * double-buffered callers on two streams never mix batches.  Not
 * thread-safe: one host thread per communicator. */
int youth_dist_allgather_poses(youth_dist* d, const float* d_local, int n_pairs, float* d_all,
                               void* stream);

/* The same from HOST memory (plain-C hosts that used youth_icp_align_batch):
 * h_local [count][16] fp32, h_all [n_pairs][16] fp32; staged through the
 * communicator's device buffers on its own stream; synchronous. */
int youth_dist_allgather_poses_host(youth_dist* d, const float* h_local, int n_pairs,
                                    float* h_all);

/* Where row `row` of a gathered batch comes from: *rank's shard, its row
 * *index (the mapping youth_dist_allgather_poses applies; host-side, for
 * callers that gather by other means).  YOUTH_OK or YOUTH_EINVAL. */
int youth_dist_row_source(int n_pairs, int nranks, int row, int* rank, int* index);

int youth_dist_nranks(const youth_dist* d);
int youth_dist_rank(const youth_dist* d);
void youth_dist_destroy(youth_dist* d);

/* Text of the last error on this thread ("" if none). */
const char* youth_dist_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* YOUTH_DIST_H */
