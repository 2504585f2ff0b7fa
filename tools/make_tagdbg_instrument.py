#!/usr/bin/env python3
"""tools/make_tagdbg.sh helper: timeout records and a short spin bound in the
tagged-partials experiment source (argv[1] -> argv[2]).  Probe only."""
import sys

s = open(sys.argv[1]).read()


def rep(a, b):
    global s
    assert s.count(a) == 1, a[:80]
    s = s.replace(a, b)


rep('''template <int kBatch, int kThreads>
__device__ __forceinline__ double sum_pair_rows_tagged(''', '''__device__ unsigned* tag_dbg;  // tools/tagdbg: timeout records
template <int kBatch, int kThreads>
__device__ __forceinline__ double sum_pair_rows_tagged(''')
rep('''                if (++spins > spin_max || ld_u32_sc1(err) != 0u) {
                    __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);''', '''                if (++spins > spin_max || ld_u32_sc1(err) != 0u) {
                    if (tag_dbg && spins > spin_max) {
                        const unsigned slot = atomicAdd(tag_dbg, 1u);
                        if (slot < 256) {
                            unsigned* r = tag_dbg + 64 + slot * 64;
                            unsigned badm = 0;
#pragma unroll
                            for (int i = 0; i < kBatch; ++i) {
                                const int b = bb + i * kSumCols;
                                badm |= ((x[i].y != tag) | (x[i].w != tag)) ? (1u << i) : 0u;
                                r[8 + i] = x[i].y;  // tag the poll last saw
                                const u4v again = __builtin_bit_cast(u4v, __builtin_amdgcn_raw_buffer_load_b128(
                                    rpart, (b < nblk ? b : 0) * kPartStride * 16 + v * 16, 0, 17));
                                r[24 + i] = again.y;  // tag a system-scope load sees now
                                const u4v again1 = __builtin_bit_cast(u4v, __builtin_amdgcn_raw_buffer_load_b128(
                                    rpart, (b < nblk ? b : 0) * kPartStride * 16 + v * 16, 0, POLL_AUX));
                                r[40 + i] = again1.y;  // tag one more poll-form load sees now
                            }
                            r[0] = blockIdx.x; r[1] = threadIdx.x; r[2] = (unsigned)bb; r[3] = (unsigned)v;
                            r[4] = tag; r[5] = spins; r[6] = badm; r[7] = (unsigned)nblk;
                            r[63] = 0xabcd1234u;
                        }
                    }
                    __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);''')
aux = sys.argv[3] if len(sys.argv) > 3 else "16"
s = s.replace("#include <hip/hip_runtime.h>", "#include <hip/hip_runtime.h>\n#define POLL_AUX " + aux, 1)
s = s.replace("rpart, (b * kPartStride + v) * 16, 0, 16)", "rpart, (b * kPartStride + v) * 16, 0, POLL_AUX)")
rep('''sum_pair_rows_tagged<16, kThreads>(rpart, G, colsum, tag, err, kCoopSpinMax, &sh_stop)''',
    '''sum_pair_rows_tagged<16, kThreads>(rpart, G, colsum, tag, err, 20000u, &sh_stop)''')
open(sys.argv[2], "w").write(s)
