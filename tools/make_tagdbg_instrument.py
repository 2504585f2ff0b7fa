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
                        if (slot < 512) {
                            unsigned* r = tag_dbg + 16 + slot * 16;
                            int bad = 0;
#pragma unroll
                            for (int i = kBatch - 1; i >= 0; --i)
                                if ((x[i].y != tag) | (x[i].w != tag)) bad = i;
                            u4v xb = x[0];
#pragma unroll
                            for (int i = 0; i < kBatch; ++i)
                                if (i == bad) xb = x[i];
                            r[0] = blockIdx.x; r[1] = threadIdx.x; r[2] = (unsigned)bb; r[3] = (unsigned)v;
                            r[4] = tag; r[5] = spins; r[6] = (unsigned)(bb + bad * kSumCols);
                            r[7] = xb.x; r[8] = xb.y; r[9] = xb.z; r[10] = xb.w; r[11] = (unsigned)nblk;
                            const u4v again = __builtin_bit_cast(u4v, __builtin_amdgcn_raw_buffer_load_b128(
                                rpart, ((bb + bad * kSumCols) * kPartStride + v) * 16, 0, 17));
                            r[12] = again.y; r[13] = again.w; r[14] = again.x; r[15] = 0xabcd1234u;
                        }
                    }
                    __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);''')
rep('''sum_pair_rows_tagged<16, kThreads>(rpart, G, colsum, tag, err, kCoopSpinMax, &sh_stop)''',
    '''sum_pair_rows_tagged<16, kThreads>(rpart, G, colsum, tag, err, 20000u, &sh_stop)''')
open(sys.argv[2], "w").write(s)
