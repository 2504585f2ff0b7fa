#!/usr/bin/env python3
"""Make a phase-instrumented copy of icp_kernels.hip (A/B tooling only; the
product kernel is never built this way).

Thread 0 of every k_icp workgroup stamps s_memtime at each step of a work
item and, at exit, adds its per-phase cycle totals into spare words of the
queue buffer (after kQWords); youth_icp_destroy prints them.  The stamps
change register allocation, so compare instrumented builds with each other,
not with the product build.

Usage: tools/phase_patch.py <in.hip> <out.hip>; then tools/ab_build.sh <name> <out.hip>
"""
import sys

s = open(sys.argv[1]).read()


def rep(a, b):
    global s
    assert s.count(a) == 1, "pattern not found once: " + a[:90]
    s = s.replace(a, b)


PH = "is.head + (kQWords - kQHead)"  # 8 u64 counters after the queue words

rep('''    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;

    if (threadIdx.x == 0) {
        const int first''', '''    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long ta = 0, tb = 0, tc = 0, td = 0, tf = 0;
#define PH_STAMP(v) v = __builtin_amdgcn_s_memtime()

    if (threadIdx.x == 0) {
        const int first''')
rep('''        const int item = __builtin_amdgcn_readfirstlane(sh_item);
        if (item >= total) return;''', '''        const int item = __builtin_amdgcn_readfirstlane(sh_item);
        PH_STAMP(ta);
        if (tf) ph[5] += ta - tf;  // item barrier
        if (item >= total) {
            if (threadIdx.x == 0) {
                unsigned long long* g = reinterpret_cast<unsigned long long*>(''' + PH + ''');
                for (int q = 0; q < 8; ++q)
                    __hip_atomic_fetch_add(g + q, ph[q], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
            }
            return;
        }''')
rep('''                                                 end, W, H, K, F, thr2, acc, nullptr);
        {
            double tot;''', '''                                                 end, W, H, K, F, thr2, acc, nullptr);
        PH_STAMP(tb);
        ph[0] += tb - ta;  // pixel loop
        ph[6] += 1;        // items
        {
            double tot;''')
rep('''            if (!(lane & 1) && (lane >> 1) < kNeq) red[wave][lane >> 1] = tot;
        }
        __syncthreads();
''', '''            if (!(lane & 1) && (lane >> 1) < kNeq) red[wave][lane >> 1] = tot;
        }
        __syncthreads();
        PH_STAMP(tc);
        ph[1] += tc - tb;  // reduce-scatter + LDS + barrier
''')
rep('''            ticket = __shfl(ticket, 0, 64);
            if (ticket == (unsigned)is.nblk - 1) {''', '''            ticket = __shfl(ticket, 0, 64);
            PH_STAMP(td);
            ph[2] += td - tc;  // publish + ticket
            if (ticket == (unsigned)is.nblk - 1) {''')
rep('''                    st_u32_sc1(is.epoch + p, (unsigned)(k + 1));
                }
            }''', '''                    st_u32_sc1(is.epoch + p, (unsigned)(k + 1));
                }
                unsigned long long te;
                PH_STAMP(te);
                ph[3] += te - td;  // last-arriver sum + solve + publish
                ph[7] += 1;        // solves
                td = te;
            }''')
rep('''                sh_item = icp_claim(is, next, total, per_iter, sh_T);
            }
        }
        __syncthreads();''', '''                sh_item = icp_claim(is, next, total, per_iter, sh_T);
            }
            PH_STAMP(tf);
            ph[4] += tf - td;  // dequeue + epoch wait + pose load
        }
        __syncthreads();''')
rep('hipMalloc(&c->d_head, kQWords * 4)', 'hipMalloc(&c->d_head, kQWords * 4 + 64)')
rep('hipMemset(c->d_head, 0, kQWords * 4)', 'hipMemset(c->d_head, 0, kQWords * 4 + 64)')
rep('''void youth_icp_destroy(youth_icp_ctx* c)
{''', '''void youth_icp_destroy(youth_icp_ctx* c)
{
    if (c && c->d_head) {
        unsigned long long g[8];
        if (hipMemcpy(g, c->d_head + kQWords, sizeof(g), hipMemcpyDeviceToHost) == hipSuccess &&
            g[6]) {
            const char* nm[6] = {"pixel loop", "reduce+barrier", "publish+ticket",
                                 "solve(last)", "dequeue+claim", "item barrier"};
            fprintf(stderr, "[phases] items %llu solves %llu; thread-0 cycles per item:\\n", g[6],
                    g[7]);
            for (int q = 0; q < 6; ++q)
                fprintf(stderr, "[phases]   %-16s %10.0f%s\\n", nm[q],
                        (double)g[q] / (double)(q == 3 ? (g[7] ? g[7] : 1) : g[6]),
                        q == 3 ? "  (per solve)" : "");
        }
    }''')
open(sys.argv[2], 'w').write(s)
