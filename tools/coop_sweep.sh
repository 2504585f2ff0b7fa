#!/bin/bash
# Small-batch A/B on the GPU box: k_icp_coop (planned, and PXS="5 8 .." forced
# pixels per lane) vs the persistent
# k_icp (YOUTH_ICP_NO_COOP=1), pairs 1/2/4, interleaved in one process tree.
# Usage: tools/coop_sweep.sh [rounds]
set -uo pipefail
R=${1:-2}
one() {  # label env... -- bench args
    local label=$1; shift
    local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
    local out
    out=$(env "${envs[@]}" timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-host-io "$@") || { echo "$label FAILED"; return 1; }
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); k=d['kernel_ms_per_step']; print(f\"{sys.argv[2]:34s} {d['value']:9.0f} aligns/s  ms/step {d['ms_per_step']*1e3:7.1f} us  icp {k['k_reduce']*1e3:7.1f} us  prep {k['k_prep']*1e3:5.1f} us\")" "$out" "$label"
}
for r in $(seq 1 $R); do
  for np in ${NPS:-1 2 4}; do
    S=$((200 / np + 20))
    one "pairs=$np persistent" YOUTH_ICP_NO_COOP=1 -- --pairs-per-gpu $np --steps $S --warmup 20 || exit 1
    one "pairs=$np coop planned 512" YOUTH_ICP_COOP_MAX_PAIRS=16 -- --pairs-per-gpu $np --steps $S --warmup 20 || exit 1
    one "pairs=$np coop planned 256" YOUTH_ICP_COOP_THREADS=256 YOUTH_ICP_COOP_MAX_PAIRS=16 -- --pairs-per-gpu $np --steps $S --warmup 20 || exit 1
    for px in ${PXS:-}; do
      one "pairs=$np coop px=$px" YOUTH_ICP_COOP_PX=$px YOUTH_ICP_COOP_MAX_PAIRS=16 -- --pairs-per-gpu $np --steps $S --warmup 20 || exit 1
    done
  done
done
