#!/bin/bash
# Same-box A/B of k_icp's work queues (YOUTH_ICP_QUEUES 1 vs 8) at the
# per-GPU shards of N = 8 / 4 / 1 (64 / 128 / 512 pairs), 2 rounds.
# Usage: tools/queues_ab.sh <tag> [extra bench args]   (on the GPU box)
set -euo pipefail
OUT=$(pwd)/gpurun_out/qab_${1:-a}; shift || true
mkdir -p $OUT
B="--no-legs --no-cpu-baseline --no-viewer --no-host-io --no-spec-parity --windows 2 --pipeline 1 $*"
for r in 1 2; do for n in 64 128 512; do for q in 1 8; do
    YOUTH_ICP_QUEUES=$q timeout -k 10 120 python bench.py $B --global-pairs $n > $OUT/b_${n}_q${q}_$r.json
    python3 -c "import json; d=json.load(open('$OUT/b_${n}_q${q}_$r.json')); print('pairs $n queues $q round $r', round(d['value']), 'windows', [round(x) for x in d['window_rates']], 'k_icp_ms', round(d['roofline']['avg_launch_ms'], 4), 'ms_per_step', round(d['ms_per_step'], 4), d['sched_last_step'])" >> $OUT/ab.txt
done; done; done
echo done
