#!/bin/bash
# Same-box A/B of bench.py --pipeline 1 vs 2 at the per-GPU shards of
# N = 8 / 4 / 1 (64 / 128 / 512 pairs), 2 rounds each.
# Usage: tools/pipeline_ab.sh <tag>   (on the GPU box)
set -euo pipefail
OUT=$(pwd)/gpurun_out/pipeab_${1:-a}
mkdir -p $OUT
B="--no-legs --no-cpu-baseline --no-viewer --no-host-io --no-spec-parity --windows 2"
for r in 1 2; do for n in 64 128 512; do for p in 1 2; do
    timeout -k 10 120 python bench.py $B --global-pairs $n --pipeline $p > $OUT/b_${n}_p${p}_$r.json
    python3 -c "import json; d=json.load(open('$OUT/b_${n}_p${p}_$r.json')); print('pairs $n pipeline $p round $r', round(d['value']), 'windows', [round(x) for x in d['window_rates']], 'k_icp_ms', round(d['roofline']['avg_launch_ms'], 4), 'ms_per_step', round(d['ms_per_step'], 4))" >> $OUT/ab.txt
done; done; done
echo done
