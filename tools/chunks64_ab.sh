#!/bin/bash
# Chunk target at N = 8's 64-pair shard (YOUTH_ICP_TARGET_CHUNKS), current build, 2 rounds;
# plus --pipeline 2 at the default target.  Usage: tools/chunks64_ab.sh <tag>
set -euo pipefail
OUT=$(pwd)/gpurun_out/c64_${1:-a}
mkdir -p $OUT
B="--no-legs --no-cpu-baseline --no-viewer --no-host-io --no-spec-parity --windows 2 --global-pairs 64"
for r in 1 2; do
  for t in 1024 1280 1536 2048 2560; do
    YOUTH_ICP_TARGET_CHUNKS=$t timeout -k 10 120 python bench.py $B --pipeline 1 > $OUT/b_${t}_$r.json
    python3 -c "import json; d=json.load(open('$OUT/b_${t}_$r.json')); print('chunks $t round $r', round(d['value']), [round(x) for x in d['window_rates']], 'k_icp_ms', round(d['roofline']['avg_launch_ms'], 4), d['sched_last_step'])" >> $OUT/ab.txt
  done
  timeout -k 10 120 python bench.py $B --pipeline 2 > $OUT/b_p2_$r.json
  python3 -c "import json; d=json.load(open('$OUT/b_p2_$r.json')); print('pipeline 2 round $r', round(d['value']), [round(x) for x in d['window_rates']])" >> $OUT/ab.txt
done
echo done
