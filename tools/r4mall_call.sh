#!/bin/bash
# Round-4 probe: does a batch whose records fit the 256 MB Infinity Cache run
# k_icp faster per pixel-iteration?  512 pairs (2.5 GB of records) vs 48 / 32
# pairs (235 / 157 MB), one step in flight, two rounds.
set -o pipefail
: > gpurun_out/mall_probe_r4.txt
for r in 1 2; do
  for p in 512 48 32; do
    timeout -k 10 240 python3 bench.py --global-pairs $p --pipeline 1 --steps 30 --warmup 5 --no-cpu-baseline \
        --no-host-io --no-legs --no-spec-parity --no-viewer > gpurun_out/mall_$p.$r.json 2>/dev/null || exit 1
    python3 -c "
import json
d=json.loads(open('gpurun_out/mall_$p.$r.json').read().strip().splitlines()[-1])
r=d['roofline']; px=$p*640*480*10
print('pairs %3d round $r: %.0f aligns/s  k_icp %.1f us = %.3f ps per px-iter  frac %.3f  sched %s' % ($p, d['value'], r['avg_launch_ms']*1e3, r['avg_launch_ms']*1e9/px, r['frac'], d.get('sched_last_step')))
" >> gpurun_out/mall_probe_r4.txt
  done
done
echo all done
