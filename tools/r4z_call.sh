#!/bin/bash
# Round-4 GPU call z: N = 8's per-rank shard (64 of the 512 pairs) against the
# 512-pair batch on one box, the current build, alternating, two rounds each.
set -o pipefail
O=gpurun_out
: > $O/shard64_r4z.txt
for r in 1 2; do
  for p in 512 64; do
    timeout -k 10 240 python3 bench.py --global-pairs $p --steps 30 --warmup 5 --no-cpu-baseline --no-host-io \
        --no-legs --no-spec-parity --no-viewer > $O/shard_${p}_$r.json 2> /dev/null || exit 1
    python3 -c "
import json,sys
d=json.loads(open('$O/shard_${p}_$r.json').read().strip().splitlines()[-1])
print('pairs $p round $r: %.0f aligns/s  k_icp %.1f us  k_prep %.1f us  %s' % (d['value'], d['roofline']['avg_launch_ms']*1e3, d['kernel_ms_per_step']['k_prep']*1e3, d['config'].get('k_icp_slot_share')))
" >> $O/shard64_r4z.txt
  done
done
echo all done
