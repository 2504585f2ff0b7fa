#!/bin/bash
# Round-4 GPU call: the 512-pair bench step with one step in flight (default)
# against two contexts / two steps in flight (k_icp on half or all of the
# slots), current build, interleaved, three rounds.
set -o pipefail
EXTRA="--no-legs --no-spec-parity --no-viewer" tools/ab_run.sh 1 p1=cur > /dev/null 2>&1 || true
for r in 1 2 3; do
  for cfg in "p1 --pipeline 1" "p2s2 --pipeline 2 --share 2" "p2s1 --pipeline 2 --share 1"; do
    set -- $cfg; label=$1; shift
    timeout -k 10 240 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-host-io --no-legs \
        --no-spec-parity --no-viewer "$@" > gpurun_out/pipe_$label.$r.json 2>/dev/null || exit 1
    python3 -c "
import json
d=json.loads(open('gpurun_out/pipe_$label.$r.json').read().strip().splitlines()[-1])
print('%5s round $r: %.0f aligns/s  k_icp %.1f us  k_prep %.1f us  %s' % ('$label', d['value'], d['roofline']['avg_launch_ms']*1e3, d['kernel_ms_per_step']['k_prep']*1e3, d['config'].get('k_icp_slot_share')))
" >> gpurun_out/pipe512_r4.txt
  done
done
echo all done
