#!/bin/bash
# k_icp chunk target per shard size (YOUTH_ICP_TARGET_CHUNKS), one box.
for gp in ${PAIRS:-64 128}; do
  for tc in ${CHUNKS:-2048 2560 3072}; do
    YOUTH_ICP_TARGET_CHUNKS=$tc timeout -k 10 120 python3 bench.py --global-pairs $gp --steps 40 --warmup 5 --windows 1 --no-cpu-baseline --no-host-io --no-legs --no-viewer > gpurun_out/cs_${gp}_${tc}.json 2>/dev/null || exit 1
    python3 -c "
import json;d=json.load(open('gpurun_out/cs_${gp}_${tc}.json'))
print('pairs ${gp} chunks ${tc}: %.0f aligns/s (window %.0f)  k_icp %.1f us  sched %s' % (d['value'], d['window_rates'][0], d['roofline']['avg_launch_ms']*1e3, d['sched_last_step']))"
  done
done
