#!/bin/bash
# The N = 8 / N = 4 shards (64 / 128 pairs) on one GPU: steps in flight x
# k_icp slot share (bench --pipeline / --share), interleaved, two rounds.
set -eo pipefail
for r in 1 2; do
  for n in 64 128; do
    for cfg in "1 1" "2 2" "3 3" "4 4" "2 1"; do
      set -- $cfg
      timeout -k 10 200 python3 bench.py --global-pairs $n --pipeline $1 --share $2 --steps 40 --warmup 5 \
          --windows 2 --no-legs --no-viewer --no-spec-parity --no-host-io --no-cpu-baseline > gpurun_out/sp.json
      python3 -c "
import json; d=json.loads(open('gpurun_out/sp.json').read().strip().splitlines()[-1])
print('round $r pairs $n pipeline $1 share $2:', round(d['value']), [round(v) for v in d['window_rates']])"
    done
  done
done
