#!/bin/bash
# Round 5, exact reduction: the per-GPU shard rates of the strong-scaling
# points (512 / 256 / 128 / 64 pairs = N 1 / 2 / 4 / 8) on one GPU, and
# k_icp_coop's per-iteration phases for C2 and C3 (tools/coopbench).
set -eo pipefail
for n in 512 256 128 64; do
  timeout -k 10 200 python3 bench.py --global-pairs $n --steps 30 --warmup 5 --windows 2 --no-legs --no-viewer \
      --no-spec-parity --no-host-io --no-cpu-baseline > gpurun_out/shard_$n.json
  python3 -c "
import json; d=json.loads(open('gpurun_out/shard_$n.json').read().strip().splitlines()[-1])
print('$n pairs', round(d['value']), [round(v) for v in d['window_rates']], 'k_icp', round(d['kernel_ms_per_step']['k_icp']*1e3,1), 'us', d['config']['steps_in_flight'], d['config']['k_icp_slot_share'], 'parity', d['ranks']['per_rank'])"
done
timeout -k 10 60 tools/coopbench 1 0
timeout -k 10 60 tools/coopbench 1 0 1280 960 20
