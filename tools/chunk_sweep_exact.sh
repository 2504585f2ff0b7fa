#!/bin/bash
# k_icp's work-item size in the exact reduction: YOUTH_ICP_TARGET_CHUNKS
# (chunks per iteration of the launch) on the 512-pair headline, interleaved.
set -eo pipefail
for r in 1 2; do
  for ch in 2048 3072 4096 6144 1536; do
    YOUTH_ICP_TARGET_CHUNKS=$ch timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --windows 1 --no-legs \
        --no-viewer --no-spec-parity --no-host-io --no-cpu-baseline > gpurun_out/cs.json
    python3 -c "
import json; d=json.loads(open('gpurun_out/cs.json').read().strip().splitlines()[-1])
print('round $r chunks $ch:', round(d['value']), round(d['kernel_ms_per_step']['k_icp']*1e3,1), 'us', d['sched_last_step'])"
  done
done
