#!/bin/bash
# Interleaved A/B of tools/ab/<name>/libyouth_icp.so builds on one box.
# Usage: tools/ab_run.sh <rounds> <name>... ; env EXTRA passes bench flags.
set -euo pipefail
R=$1; shift
mkdir -p gpurun_out/ab
for r in $(seq 1 $R); do
  for n in "$@"; do
    YOUTH_ICP_LIB=tools/ab/$n/libyouth_icp.so timeout -k 10 240 python3 bench.py --steps 30 --warmup 5 \
        --no-cpu-baseline --no-host-io ${EXTRA:-} > gpurun_out/ab/$n.$r.json 2> gpurun_out/ab/$n.$r.err
    python3 - "$n" "$r" <<'PY'
import json,sys
d=json.loads(open(f"gpurun_out/ab/{sys.argv[1]}.{sys.argv[2]}.json").read().strip().splitlines()[-1])
print(f"{sys.argv[1]:>10s} round {sys.argv[2]}: {d['value']:9.0f} aligns/s  kernel {d['roofline']['avg_launch_ms']*1e3:7.1f} us  sched {d.get('sched_last_step')}", flush=True)
PY
  done
done
