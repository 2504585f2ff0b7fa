#!/bin/bash
# Same-box A/B of k_icp's LDS tables (YOUTH_ICP_TAB=0: conversions, 1: tables)
# (YOUTH_ICP_TAB exists only with profiles/r03/k_icp_tables_experiment.patch applied: the tables were dropped, ab_icp_tables.txt)
# on the default bench workload (512 pairs @640x480), interleaved.
# Usage (GPU box): tools/tab_ab.sh <rounds> [extra bench flags]
set -euo pipefail
R=${1:-3}; shift || true
OUT=gpurun_out/tab_ab
mkdir -p $OUT
for r in $(seq 1 $R); do
  for m in 0 1; do
    YOUTH_ICP_TAB=$m timeout -k 10 240 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline \
        --no-host-io --no-legs --no-viewer --no-spec-parity "$@" > $OUT/tab$m.$r.json 2> $OUT/tab$m.$r.err
    python3 - $OUT/tab$m.$r.json "tab=$m" "$r" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]} round {sys.argv[3]}: {d['value']:9.0f} aligns/s  k_icp {d['roofline']['avg_launch_ms']*1e3:7.1f} us"
      f"  k_prep {d['kernel_ms_per_step']['k_prep']*1e3:6.1f} us  err {d.get('parity', {}).get('pose_max_abs_err_vs_cpu', float('nan')):.1e}", flush=True)
PY
  done
done
