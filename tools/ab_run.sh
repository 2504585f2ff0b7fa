#!/bin/bash
# Interleaved A/B of tools/ab/<lib>/libyouth_icp.so builds on one box.
# Usage: tools/ab_run.sh <rounds> <spec>... ; a spec is <lib> or
# <label>=<lib>[,VAR=value...] (environment for that run only, e.g.
# nofuse=cur,YOUTH_ICP_FUSED_PREP=0).  env EXTRA passes bench flags.
set -euo pipefail
R=$1; shift
mkdir -p gpurun_out/ab
for r in $(seq 1 $R); do
  for spec in "$@"; do
    label=${spec%%=*}; rest=${spec#*=}
    [ "$label" = "$spec" ] && rest=$spec
    IFS=, read -r lib envs <<< "$rest"
    envargs=()
    if [ -n "${envs:-}" ]; then IFS=, read -ra envargs <<< "$envs"; fi
    env "${envargs[@]}" YOUTH_ICP_LIB=tools/ab/$lib/libyouth_icp.so timeout -k 10 240 python3 bench.py \
        --steps 30 --warmup 5 --no-cpu-baseline --no-host-io ${EXTRA:-} \
        > gpurun_out/ab/$label.$r.json 2> gpurun_out/ab/$label.$r.err
    python3 - "$label" "$r" <<'PY'
import json,sys
d=json.loads(open(f"gpurun_out/ab/{sys.argv[1]}.{sys.argv[2]}.json").read().strip().splitlines()[-1])
print(f"{sys.argv[1]:>10s} round {sys.argv[2]}: {d['value']:9.0f} aligns/s  kernel {d['roofline']['avg_launch_ms']*1e3:7.1f} us  prep {d['kernel_ms_per_step']['k_prep']*1e3:6.1f} us  err {d.get('parity',{}).get('pose_max_abs_err_vs_cpu',float('nan')):.1e}  sched {d.get('sched_last_step')}" + (f"  viewer {d['viewer_cloud']['us_per_call']:.1f} us" if 'viewer_cloud' in d else ""), flush=True)
PY
  done
done
