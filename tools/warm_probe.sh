#!/bin/bash
# First-window vs later-window rate at small shards: is the gap warm-up
# (clock ramp) or the HIP events of the first window?  Run on the GPU box.
set -euo pipefail
mkdir -p gpurun_out/warm
for gp in 64 128; do
  for w in ${WARMS:-5 50 400}; do
    timeout -k 10 120 python3 bench.py --global-pairs $gp --steps 20 --warmup $w --no-cpu-baseline \
        --no-host-io --no-legs --no-viewer > gpurun_out/warm/g${gp}_w$w.json 2> gpurun_out/warm/g${gp}_w$w.err
    python3 - gpurun_out/warm/g${gp}_w$w.json $gp $w <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"pairs {sys.argv[2]:>4} warmup {sys.argv[3]:>4}: value {d['value']:8.0f}  windows "
      + " ".join(f"{v:8.0f}" for v in d['window_rates'])
      + f"  k_icp {d['roofline']['avg_launch_ms']*1e3:7.1f} us  ms/step {d['ms_per_step']:.3f}", flush=True)
PY
  done
done
