#!/bin/bash
# Round-4 GPU call y: C3 single-pair (1280x960, 20 it) plan sweep: pixels per
# lane 10 (the planner's) .. 16, 512 or 256 threads, product build, two rounds.
set -o pipefail
O=gpurun_out/c3_sweep_r4y.txt
: > $O
for r in 1 2; do
  for cfg in "plan" "px11 YOUTH_ICP_COOP_PX=11" "px12 YOUTH_ICP_COOP_PX=12" "px14 YOUTH_ICP_COOP_PX=14" \
             "px16 YOUTH_ICP_COOP_PX=16" "t256px20 YOUTH_ICP_COOP_THREADS=256 YOUTH_ICP_COOP_PX=20" \
             "t256px24 YOUTH_ICP_COOP_THREADS=256 YOUTH_ICP_COOP_PX=24"; do
    set -- $cfg
    label=$1; shift
    env "$@" timeout -k 10 120 python3 tools/c2_ab.py $label 2>/dev/null | grep 1280x960 >> $O || exit 1
  done
done
echo all done
