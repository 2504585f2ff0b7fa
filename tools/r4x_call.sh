#!/bin/bash
# Round-4 GPU call x: C2 / C3 single-pair plan sweep after lane32 (pixels per
# lane, 512 or 256 threads per workgroup), product build, two rounds.
set -o pipefail
O=gpurun_out/c2_sweep_r4x.txt
: > $O
for r in 1 2; do
  for cfg in "plan" "px2 YOUTH_ICP_COOP_PX=2" "px4 YOUTH_ICP_COOP_PX=4" "px5 YOUTH_ICP_COOP_PX=5" \
             "t256 YOUTH_ICP_COOP_THREADS=256" "t256px5 YOUTH_ICP_COOP_THREADS=256 YOUTH_ICP_COOP_PX=5" \
             "t256px6 YOUTH_ICP_COOP_THREADS=256 YOUTH_ICP_COOP_PX=6"; do
    set -- $cfg
    label=$1; shift
    env "$@" timeout -k 10 120 python3 tools/c2_ab.py $label 2>/dev/null | grep -v amdgpu.ids >> $O || exit 1
  done
done
echo all done
