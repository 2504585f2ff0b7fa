#!/bin/bash
# Round-4 GPU call: k_prep tile order (YOUTH_ICP_PREP_XCD_MAP 0 / 1 / 2) on the
# current kernel, interleaved, three rounds.
set -o pipefail
EXTRA="--no-legs --no-spec-parity --no-viewer" tools/ab_run.sh 3 map0=cur map1=cur,YOUTH_ICP_PREP_XCD_MAP=1 \
    map2=cur,YOUTH_ICP_PREP_XCD_MAP=2 > gpurun_out/ab_prepmap_r4.txt 2>&1 || exit 1
echo all done
