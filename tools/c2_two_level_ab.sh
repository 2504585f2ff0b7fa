#!/bin/bash
# k_icp_coop's two-level partial-row hand-off (YOUTH_ICP_COOP_TWO_LEVEL=1):
# its coop / tracker GPU tests, then an interleaved C2 / C3-single-pair A/B
# against the one-level pass with level-1 / level-2 poll delays, then the
# per-iteration phases of both (tools/coopbench).  Every step under its own
# time limit; stops at the first failure.
set -o pipefail
O=gpurun_out
mkdir -p $O
TAG=${1:-tl}
YOUTH_ICP_COOP_TWO_LEVEL=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 \
  --timeout-method thread -k "coop or track or recovery or slam or single_pair" > $O/tl_tests_$TAG.txt 2>&1 \
  || { tail -30 $O/tl_tests_$TAG.txt; exit 1; }
tail -2 $O/tl_tests_$TAG.txt
bash tools/c2_ab.sh 2 one=cur,YOUTH_ICP_COOP_TWO_LEVEL=0 \
  two_4_8=cur,YOUTH_ICP_COOP_TWO_LEVEL=1 \
  two_0_0=cur,YOUTH_ICP_COOP_TWO_LEVEL=1,YOUTH_ICP_COOP_POLL_DELAY=0,YOUTH_ICP_COOP_POLL_DELAY2=0 \
  two_8_16=cur,YOUTH_ICP_COOP_TWO_LEVEL=1,YOUTH_ICP_COOP_POLL_DELAY=8,YOUTH_ICP_COOP_POLL_DELAY2=16 \
  two_2_24=cur,YOUTH_ICP_COOP_TWO_LEVEL=1,YOUTH_ICP_COOP_POLL_DELAY=2,YOUTH_ICP_COOP_POLL_DELAY2=24 \
  > $O/tl_ab_$TAG.txt 2>&1 || { tail -20 $O/tl_ab_$TAG.txt; exit 2; }
cat $O/tl_ab_$TAG.txt
make -C tools coopbench > /dev/null || exit 3
for tl in 0 1; do
  YOUTH_ICP_COOP_TWO_LEVEL=$tl timeout -k 10 120 tools/coopbench 1 0 640 480 10 > $O/tl_phases_${tl}_$TAG.txt 2>&1 \
    || { cat $O/tl_phases_${tl}_$TAG.txt; exit 4; }
  cat $O/tl_phases_${tl}_$TAG.txt
done
