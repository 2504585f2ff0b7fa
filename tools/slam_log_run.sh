#!/bin/bash
# slam_rate with the HIP runtime's own log (AMD_LOG_LEVEL=4, timestamps) and
# the module's event trace: what the runtime does inside a slow submission.
set -eo pipefail
O=gpurun_out/slamlog
mkdir -p $O
for r in 1 2 3; do
  AMD_LOG_LEVEL=4 YOUTH_SLAM_TRACE=$O/events_$r.txt timeout -k 10 120 slam-rgbd_amd/slam_rate 300 4 \
      > $O/slam_rate_$r.json 2> $O/hiplog_$r.txt
  python3 tools/slam_trace.py $O/events_$r.txt > $O/summary_$r.txt
  grep "slow submit\|^pass" $O/summary_$r.txt || true
  if grep -q "slow submit" $O/summary_$r.txt; then break; fi
done
ls -la $O
