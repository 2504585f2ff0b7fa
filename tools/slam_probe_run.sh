#!/bin/bash
# The SLAM drop-in's backlogged passes (examples/slam_rate, 20 passes) with
# the defaults (pull, LDS reservation, 32 free CUs, auto workgroups) against
# SDMA, twice each.
set -eo pipefail
O=gpurun_out/slamtrace11
mkdir -p $O
echo "host: $(nproc) cpus visible, loadavg $(cat /proc/loadavg)"
for cfg in "pull" "sdma YOUTH_ICP_TRACK_COPY=sdma" "pull_b" "sdma_b YOUTH_ICP_TRACK_COPY=sdma" "pull_w4 YOUTH_ICP_PULL_WG=4"; do
  set -- $cfg
  label=$1; shift
  env "$@" YOUTH_SLAM_TRACE=$O/events_$label.txt timeout -k 10 120 slam-rgbd_amd/slam_rate 300 20 \
      > $O/slam_rate_$label.json 2> $O/slam_rate_$label.err
  python3 tools/slam_trace.py $O/events_$label.txt > $O/summary_$label.txt
  echo "== $label: $(python3 -c "import json;d=json.load(open('$O/slam_rate_$label.json'));print(d['value'], [round(v/1e3,1) for v in d['pass_values']], 'live', d['live_latency_us_median'])")"
  grep "slow submit" $O/summary_$label.txt || true
done
