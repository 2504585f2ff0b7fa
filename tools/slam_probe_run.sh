#!/bin/bash
# The SLAM drop-in's backlogged passes (examples/slam_rate, 20 passes) with the
# event trace, per tracker copy path; the slow submissions and their steps
# (VERDICT r4 item 3).
set -eo pipefail
O=gpurun_out/slamtrace4
mkdir -p $O
echo "host: $(nproc) cpus visible, loadavg $(cat /proc/loadavg)"
cat /sys/fs/cgroup/cpu.max 2>/dev/null || true
grep -E "nr_throttled|throttled_usec" /sys/fs/cgroup/cpu.stat 2>/dev/null || true
for cfg in "sdma" "kernel YOUTH_ICP_TRACK_COPY=kernel" "sdma2" "kernel2 YOUTH_ICP_TRACK_COPY=kernel"; do
  set -- $cfg
  label=$1; shift
  env "$@" YOUTH_SLAM_TRACE=$O/events_$label.txt timeout -k 10 120 slam-rgbd_amd/slam_rate 300 20 \
      > $O/slam_rate_$label.json 2> $O/slam_rate_$label.err
  python3 tools/slam_trace.py $O/events_$label.txt > $O/summary_$label.txt
  echo "== $label: $(python3 -c "import json;d=json.load(open('$O/slam_rate_$label.json'));print(d['value'], [round(v/1e3,1) for v in d['pass_values']], d['pose_checksum'])")"
  grep "slow submit" $O/summary_$label.txt || true
  grep -E "nr_throttled|throttled_usec" /sys/fs/cgroup/cpu.stat 2>/dev/null || true
  echo "loadavg $(cat /proc/loadavg)"
done
