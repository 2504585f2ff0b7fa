#!/bin/bash
# k_icp_coop's first-pass delay (YOUTH_ICP_COOP_POLL_DELAY, x 64 clocks):
# C2 / C3 single pair (tools/c2_ab.py) and the SLAM drop-in's backlogged
# tracker (slam_rate) per delay, interleaved, on one box.
# Usage: tools/poll_delay_sweep.sh <rounds> <delay>...
set -o pipefail
R=$1; shift
for r in $(seq 1 $R); do
  for d in "$@"; do
    YOUTH_ICP_COOP_POLL_DELAY=$d timeout -k 10 150 python3 -u tools/c2_ab.py d$d || exit 1
    YOUTH_ICP_COOP_POLL_DELAY=$d timeout -k 10 120 slam-rgbd_amd/slam_rate 600 5 > /tmp/sr.json || exit 1
    python3 -c "import json;d=json.load(open('/tmp/sr.json'));print('   d$d slam_rate', d['value'], d['pass_values'], 'live us', d['live_latency_us_median'], d['live_latency_us_p90'], 'chk', d['pose_checksum'])"
  done
done
