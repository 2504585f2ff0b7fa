#!/bin/bash
# The drop-in path's backlogged passes (examples/slam_rate, plain-C producer)
# under a rocprofv3 kernel + copy trace with the module's event trace on, per
# tracker copy path (SDMA, or k_pull_frames: YOUTH_ICP_TRACK_COPY=kernel);
# tools/slam_trace.py per pass, and the overlap of the copies with k_icp_coop.
set -eo pipefail
export TMPDIR=/tmp
O=gpurun_out/slamtrace5
mkdir -p $O
for cfg in "kernel YOUTH_ICP_TRACK_COPY=kernel" "sdma"; do
  set -- $cfg
  label=$1; shift
  env "$@" YOUTH_SLAM_TRACE=$O/events_$label.txt timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace \
      --output-format csv -d $O/kt_$label -o kt -- slam-rgbd_amd/slam_rate 300 6 > $O/slam_rate_$label.json 2> $O/slam_rate_$label.err
  KT=$(find $O/kt_$label -name '*kernel_trace.csv' -print -quit)
  python3 tools/slam_trace.py $O/events_$label.txt $KT > $O/summary_$label.txt
  echo "== $label"; grep "^pass\|slow submit" $O/summary_$label.txt
  python3 tools/copy_overlap.py $O/kt_$label
done
