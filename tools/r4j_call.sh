#!/bin/bash
# Round-4 GPU call j: drop-in backlogged rate (slam_rate, C producer) with the
# queue depth / trajectory length read without locks and at most two
# submissions in flight (current build) against the previous slam_api (tools/ab/slamold),
# interleaved; then the SLAM-worker GPU tests on the current build.
set -o pipefail
O=gpurun_out/slam_lockfree_r4j.txt
: > $O
for r in 1 2; do
  echo "variant=old" >> $O
  LD_LIBRARY_PATH=tools/ab/slamold timeout -k 10 120 slam-rgbd_amd/slam_rate 300 9 2>/dev/null >> $O || exit 1
  echo "variant=new" >> $O
  timeout -k 10 120 slam-rgbd_amd/slam_rate 300 9 2>/dev/null >> $O || exit 1
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "slam or worker or algorithm_module or processSlamFrame" > gpurun_out/slam_tests_r4j.txt 2>&1 || exit 2
echo all done
