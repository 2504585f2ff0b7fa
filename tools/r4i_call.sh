#!/bin/bash
# Round-4 GPU call i: drop-in backlogged rate (slam_rate, C producer) with the
# queue depth / trajectory length read without locks (current build, streamed
# or memcpy frame copy) against the previous slam_api (tools/ab/slamold),
# interleaved; then the SLAM-worker GPU tests on the current build.
set -o pipefail
O=gpurun_out/slam_lockfree_r4i.txt
: > $O
for r in 1 2; do
  echo "variant=old" >> $O
  LD_LIBRARY_PATH=tools/ab/slamold timeout -k 10 120 slam-rgbd_amd/slam_rate 300 9 2>/dev/null >> $O || exit 1
  echo "variant=new_stream" >> $O
  timeout -k 10 120 slam-rgbd_amd/slam_rate 300 9 2>/dev/null >> $O || exit 1
  echo "variant=new_memcpy" >> $O
  YOUTH_SLAM_COPY=memcpy timeout -k 10 120 slam-rgbd_amd/slam_rate 300 9 2>/dev/null >> $O || exit 1
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "slam or worker or algorithm_module or processSlamFrame" > gpurun_out/slam_tests_r4i.txt 2>&1 || exit 2
echo all done
