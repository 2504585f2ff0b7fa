#!/bin/bash
# Round-4 GPU call h: the drop-in's backlogged rate from a C producer, frame
# copy into the page-locked queue by memcpy vs streaming stores, interleaved;
# push_us_per_frame is the producer's time inside processSlamFrame.
set -o pipefail
O=gpurun_out/slam_copy_r4h.txt
: > $O
for r in 1 2; do
  for m in memcpy stream; do
    echo "copy=$m" >> $O
    YOUTH_SLAM_COPY=$m timeout -k 10 120 slam-rgbd_amd/slam_rate 300 9 >> $O 2>&1 || exit 1
  done
done
echo all done
