#!/bin/bash
# A/B of the designated-summer k_icp (tools/ab/vol) against tools/ab/head:
# C4 (512 pairs), the 64-pair shard, the C3 batch (16 pairs @1280x960, 20 it)
set -o pipefail
X="--no-legs --no-viewer --no-spec-parity"
EXTRA="$X" timeout -k 10 400 tools/ab_run.sh 2 head vol > gpurun_out/ab_vol_c4.txt 2>&1 || exit 1
EXTRA="$X --global-pairs 64" timeout -k 10 300 tools/ab_run.sh 2 head vol > gpurun_out/ab_vol_64.txt 2>&1 || exit 1
EXTRA="$X --global-pairs 16 --width 1280 --height 960 --iters 20" timeout -k 10 300 tools/ab_run.sh 2 head vol > gpurun_out/ab_vol_c3.txt 2>&1 || exit 1
