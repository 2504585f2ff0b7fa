#!/bin/bash
# C2 (one pair per call, k_icp_coop) under rocprofv3 --kernel-trace: kernel
# duration and the idle gap between consecutive aligns (tools/kt_gaps.py).
set -eo pipefail
export TMPDIR=/tmp
O=gpurun_out/c2trace
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- python3 tools/c2_ab.py c2 > $O/c2.txt 2>&1
cat $O/c2.txt | tail -3
KT=$(find $O/kt -name '*kernel_trace.csv' -print -quit)
python3 tools/kt_gaps.py $KT 100
