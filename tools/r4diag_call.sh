#!/bin/bash
# Round-4 GPU call: staggered k_icp item order (YOUTH_ICP_DIAG=D) with fewer
# queues, so a window of pairs' records can stay in the Infinity Cache:
# parity of the persistent path under two settings, then the A/B.
set -o pipefail
O=gpurun_out
YOUTH_ICP_LIB=tools/ab/diag/libyouth_icp.so YOUTH_ICP_DIAG=1 timeout -k 10 300 python -u -m pytest \
    tests/test_gpu_reduce.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "persistent or random_poses or every_kernel_path" > $O/diag_tests_r4.txt 2>&1 || exit 1
YOUTH_ICP_LIB=tools/ab/diag/libyouth_icp.so YOUTH_ICP_DIAG=5 YOUTH_ICP_QUEUES=1 timeout -k 10 300 python -u -m pytest \
    tests/test_gpu_reduce.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "persistent or random_poses or every_kernel_path" >> $O/diag_tests_r4.txt 2>&1 || exit 2
EXTRA="--no-legs --no-spec-parity --no-viewer" tools/ab_run.sh 2 base=cur d0q8=diag \
    d1q8=diag,YOUTH_ICP_DIAG=1 d2q4=diag,YOUTH_ICP_DIAG=2,YOUTH_ICP_QUEUES=4 \
    d3q2=diag,YOUTH_ICP_DIAG=3,YOUTH_ICP_QUEUES=2 d5q1=diag,YOUTH_ICP_DIAG=5,YOUTH_ICP_QUEUES=1 \
    d8q1=diag,YOUTH_ICP_DIAG=8,YOUTH_ICP_QUEUES=1 > $O/ab_diag_r4.txt 2>&1 || exit 3
echo all done
