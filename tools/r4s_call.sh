#!/bin/bash
# Round-4 GPU call s: k_prep records reading their 15 plane values off one base
# register (asm ds_read_b32 with immediate offsets) and the centred-column
# exactness guard of k_icp's aligned loop: GPU tests on the product build, the
# off-centre principal point test on HEAD's build (expected to fail there),
# then the interleaved A/B against HEAD.
set -o pipefail
O=gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_spec.py tests/test_gpu_fuzz.py \
    tests/test_gpu_reduce.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/prep_tests_r4s.txt 2>&1 || exit 1
YOUTH_ICP_LIB=tools/ab/prepnew2/libyouth_icp.so timeout -k 10 120 python -u -m pytest tests/test_gpu_reduce.py -m gpu -q \
    --timeout 60 --timeout-method thread -k off_centre > $O/off_centre_head_r4s.txt 2>&1
echo "head off-centre rc $?" >> $O/off_centre_head_r4s.txt
EXTRA="--no-legs --no-spec-parity --no-viewer" tools/ab_run.sh 3 head=prepnew2 prepasm > $O/ab_prep_r4s.txt 2>&1 || exit 2
echo all done
