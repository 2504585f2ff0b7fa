#!/bin/bash
# Round-4 GPU call q: k_prep with tpb tiles per workgroup, the next tile's
# depth loads in flight while this tile's records are formed: GPU tests on the
# product build (tpb 2), then the interleaved A/B of tpb 1 / 2 / 4.
set -o pipefail
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_spec.py tests/test_gpu_fuzz.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > $O/prep_tests_r4q.txt 2>&1 || exit 1
EXTRA="--no-legs --no-spec-parity --no-viewer" tools/ab_run.sh 3 tpb1=prepmt,YOUTH_ICP_PREP_TPB=1 \
    tpb2=prepmt,YOUTH_ICP_PREP_TPB=2 tpb4=prepmt,YOUTH_ICP_PREP_TPB=4 > $O/ab_prep_r4q.txt 2>&1 || exit 2
echo all done
