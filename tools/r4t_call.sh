#!/bin/bash
# Round-4 GPU call t: k_prep LDS row stride 131 with 4-row x 16-word halo
# blocks per wave (conflict-free halo stores): GPU tests on the product build,
# then the interleaved A/B against HEAD's kernel.
set -o pipefail
O=gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_spec.py tests/test_gpu_fuzz.py \
    tests/test_gpu_reduce.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/prep_tests_r4t.txt 2>&1 || exit 1
EXTRA="--no-legs --no-spec-parity --no-viewer" tools/ab_run.sh 3 head=prepnew2 prepls > $O/ab_prep_r4t.txt 2>&1 || exit 2
echo all done
