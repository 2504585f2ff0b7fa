#!/bin/bash
# Round-4 GPU call p (all halo loads in flight before the first use): k_prep with branch-free halo words (buffer loads, edge
# columns one pixel per lane) and buffer-descriptor record stores: the GPU
# tests that cover k_prep / the records on the product build, then the
# interleaved A/B against HEAD's kernel (tools/ab/prepbase).
set -o pipefail
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_spec.py tests/test_gpu_fuzz.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > $O/prep_tests_r4p.txt 2>&1 || exit 1
EXTRA="--no-legs --no-spec-parity --no-viewer" tools/ab_run.sh 3 prepbase prepnew2 > $O/ab_prep_r4p.txt 2>&1 || exit 2
echo all done
