#!/bin/bash
# Round-4 GPU call g: the tagged hand-off with opaque re-read offsets (tools/ab/tagfix)
# against the product (tools/ab/base): parity tests of the coop paths on the
# variant, then the C2 / C3 single-pair rates, interleaved.
set -o pipefail
O=gpurun_out
YOUTH_ICP_LIB=tools/ab/tagfix/libyouth_icp.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py \
    tests/test_gpu_reduce.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "coop or single_pair or kernel_paths or track_frame or micro_batches or every_kernel_path or tracker" \
    > $O/tagfix_tests_r4g.txt 2>&1 || exit 1
for r in 1 2 3; do
  for v in base tagfix; do
    YOUTH_ICP_LIB=tools/ab/$v/libyouth_icp.so timeout -k 10 200 python3 tools/c2_ab.py $v >> $O/c2_ab_r4g.txt 2>&1 || exit 2
  done
done
echo all done
