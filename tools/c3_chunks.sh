#!/bin/bash
# C3 batch (16 pairs @1280x960, 20 iterations): k_icp's chunks per iteration,
# two interleaved rounds (tools/c3_chunks.py, one process per setting).
set -o pipefail
for r in 1 2; do
  for ch in default 1024 1536 3072 4096 6144 8192; do
    if [ $ch = default ]; then
      timeout -k 10 120 python3 tools/c3_chunks.py || exit 1
    else
      YOUTH_ICP_TARGET_CHUNKS=$ch timeout -k 10 120 python3 tools/c3_chunks.py || exit 1
    fi
  done
done
