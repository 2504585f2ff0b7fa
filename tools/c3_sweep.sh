#!/bin/bash
set -e
for r in 1 2; do
  for tc in ${CHUNKS:-default 1024 1536 3072 4096}; do
    if [ "$tc" = default ]; then timeout -k 10 120 python3 tools/c3_sweep.py
    else YOUTH_ICP_TARGET_CHUNKS=$tc timeout -k 10 120 python3 tools/c3_sweep.py; fi
  done
done
