#!/bin/bash
# Build tools/coopbench on the box (not pushed) and print k_icp_coop's
# per-iteration phases for C2 (640x480, 1 pair) and C3 (1280x960, 20 iters).
set -o pipefail
make -C tools coopbench > /dev/null && timeout -k 10 120 tools/coopbench 1 0 640 480 10 && \
    timeout -k 10 120 tools/coopbench 1 0 1280 960 20
