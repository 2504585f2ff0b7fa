#!/bin/bash
set -eo pipefail
echo "== 2000 iterations, 5 ms pause every 40"; timeout -k 10 60 tools/sdma_probe 2000 40 5
echo "== 2000 iterations, no pause"; timeout -k 10 60 tools/sdma_probe 2000 0 0
echo "== 600 iterations, 50 ms pause every 40"; timeout -k 10 60 tools/sdma_probe 600 40 50
