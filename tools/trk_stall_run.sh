#!/bin/bash
set -eo pipefail
for mode in reuse fresh fresh-thread; do
  echo "== $mode"; timeout -k 10 120 python3 tools/trk_stall_probe.py 20 $mode
done
