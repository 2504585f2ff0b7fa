#!/bin/bash
# Round-4 GPU call (run through gpurun): GPU suite, smoke, default bench, the
# tagged hand-off probe, same-box A/B of kernel variants, coop phase timings.
set -o pipefail
O=gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests_r4a.txt 2>&1 || exit 1
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke_r4a.txt 2>&1 || exit 2
timeout -k 10 300 python -u bench.py > $O/bench_r4a.json 2> $O/bench_r4a.err || exit 3
timeout -k 10 150 tools/tag_probe > $O/tag_probe_r4a.txt 2>&1 || exit 4
EXTRA="--no-legs --no-spec-parity --no-viewer" tools/ab_run.sh 2 ${AB:-occ4 occ5 pipe4 pipe5 pipe6 prep128x24 ko_fma} > $O/ab_r4a.txt 2>&1 || exit 5
timeout -k 10 120 tools/coopbench 1 0 640 480 10 > $O/coopbench_c2_r4a.txt 2>&1 || exit 6
timeout -k 10 120 tools/coopbench 1 0 1280 960 20 > $O/coopbench_c3_r4a.txt 2>&1 || exit 7
echo all done
