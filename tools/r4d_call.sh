#!/bin/bash
# Round-4 GPU call d: the tagged hand-off probe inside k_icp_coop (tools/tagdbg),
# then the product with 128x24 k_prep tiles: GPU suite, smoke, bench, profile.
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 90 tools/tagdbg 2 > $O/tagdbg_r4d.txt 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests_r4d.txt 2>&1 || exit 2
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke_r4d.txt 2>&1 || exit 3
timeout -k 10 300 python -u bench.py > $O/bench_r4d.json 2> $O/bench_r4d.err || exit 4
tools/profile.sh r04d > $O/profile_r04d.log 2>&1 || exit 5
echo all done
