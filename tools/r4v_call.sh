#!/bin/bash
# Round-4 GPU call v: the product after the k_prep halo loads (branch-free, all in
# flight) and the centred-column guard: GPU suite, smoke, bench, profile.
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests_r4v.txt 2>&1 || exit 2
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke_r4v.txt 2>&1 || exit 3
timeout -k 10 300 python -u bench.py > $O/bench_r4v.json 2> $O/bench_r4v.err || exit 4
tools/profile.sh r04v > $O/profile_r04v.log 2>&1 || exit 5
echo all done
