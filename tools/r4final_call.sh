#!/bin/bash
# Round-4 GPU call f2 (final): the product as committed: GPU suite, smoke, bench,
# rocprof kernel trace + PMC passes.
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests_r4f2.txt 2>&1 || exit 2
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke_r4f2.txt 2>&1 || exit 3
timeout -k 10 300 python -u bench.py > $O/bench_r4f2.json 2> $O/bench_r4f2.err || exit 4
tools/profile.sh r04f > $O/profile_r04f.log 2>&1 || exit 5
echo all done
