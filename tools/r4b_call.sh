#!/bin/bash
# Round-4 GPU call b: GPU suite, smoke, default bench, the rocprof profile of
# the product build (kernel trace + PMC passes -> traffic.json), k_prep's PMC
# traffic with 128x24 tiles, and the 64-pair shard (N = 8's per-GPU work).
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests_r4b.txt 2>&1 || exit 1
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke_r4b.txt 2>&1 || exit 2
timeout -k 10 300 python -u bench.py > $O/bench_r4b.json 2> $O/bench_r4b.err || exit 3
tools/profile.sh r04b > $O/profile_r04b.log 2>&1 || exit 4
ARGS="--steps 30 --warmup 5 --windows 0 --no-cpu-baseline --no-host-io --no-legs --no-viewer --no-spec-parity"
for c in FETCH_SIZE WRITE_SIZE; do
  YOUTH_ICP_LIB=tools/ab/prep128x24/libyouth_icp.so timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace -T --output-format csv \
      -d $O/prof_prep128_$c -o pmc -- python3 bench.py $ARGS > $O/prep128_$c.log 2>&1 || exit 5
done
timeout -k 10 300 python -u bench.py --global-pairs 64 --no-legs --no-spec-parity --no-viewer --no-host-io \
    --no-cpu-baseline > $O/bench64_r4b.json 2> $O/bench64_r4b.err || exit 6
echo all done
