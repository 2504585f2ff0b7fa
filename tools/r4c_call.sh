#!/bin/bash
# Round-4 GPU call c: k_icp at five waves per SIMD with more work chunks per
# iteration (the persistent queue's pose waits), k_prep tile shapes with their
# PMC traffic.  Same box, interleaved rounds.
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
EXTRA="--no-legs --no-spec-parity --no-viewer" tools/ab_run.sh 2 base occ5 occ5c4k=occ5,YOUTH_ICP_TARGET_CHUNKS=4096 \
    occ5c5k=occ5,YOUTH_ICP_TARGET_CHUNKS=5120 basec4k=base,YOUTH_ICP_TARGET_CHUNKS=4096 \
    prep128x24 prep128x16 prep256x12 > $O/ab_r4c.txt 2>&1 || exit 1
ARGS="--steps 30 --warmup 5 --windows 0 --no-cpu-baseline --no-host-io --no-legs --no-viewer --no-spec-parity"
for v in prep128x16 prep256x12; do
  for c in FETCH_SIZE WRITE_SIZE; do
    YOUTH_ICP_LIB=tools/ab/$v/libyouth_icp.so timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace -T --output-format csv \
        -d $O/prof_${v}_$c -o pmc -- python3 bench.py $ARGS > $O/${v}_$c.log 2>&1 || exit 2
  done
done
echo all done
