#!/bin/bash
# Same-box A/B of k_prep's workgroup -> tile order (YOUTH_ICP_PREP_XCD_MAP 0/1/2):
# k_prep time from the bench's HIP events (2 rounds each), then one FETCH_SIZE
# and one WRITE_SIZE rocprofv3 pass per order (k_prep's read over-fetch).
# Usage: tools/prep_map_ab.sh <tag>   (on the GPU box)
set -euo pipefail
OUT=$(pwd)/gpurun_out/prepab_${1:-a}
mkdir -p $OUT
export TMPDIR=/tmp
B="--no-legs --no-cpu-baseline --no-viewer --no-host-io --no-spec-parity --windows 1"
for r in 1 2; do for m in 0 1 2; do
    YOUTH_ICP_PREP_XCD_MAP=$m timeout -k 10 120 python bench.py $B > $OUT/bench_m${m}_$r.json
    python3 -c "import json; d=json.load(open('$OUT/bench_m${m}_$r.json')); print('map $m round $r', round(d['value']), 'k_prep_ms', round(d['roofline_prep']['avg_launch_ms'], 4), 'k_icp_ms', round(d['roofline']['avg_launch_ms'], 4))" >> $OUT/ab.txt
done; done
for m in 0 1 2; do
    export YOUTH_ICP_PREP_XCD_MAP=$m
    timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T --output-format csv -d $OUT/m$m/pmc_fetch -o pmc -- python3 bench.py $B --steps 10 > $OUT/fetch_m$m.log 2>&1
    timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T --output-format csv -d $OUT/m$m/pmc_write -o pmc -- python3 bench.py $B --steps 10 > $OUT/write_m$m.log 2>&1
    python3 tools/pmc_summary.py $OUT/m$m k_prep > $OUT/m$m/pmc_summary.txt
done
unset YOUTH_ICP_PREP_XCD_MAP
echo done
