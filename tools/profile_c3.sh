#!/bin/bash
# rocprofv3 passes of the C3 workload (1280x960, 20 iterations; tools/c3_probe.py):
# kernel trace + FETCH_SIZE / WRITE_SIZE / SQ passes, summarised per kernel.
# Usage: tools/profile_c3.sh <tag>   (on the GPU box via gpurun)
set -euo pipefail
TAG=${1:-c3}
OUT=$(pwd)/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/kt -o kt \
    -- python3 tools/c3_probe.py 30 > $OUT/probe_kt.log 2>&1
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T --output-format csv -d $OUT/pmc_fetch -o pmc \
    -- python3 tools/c3_probe.py 10 > $OUT/probe_fetch.log 2>&1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T --output-format csv -d $OUT/pmc_write -o pmc \
    -- python3 tools/c3_probe.py 10 > $OUT/probe_write.log 2>&1
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-trace -T --output-format csv -d $OUT/pmc_sq -o pmc \
    -- python3 tools/c3_probe.py 10 > $OUT/probe_sq.log 2>&1
python3 tools/pmc_summary.py $OUT > $OUT/pmc_summary.txt
KT=$(find $OUT/kt -name '*kernel_trace.csv' -print -quit)
python3 tools/kt_summary.py $KT 3 > $OUT/kt_summary.txt
echo done
