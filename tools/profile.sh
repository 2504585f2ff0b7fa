#!/bin/bash
# rocprofv3 passes for the bench workload (run on the GPU box via gpurun).
#   1. --kernel-trace --stats: per-kernel average durations (committed summary)
#   2. PMC passes, one counter group each (FETCH_SIZE and WRITE_SIZE cannot
#      share a pass on gfx950): HBM traffic of k_icp / k_prep; SQ pass: VALU
#      issue (valu_busy_frac) and wave state
#   3. tools/pmc_traffic.py -> $OUT/traffic.json (kernel source sha included)
# Usage: tools/profile.sh <tag> [bench args...]
set -euo pipefail
TAG=${1:-r02}; shift || true
ARGS=${*:---steps 30 --warmup 5 --windows 0 --no-cpu-baseline --no-host-io --no-legs --no-viewer --no-spec-parity}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/kt -o kt \
    -- python3 bench.py $ARGS > $OUT/bench_kt.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T --output-format csv -d $OUT/pmc_fetch -o pmc \
    -- python3 bench.py $ARGS > $OUT/bench_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T --output-format csv -d $OUT/pmc_write -o pmc \
    -- python3 bench.py $ARGS > $OUT/bench_write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-trace -T --output-format csv -d $OUT/pmc_sq -o pmc \
    -- python3 bench.py $ARGS > $OUT/bench_sq.log 2>&1
# instruction mix by type and wave-state cycles (the k_icp cycle account,
# DESIGN.md §5; at most 8 SQ counters per pass)
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace -T --output-format csv -d $OUT/pmc_types -o pmc \
    -- python3 bench.py $ARGS > $OUT/bench_types.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_INT64 SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM GRBM_GUI_ACTIVE --kernel-trace -T --output-format csv -d $OUT/pmc_types2 -o pmc \
    -- python3 bench.py $ARGS > $OUT/bench_types2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-trace -T --output-format csv -d $OUT/pmc_active -o pmc \
    -- python3 bench.py $ARGS > $OUT/bench_active.log 2>&1
python3 tools/pmc_summary.py $OUT > $OUT/pmc_summary.txt
python3 tools/pmc_traffic.py $OUT $OUT/traffic.json ${PAIRS:-512} 640 480 10 > /dev/null
KT=$(find $OUT/kt -name '*kernel_trace.csv' -print -quit)
python3 tools/kt_summary.py $KT 5 > $OUT/kt_summary.txt
cp "$(find $OUT/kt -name '*kernel_stats.csv' -print -quit)" $OUT/kernel_stats.csv
echo done
