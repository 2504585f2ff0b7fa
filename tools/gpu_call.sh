#!/bin/bash
# One GPU call (run through gpurun from the repo root), replacing the per-round
# one-off scripts: `tools/gpu_call.sh TAG STEP...` runs each STEP in order,
# every GPU step under its own time limit, output to gpurun_out/<step>_TAG.*,
# and stops at the first failure (nothing more runs on the GPU after it).
#   tests        python -m pytest tests -m gpu (one process, per-test timeout)
#   tests:EXPR   the same with -k EXPR
#   smoke        __graft_entry__.smoke()
#   bench        python bench.py (the driver's default line)
#   bench:ARGS   python bench.py ARGS (comma-separated, e.g. bench:--no-legs,--steps,50)
#   profile      tools/profile.sh TAG (kernel trace + PMC passes)
#   py:FILE      python FILE (a probe under tools/)
#   sh:FILE      bash FILE (a multi-step probe under tools/, its own timeouts inside)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
TAG=$1
shift
nb=0
for step in "$@"; do
  name=${step%%:*}
  arg=${step#*:}
  [ "$arg" = "$step" ] && arg=""
  echo "[$(date +%T)] $step"
  case $name in
    tests)
      k=()
      [ -n "$arg" ] && k=(-k "$arg")
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 \
        --timeout-method thread "${k[@]}" > $O/gpu_tests_$TAG.txt 2>&1 || { tail -30 $O/gpu_tests_$TAG.txt; exit 2; } ;;
    smoke)
      timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" \
        > $O/smoke_$TAG.txt 2>&1 || { cat $O/smoke_$TAG.txt; exit 3; } ;;
    bench)
      IFS=, read -r -a ba <<< "$arg"
      nb=$((nb + 1)); bt=$TAG; [ $nb -gt 1 ] && bt=${TAG}_$nb   # one file per bench step
      timeout -k 10 400 python -u bench.py "${ba[@]}" > $O/bench_$bt.json 2> $O/bench_$bt.err \
        || { tail -30 $O/bench_$bt.err; exit 4; } ;;
    profile)
      tools/profile.sh $TAG > $O/profile_$TAG.log 2>&1 || { tail -30 $O/profile_$TAG.log; exit 5; } ;;
    py)
      timeout -k 10 300 python -u $arg > $O/py_$(basename $arg .py)_$TAG.txt 2>&1 \
        || { tail -30 $O/py_$(basename $arg .py)_$TAG.txt; exit 6; } ;;
    sh)
      timeout -k 10 900 bash $arg > $O/sh_$(basename $arg .sh)_$TAG.txt 2>&1 \
        || { tail -30 $O/sh_$(basename $arg .sh)_$TAG.txt; exit 7; } ;;
    *)
      echo "unknown step $step"; exit 9 ;;
  esac
done
echo "[$(date +%T)] all done"
