#!/bin/bash
# Pose error vs the C oracle (bench pairs and SURVEY §8d noise) for A/B builds
# under tools/ab/<name>/.  usage: tools/prec_par.sh <name>...
set -e
for v in "$@"; do
  YOUTH_ICP_LIB=tools/ab/$v/libyouth_icp.so timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-host-io --no-legs --no-viewer > gpurun_out/par_$v.json 2>/dev/null
  python3 -c "
import json;d=json.loads(open('gpurun_out/par_$v.json').read().strip().splitlines()[-1]);p=d['parity'];print('$v', round(d['value']), 'err', p['pose_max_abs_err_vs_cpu'], 'survey', p['survey_noise']['pose_max_abs_err_vs_cpu'])"
done
