#!/bin/bash
# A/B of the 16-B/px target layout (tools/ab/rec16.hip:
# normals 12 B + the target's int16 depth masked by its normal, z recomputed)
# against the product build, C4 headline, interleaved, then the variant's
# parity (64-pair oracle check + 128 pairs at SURVEY 8d noise).
set -eo pipefail
EXTRA="--no-legs --no-viewer --no-spec-parity" tools/ab_run.sh 3 cur rec16
YOUTH_ICP_LIB=tools/ab/rec16/libyouth_icp.so timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 \
    --windows 0 --no-legs --no-viewer --no-spec-parity --no-host-io > gpurun_out/ab/rec16_parity.json
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/ab/rec16_parity.json").read().strip().splitlines()[-1])
print("rec16 parity", d["parity"]["pose_max_abs_err_vs_cpu"], d["parity"]["survey_noise"])
PY
