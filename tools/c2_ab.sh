#!/bin/bash
# Interleaved C2 / C3-single-pair A/B (tools/c2_ab.py) on one box.
# Usage: tools/c2_ab.sh <rounds> <spec>... ; a spec is <lib> or
# <label>=<lib>[,VAR=value...]; <lib> "cur" is the in-tree build, anything
# else tools/ab/<lib>/libyouth_icp.so (tools/ab_build.sh)
set -o pipefail
R=$1; shift
for r in $(seq 1 $R); do
  for spec in "$@"; do
    label=${spec%%=*}; rest=${spec#*=}
    [ "$label" = "$spec" ] && rest=$spec
    IFS=, read -r lib envs <<< "$rest"
    envargs=()
    if [ -n "${envs:-}" ]; then IFS=, read -ra envargs <<< "$envs"; fi
    [ "$lib" != cur ] && envargs+=("YOUTH_ICP_LIB=tools/ab/$lib/libyouth_icp.so")
    env "${envargs[@]}" timeout -k 10 150 python3 -u tools/c2_ab.py "$label" || exit 1
  done
done
