#!/bin/bash
# Build tools/tagdbg (see tools/tagdbg.cpp): the product kernel source with the
# parked tagged-partials patch and timeout records, for a one-GPU probe.
set -euo pipefail
cd "$(dirname "$0")"
cp ../slam-rgbd_amd/csrc/icp_kernels.hip /tmp/tagk.hip
sed 's|^--- a/slam-rgbd_amd/csrc/icp_kernels.hip|--- tagk.hip|; s|^+++ b/slam-rgbd_amd/csrc/icp_kernels.hip|+++ tagk.hip|' \
    ../profiles/r03/k_icp_coop_tagged_partials_experiment.patch | (cd /tmp && patch -s -p0 tagk.hip)
for aux in 16 17; do
  python3 make_tagdbg_instrument.py /tmp/tagk.hip tagdbg_kernel.hip $aux
  /opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -Wno-unused-result \
      -I../include -I../slam-rgbd_amd/csrc tagdbg.cpp -o tagdbg$aux -L../slam-rgbd_amd -lyouth_synth \
      -Wl,-rpath,'$ORIGIN/../slam-rgbd_amd'
done
