#!/bin/bash
# Build libyouth_icp.so from a git revision of csrc/icp_kernels.hip into
# tools/ab/<name>/ so two kernel versions can be timed in ONE gpurun call
# (devices differ by several % on this VALU-bound kernel; never compare
# across boxes).  Usage: tools/ab_build.sh <name> <git-rev | file.hip>
# (env HIPFLAGS_EXTRA: extra hipcc flags for the kernel TU; product flags are the Makefile's)
set -euo pipefail
NAME=$1; SRC=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/tools/ab/$NAME
mkdir -p $OUT
mkdir -p $OUT/include
if [ -f "$SRC" ]; then cp "$SRC" $OUT/icp_kernels.hip; cp $ROOT/include/youth_icp.h $OUT/include/
else git -C $ROOT show "$SRC:slam-rgbd_amd/csrc/icp_kernels.hip" > $OUT/icp_kernels.hip
     git -C $ROOT show "$SRC:include/youth_icp.h" > $OUT/include/youth_icp.h; fi
cd $ROOT/slam-rgbd_amd
make -s build/slam_api.o build/algorithm_module.o build/wire.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize \
    ${HIPFLAGS_EXTRA:-} -I$OUT/include -I../include -Icsrc -c $OUT/icp_kernels.hip -o $OUT/icp_kernels.o
# the viewer kernels: the tree's, or env VIEWER_SRC (a viewer_cloud.hip variant)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize \
    -I../include -Icsrc -c ${VIEWER_SRC:-csrc/viewer_cloud.hip} -o $OUT/viewer_cloud.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libyouth_icp.so $OUT/icp_kernels.o \
    $OUT/viewer_cloud.o build/slam_api.o build/algorithm_module.o build/wire.o -lpthread -lrt -Wl,-rpath,/opt/rocm/lib -Wl,--no-undefined
echo "$OUT/libyouth_icp.so"
