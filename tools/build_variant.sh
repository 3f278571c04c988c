#!/bin/bash
# Build an experiment variant of librgbd_hip.so with extra compiler flags (e.g. -DC4_NODMA=3):
#   [REB=file.hip] tools/build_variant.sh NAME FLAGS...  ->  rgb-d-instance-segmentation_amd/gpurun_ab_NAME.so
# (REB, default ratio.hip, is compiled with FLAGS; the other objects come from the in-tree build;
# objects under /tmp/variant_NAME; the in-tree build is untouched)
set -e
N=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
C="$R/rgb-d-instance-segmentation_amd/csrc"
B=/tmp/variant_$N; mkdir -p $B
cd "$C"
for f in $(sed -n 's/^SRCS = //p' Makefile); do
  o=$B/${f%.hip}.o
  if [ "$f" = "${REB:-ratio.hip}" ] || [ ! -f $B/ok_$f ]; then
    if [ -f build/${f%.hip}.o ] && [ "$f" != "${REB:-ratio.hip}" ]; then cp build/${f%.hip}.o $o; else
      /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -Wno-unused-result "$@" -c $f -o $o; fi
    touch $B/ok_$f
  fi
done
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared $B/*.o -o "$R/rgb-d-instance-segmentation_amd/gpurun_ab_$N.so"
echo built gpurun_ab_$N.so
