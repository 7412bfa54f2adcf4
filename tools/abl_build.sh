#!/bin/bash
# Build ablation variants of libimgcomp.so into tools/_abl/lib_<tag>.so:
#   bash tools/abl_build.sh TAG "-DMACRO=VAL ..."
# (the GPU side selects one with IMGCOMP_LIB=tools/_abl/lib_TAG.so)
set -e
TAG=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/image_compression_amd/csrc
B=$R/tools/_abl/build_$TAG
mkdir -p $B
for f in igemm wgrad pack conv_api gdn elementwise entropy msssim im2col gdn_fused edge optim metrics; do
  if [ "$f" = "igemm" ] || [ "$f" = "wgrad" ] || [ "$f" = "gdn_fused" ] || [ "$f" = "edge" ] || [ ! -f $B/$f.o ]; then
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I$C "$@" -c $C/$f.hip -o $B/$f.o &
  fi
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/tools/_abl/lib_$TAG.so $B/*.o
echo built tools/_abl/lib_$TAG.so
