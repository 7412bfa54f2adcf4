#!/bin/bash
# Build an ablation variant of the library pair into tools/_abl/<tag>/:
#   bash tools/abl_build.sh TAG "-DMACRO=VAL ..."
# libimgcomp.so with the macros and its own libimgcomp_torch.so (rpath $ORIGIN, so torch.ops.imgcomp
# calls the variant too).  The GPU side selects it with IMGCOMP_LIB=tools/_abl/TAG/libimgcomp.so
set -e
TAG=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
# SRC_ROOT: a patched copy of the tree's include/ and image_compression_amd/csrc/ (diagnostic variants)
C=${SRC_ROOT:-$R}/image_compression_amd/csrc
B=$R/tools/_abl/build_$TAG
O=$R/tools/_abl/$TAG
mkdir -p $B $O
NOPK_SRCS=${NOPK_SRCS-"igemm wgrad pack conv_api gdn elementwise entropy msssim im2col gdn_fused edge optim metrics"}  # as the Makefile: all (override: NOPK_SRCS=...)
for f in igemm wgrad pack conv_api gdn elementwise entropy msssim im2col gdn_fused edge optim metrics; do
  extra=""
  case " $NOPK_SRCS " in *" $f "*) extra="-Xclang -target-feature -Xclang -packed-fp32-ops";; esac
  [ $f = gdn_fused ] && extra="$extra -mllvm -amdgpu-mfma-vgpr-form $GDN_FLAGS"  # as the Makefile (FLAGS_gdn_fused); GDN_FLAGS: extra flags for this file only
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I$C $extra "$@" -c $C/$f.hip -o $B/$f.o 2>&1 \
    | grep -v "not a recognized feature" &
done
wait
ls $B/*.o | wc -l | grep -qx 13 || { echo "abl_build: an object failed to build"; exit 1; }
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $O/libimgcomp.so $B/*.o
TORCH_DIR=$(python3 -c 'import os, torch; print(os.path.dirname(torch.__file__))')
g++ -shared -o $O/libimgcomp_torch.so $R/image_compression_amd/csrc/build/torch_ops.o -L$O -limgcomp -L$TORCH_DIR/lib -ltorch -ltorch_cpu -lc10 \
  -lc10_hip -ltorch_hip -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,'$ORIGIN' -Wl,-rpath,$TORCH_DIR/lib
rm -rf $B
echo built tools/_abl/$TAG/
