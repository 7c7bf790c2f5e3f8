#!/bin/bash
# Build a libvit_hip.so variant with a different vit_gemm.hip source and/or -D flags (A/B runs: tools/gemm_ab.py).
# usage: tools/build_variant.sh TAG GEMM_SOURCE "EXTRA FLAGS"   -> tools/variants/libvit_hip_TAG.so
set -e
TAG=$1; SRC=$2; EXTRA=${3:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/vision-transformer_amd/csrc
make -s -C $C >/dev/null
OBJ=/tmp/vit_gemm_$TAG.o
cp "$SRC" $C/.variant_$TAG.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -mllvm -pragma-unroll-threshold=1000000 \
  -Wno-unused-variable $EXTRA -c $C/.variant_$TAG.hip -o $OBJ
rm -f $C/.variant_$TAG.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/tools/variants/libvit_hip_$TAG.so $OBJ \
  $C/build/vit_attention.o $C/build/vit_norm.o $C/build/vit_misc.o $C/build/vit_image.o
echo built tools/variants/libvit_hip_$TAG.so
