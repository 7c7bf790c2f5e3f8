#!/bin/bash
# Build a libvit_hip.so variant with a different source for one module and/or -D flags (A/B runs: tools/gemm_ab.py,
# or any tool under VIT_HIP_LIB=tools/variants/libvit_hip_TAG.so).
# usage: tools/build_variant.sh TAG SOURCE "EXTRA FLAGS" [MODULE=vit_gemm]   -> tools/variants/libvit_hip_TAG.so
set -e
TAG=$1; SRC=$2; EXTRA=${3:-}; MOD=${4:-vit_gemm}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/vision-transformer_amd/csrc
make -s -C $C >/dev/null
mkdir -p $ROOT/tools/variants
OBJ=/tmp/${MOD}_$TAG.o
cp "$SRC" $C/.variant_$TAG.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -mllvm -pragma-unroll-threshold=1000000 \
  -Wno-unused-variable $EXTRA -c $C/.variant_$TAG.hip -o $OBJ
rm -f $C/.variant_$TAG.hip
OBJS=""
for m in vit_gemm vit_attention vit_norm vit_misc vit_image; do
  if [ "$m" = "$MOD" ]; then OBJS="$OBJS $OBJ"; else OBJS="$OBJS $C/build/$m.o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/tools/variants/libvit_hip_$TAG.so $OBJS
echo built tools/variants/libvit_hip_$TAG.so
