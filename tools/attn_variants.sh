#!/bin/bash
# A/B of attention kernel variants (tools/build_variant.sh ... vit_attention): the shipped library, then each variant.
# usage: bash tools/attn_variants.sh OUTDIR TAG...
set -u
OUT=$1; shift
mkdir -p "$OUT"
timeout -k 10 120 python -u tools/attn_bench.py --reps 30 > "$OUT/attn_base.log" 2>&1 || exit $?
for v in "$@"; do
  VIT_HIP_LIB=tools/variants/libvit_hip_$v.so timeout -k 10 120 python -u tools/attn_bench.py --reps 30 > "$OUT/attn_$v.log" 2>&1 || exit $?
done
