#!/bin/bash
# Per-kernel A/B of the T = 577 tiled attention kernels (rocprofv3 kernel stats over tools/attn_bench.py) for the
# shipped library and tools/variants/libvit_hip_TAG.so builds.
# usage: bash tools/attn_t577_ab.sh OUTDIR TAG...
set -u
OUT=$1; shift
mkdir -p "$OUT"; export TMPDIR=/tmp
run() {  # tag [lib]
  local tag=$1
  if [ $# -gt 1 ]; then export VIT_HIP_LIB=$2; else unset VIT_HIP_LIB; fi
  timeout -k 10 150 rocprofv3 --kernel-trace --stats -d "$OUT/$tag" -o run --output-format csv -- \
    python tools/attn_bench.py --reps 10 --T 577 --batch 64 > "$OUT/$tag.log" 2>&1 || { echo "$tag failed"; exit 1; }
  local st
  st=$(find "$OUT/$tag" -name "*kernel_stats.csv" | head -1)
  { echo "== $tag"; grep -E "attn_" "$st" | cut -d, -f1-5; } >> "$OUT/summary.txt"
}
run base
for v in "$@"; do run "$v" "tools/variants/libvit_hip_$v.so"; done
