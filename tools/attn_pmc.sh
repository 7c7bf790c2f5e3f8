#!/bin/bash
# PMC of the attention kernels under tools/attn_bench.py for the shipped library and the given variants.
# usage: bash tools/attn_pmc.sh OUTDIR TAG...   (TAG "base" = the in-tree library)
set -u
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = base ]; then LIB=vision-transformer_amd/VisionTransformer/libvit_hip.so; else LIB=tools/variants/libvit_hip_$v.so; fi
  i=0
  mkdir -p "$OUT/$v"
  for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS" \
             "SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM"; do
    i=$((i+1))
    VIT_HIP_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc $grp -d "$OUT/$v/p$i" -o run --output-format csv -- \
      python tools/attn_bench.py --reps 3 > "$OUT/$v/p$i.log" 2>&1 || { echo "pmc $v pass $i failed"; exit 1; }
  done
  python tools/kernel_pmc.py "attn_bwd_fused|attn_delta|attn_fwd_fused" "$OUT/$v/p1" "$OUT/$v/p2" > "$OUT/pmc_$v.txt"
  rm -rf "$OUT/$v/p1" "$OUT/$v/p2"
done
