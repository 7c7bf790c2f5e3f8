#!/bin/bash
# LDS / issue / L2-miss-bytes PMC of the tiled attention kernels (T = 577, config 5's sequence) under tools/attn_bench.py.
set -u
OUT=$1; mkdir -p "$OUT"; export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d "$OUT/p$i" -o run --output-format csv -- \
    python tools/attn_bench.py --reps 3 --T 577 --batch 64 > "$OUT/p$i.log" 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
python tools/kernel_pmc.py "attn_" "$OUT/p1" "$OUT/p2" "$OUT/p3" "$OUT/p4" > "$OUT/pmc.txt"
rm -rf "$OUT/p1" "$OUT/p2" "$OUT/p3" "$OUT/p4"
