#!/bin/bash
# LDS / MFMA counters of the v4 GEMM at 8192^3 in the three operand layouts (kk fwd, kr dgrad, rr weight gradient).
OUT=gpurun_out/${1:-lay}; mkdir -p "$OUT"; export TMPDIR=/tmp
for lay in kk kr rr; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY \
    -d "$OUT/p_$lay" -o run --output-format csv -- python tools/gemm_one.py 8192 8192 8192 0 $lay > "$OUT/$lay.log" 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$OUT/t_$lay" -o run --output-format csv -- python tools/gemm_one.py 8192 8192 8192 0 $lay >> "$OUT/$lay.log" 2>&1 || exit 1
done
for f in $(find "$OUT" -name "*counter_collection.csv"); do echo "== $f"; python - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(float)
for r in rows:
    if "gemm_bf16_v4" in r["Kernel_Name"]:
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(agg.items()): print(f"  {k:28s} {v:16.0f}")
PY
done
for f in $(find "$OUT" -name "*kernel_stats.csv"); do echo "== $f"; grep gemm_bf16 "$f" | cut -c1-200; done
