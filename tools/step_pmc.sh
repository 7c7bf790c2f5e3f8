#!/bin/bash
# One rocprofv3 --pmc pass over a short bench run; per-kernel averages of the counters (tools/kernel_pmc.py).
# usage: bash tools/step_pmc.sh OUTDIR "COUNTERS" [extra bench args]
set -u
OUT=$1; CNT=$2; shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc $CNT -d "$OUT/p" -o run --output-format csv -- \
  python bench.py --steps 2 --warmup 1 --no-roofline --no-cpu-baseline --no-gemm-peak "$@" > "$OUT/pmc.log" 2>&1 || exit 1
python tools/kernel_pmc.py "." "$OUT/p" > "$OUT/pmc.txt"
rm -rf "$OUT/p"
