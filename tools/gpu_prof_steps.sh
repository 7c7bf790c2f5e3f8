#!/bin/bash
# rocprofv3 kernel trace of a bench run WITHOUT the GEMM-peak / CPU legs, reduced to the timed steps only
# (tools/prof_steps.py).  usage: bash tools/gpu_prof_steps.sh TAG [extra bench args]  -> gpurun_out/TAG/steps.md
set -u
TAG=${1:-profsteps}; shift || true
EXTRA="$*"
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d "$OUT/trace" -o run --output-format csv -- \
  python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-gemm-peak --no-roofline $EXTRA \
  > "$OUT/prof.json" 2> "$OUT/prof.err" || { echo "kernel-trace run failed"; exit 1; }
T=$(find "$OUT/trace" -name "*kernel_trace.csv" | head -1)
python tools/prof_steps.py "$T" 3 10 "rocprofv3 --kernel-trace -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-gemm-peak --no-roofline $EXTRA" "$OUT/prof.json" > "$OUT/steps.md"
rm -rf "$OUT/trace"
echo done
