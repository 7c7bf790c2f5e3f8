#!/bin/bash
# Profile the bench step on the GPU box: rocprofv3 kernel-trace stats of the bench command, then one rocprofv3 --pmc
# pass per counter group (never combined with tracing), reduced per kernel family / kernel by tools/pmc_families.py.
# usage: bash tools/gpu_profile.sh TAG [extra bench args]   -> gpurun_out/TAG/{stats.md, pmc_<key>.json, ...}
set -u
TAG=${1:-prof}; shift || true
EXTRA="$*"
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
KEY=${PMC_KEY:-base_224_b256_bf16}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python bench.py --steps 10 --warmup 3 --no-cpu-baseline $EXTRA > "$OUT/prof.json" 2> "$OUT/prof.err" || {
  echo "kernel-trace run failed"; exit 1; }
S=$(find "$OUT/prof" -name "*kernel_stats.csv" | head -1)
python tools/prof_summary.py "$S" 13 "rocprofv3 --kernel-trace --stats -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline $EXTRA" > "$OUT/stats.md"
cp "$S" "$OUT/kernel_stats.csv"
# PMC passes under the schedule bench.py's event-bracketed roofline step times (round 6): in order,
# one forward chain and the weight gradients on the compute stream, so per-family counters and the live per-launch
# timings describe the same launches.  PMC_SCHEDULE=default profiles the shipped multi-stream schedule instead.
SCHED=${PMC_SCHEDULE:-inorder}
SARGS=""
[ "$SCHED" = inorder ] && SARGS="--engine fwd_streams=1 --engine concurrent_wgrad=0"
P="python bench.py --steps 2 --warmup 1 --no-roofline --no-cpu-baseline --no-gemm-peak $EXTRA $SARGS"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS" "GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $grp -d "$OUT/pmc$i" -o run --output-format csv -- $P > "$OUT/pmc$i.log" 2>&1 || {
    echo "pmc pass $i failed"; exit 1; }
  echo "pmc pass $i ok"
done
PMC_SCHEDULE_ARGS="$SARGS" python tools/pmc_families.py "$KEY" 3 "$OUT/pmc_$KEY.json" "$OUT/pmc1" "$OUT/pmc2" "$OUT/pmc3" "$OUT/pmc4" > "$OUT/pmc_summary.txt" 2>&1
rm -rf "$OUT/prof" "$OUT"/pmc[1-4]
echo done
