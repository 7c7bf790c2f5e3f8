#!/bin/bash
# Interleaved whole-step A/B of runtime switches: usage bash tools/bench_ab.sh TAG ROUNDS "ARGS_A" "ARGS_B" ...
# (extra bench.py arguments, e.g. "--engine row0_attention=0" or "--opt attn_fwd_ring=0"; "-" = none).  Each run: bench.py, 20 steps, no CPU leg / GEMM peak / per-launch events.
TAG=$1; R=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for r in $(seq 1 "$R"); do
  for v in "$@"; do
    e=$v; [ "$e" = "-" ] && e=""
    line=$(timeout -k 10 180 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-gemm-peak --no-roofline $e \
           2>>"$OUT/err.log") || exit 1
    echo "$r [$v] $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a "$OUT/ab.log"
  done
done
