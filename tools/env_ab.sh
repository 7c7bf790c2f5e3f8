#!/bin/bash
# Interleaved whole-step A/B of an environment setting: bench.py, 20 steps, no CPU leg / GEMM peak / per-launch events.
# usage: bash tools/env_ab.sh TAG ROUNDS "VAR=VALUE"   (arm A: unset, arm B: set)
TAG=$1; R=$2; KV=$3
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for r in $(seq 1 "$R"); do
  for arm in A B; do
    line=$( if [ $arm = B ]; then export "$KV"; fi
            timeout -k 10 180 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-gemm-peak --no-roofline \
              2>>"$OUT/err.log" ) || exit 1
    echo "$r [$arm] $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a "$OUT/ab.log"
  done
done
