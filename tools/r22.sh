#!/bin/bash
# r22: A/B of the deferred .grad attach (engine.defer_grad_attach) — whole-step interleaved
OUT=gpurun_out/r22; mkdir -p $OUT
bash tools/bench_ab.sh r22 4 "-" "--engine defer_grad_attach=0" && echo "ab ok" | tee -a $OUT/status.txt
