#!/bin/bash
# r29: the T <= 256 fused attention backward vs the tiled dQ + dK/dV kernels (option attn_bwd_split=1, the forward then
# keeps its fp32 O) at C2, whole step, interleaved
OUT=gpurun_out/r29; mkdir -p $OUT
bash tools/bench_ab.sh r29 2 "-" "--opt attn_bwd_split=1" && echo "ab ok" | tee -a $OUT/status.txt
