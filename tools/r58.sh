#!/bin/bash
# r58: the two-chain forward's ring-attention grid (default 3/4 of the CUs = 192) re-swept after the Q double buffer
OUT=gpurun_out/r58; mkdir -p $OUT
bash tools/bench_ab.sh r58 2 "-" "--opt attn_fwd_grid=224" "--opt attn_fwd_grid=160" "--opt attn_fwd_grid=256" && echo "ab ok" | tee -a $OUT/status.txt
