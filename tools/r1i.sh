mkdir -p gpurun_out/r1i
for v in NOSTAGE NOPAIR NODQ STAGEONLY; do
  echo "== $v"; VIT_HIP_LIB=$PWD/vision-transformer_amd/csrc/diag/lib_a_$v.so timeout -k 10 120 python tools/attn_bench.py --reps 10 2>&1 | grep fused || exit 1
done
