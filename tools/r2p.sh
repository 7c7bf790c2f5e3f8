# round-2p: persistent attention backward ablations (skip the pair phase / the dQ phase)
mkdir -p gpurun_out/r2p
timeout -k 10 120 python tools/attn_bench.py --reps 10 2>&1 | grep fused || exit 1
for v in NOPAIR NODQ; do
  echo "== $v"; VIT_HIP_LIB=$PWD/vision-transformer_amd/csrc/diag/lib_a_$v.so timeout -k 10 120 python tools/attn_bench.py --reps 10 2>&1 | grep fused || exit 1
done
