# round-3a: attn_fwd_mfma (T > 256) at 3 waves/SIMD (launch bound 256,3: 162 VGPRs, no spills) vs 2 (174 VGPR + 48 AGPR)
mkdir -p gpurun_out/r3a
D=$PWD/vision-transformer_amd/csrc/diag
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "attention" > gpurun_out/r3a/k.log 2>&1 || { tail -30 gpurun_out/r3a/k.log; exit 1; }
tail -1 gpurun_out/r3a/k.log
for rep in 1 2; do
  echo "== prev T=577"; VIT_HIP_LIB=$D/lib_a_prev.so timeout -k 10 120 python tools/attn_bench.py --reps 10 --T 577 --batch 64 2>&1 | grep fwd || exit 1
  echo "== fwd 3 waves/SIMD T=577"; timeout -k 10 120 python tools/attn_bench.py --reps 10 --T 577 --batch 64 2>&1 | grep fwd || exit 1
done
