# round-2u: hardware exp2 (v_exp_f32, no denormal range scaling) in the tiled / fused-forward attention kernels vs previous
mkdir -p gpurun_out/r2u
D=$PWD/vision-transformer_amd/csrc/diag
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "attention" > gpurun_out/r2u/k.log 2>&1 || { tail -30 gpurun_out/r2u/k.log; exit 1; }
tail -1 gpurun_out/r2u/k.log
for rep in 1 2; do
  echo "== prev"; VIT_HIP_LIB=$D/lib_a_prev.so timeout -k 10 120 python tools/attn_bench.py --reps 20 2>&1 | grep -v amdgpu || exit 1
  echo "== hw exp2"; timeout -k 10 120 python tools/attn_bench.py --reps 20 2>&1 | grep -v amdgpu || exit 1
done
