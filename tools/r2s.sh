# round-2s: persistent attention backward with V staged in LDS (VLDS) vs the committed persistent kernel (V from global per item)
mkdir -p gpurun_out/r2s
D=$PWD/vision-transformer_amd/csrc/diag
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "attention" > gpurun_out/r2s/k.log 2>&1 || { tail -30 gpurun_out/r2s/k.log; exit 1; }
tail -1 gpurun_out/r2s/k.log
for rep in 1 2; do
  echo "== prev (V from global)"; VIT_HIP_LIB=$D/lib_a_prev.so timeout -k 10 120 python tools/attn_bench.py --reps 20 2>&1 | grep fused || exit 1
  echo "== VLDS"; timeout -k 10 120 python tools/attn_bench.py --reps 20 2>&1 | grep fused || exit 1
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-gemm-peak > gpurun_out/r2s/bench.json 2> gpurun_out/r2s/bench.err || exit 1
cat gpurun_out/r2s/bench.json
