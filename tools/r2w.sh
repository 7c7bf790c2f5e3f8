# round-2w: persistent fused attention backward with the row constants as initial S / dP accumulators (kbias folded into the exp2 FMA)
mkdir -p gpurun_out/r2w
D=$PWD/vision-transformer_amd/csrc/diag
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "attention" > gpurun_out/r2w/k.log 2>&1 || { tail -30 gpurun_out/r2w/k.log; exit 1; }
tail -1 gpurun_out/r2w/k.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -q -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread -k "long_sequence or full_size_configs" > gpurun_out/r2w/m.log 2>&1 || { tail -30 gpurun_out/r2w/m.log; exit 1; }
tail -1 gpurun_out/r2w/m.log
for rep in 1 2; do
  echo "== prev T=197"; VIT_HIP_LIB=$D/lib_a_prev.so timeout -k 10 120 python tools/attn_bench.py --reps 10 --T 197 --batch 256 2>&1 | grep -v amdgpu || exit 1
  echo "== row-constant init T=197"; timeout -k 10 120 python tools/attn_bench.py --reps 10 --T 197 --batch 256 2>&1 | grep -v amdgpu || exit 1
done
