# round-2q: attention backward A/B: round-start kernel (one item per workgroup, LDS-staged dK/dV) vs persistent
# (direct dK/dV stores) vs persistent with LDS-staged dK/dV; kernel tests on the staged variant
mkdir -p gpurun_out/r2q
D=$PWD/vision-transformer_amd/csrc/diag
VIT_HIP_LIB=$D/lib_a_staged.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "attention" > gpurun_out/r2q/k.log 2>&1 || { tail -30 gpurun_out/r2q/k.log; exit 1; }
tail -1 gpurun_out/r2q/k.log
for rep in 1 2; do
  echo "== old"; VIT_HIP_LIB=$D/lib_a_old.so timeout -k 10 120 python tools/attn_bench.py --reps 20 2>&1 | grep fused || exit 1
  echo "== persistent direct"; timeout -k 10 120 python tools/attn_bench.py --reps 20 2>&1 | grep fused || exit 1
  echo "== persistent staged"; VIT_HIP_LIB=$D/lib_a_staged.so timeout -k 10 120 python tools/attn_bench.py --reps 20 2>&1 | grep fused || exit 1
done
