# round-2g: v4 LDS ring depth: 10 slots / lead 8 (default) vs 10/7 vs 8/6 (the former layout)
mkdir -p gpurun_out/r2g
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -x -p no:cacheprovider -k "gemm" > gpurun_out/r2g/k.log 2>&1 || { echo "kernel tests failed"; tail -30 gpurun_out/r2g/k.log; exit 1; }
tail -1 gpurun_out/r2g/k.log
timeout -k 10 300 python tools/gemm_bench.py --impls 4 --reps 10 --epi --no-ref > gpurun_out/r2g/s10_l8.log 2>&1 || exit 1
for v in s10_l7 s8_l6; do
VIT_HIP_LIB=$PWD/vision-transformer_amd/csrc/diag/lib_$v.so timeout -k 10 300 python tools/gemm_bench.py --impls 4 --reps 10 --epi --no-ref > gpurun_out/r2g/$v.log 2>&1 || exit 1
done
for v in s10_l8 s10_l7 s8_l6; do echo "== $v"; grep -v amdgpu gpurun_out/r2g/$v.log; done
