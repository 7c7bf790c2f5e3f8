# round-2l: v4 staging by global_load_lds (diag/lib_glds.so) vs buffer_load ... lds (default)
mkdir -p gpurun_out/r2l
VIT_HIP_LIB=$PWD/vision-transformer_amd/csrc/diag/lib_glds.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -x -p no:cacheprovider -k "gemm" > gpurun_out/r2l/k.log 2>&1 || { echo "kernel tests failed"; tail -30 gpurun_out/r2l/k.log; exit 1; }
tail -1 gpurun_out/r2l/k.log
timeout -k 10 300 python tools/gemm_bench.py --impls 4 --reps 10 --epi --no-ref > gpurun_out/r2l/buf.log 2>&1 || exit 1
VIT_HIP_LIB=$PWD/vision-transformer_amd/csrc/diag/lib_glds.so timeout -k 10 300 python tools/gemm_bench.py --impls 4 --reps 10 --epi --no-ref > gpurun_out/r2l/glds.log 2>&1 || exit 1
echo "== buffer_load lds"; grep -v amdgpu gpurun_out/r2l/buf.log; echo "== global_load_lds"; grep -v amdgpu gpurun_out/r2l/glds.log
