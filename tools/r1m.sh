mkdir -p gpurun_out/r1m
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -m gpu -p no:cacheprovider -k "gemm" -x > gpurun_out/r1m/k.log 2>&1 || { echo "kernel tests failed"; tail -30 gpurun_out/r1m/k.log; exit 1; }
tail -1 gpurun_out/r1m/k.log
timeout -k 10 300 python tools/gemm_bench.py --impls 4 --reps 10 > gpurun_out/r1m/gemm.log 2>&1 || exit 1
VIT_GEMM_EPI_GENERAL=1 timeout -k 10 300 python tools/gemm_bench.py --impls 4 --reps 10 --no-ref --only "fwd qkv,fwd fc1" > gpurun_out/r1m/gen.log 2>&1 || exit 1
grep -hv amdgpu gpurun_out/r1m/gemm.log gpurun_out/r1m/gen.log
