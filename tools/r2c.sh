# round-2c: GEMM v4 read rebalance (A_0 of the next k-tile in phase r=3) vs the previous build (diag/lib_base.so)
mkdir -p gpurun_out/r2c
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -x -p no:cacheprovider -k "gemm" > gpurun_out/r2c/k.log 2>&1 || { echo "kernel tests failed"; tail -30 gpurun_out/r2c/k.log; exit 1; }
tail -1 gpurun_out/r2c/k.log
timeout -k 10 300 python tools/gemm_bench.py --impls 4 --reps 10 --epi > gpurun_out/r2c/new.log 2>&1 || exit 1
VIT_HIP_LIB=$PWD/vision-transformer_amd/csrc/diag/lib_base.so timeout -k 10 300 python tools/gemm_bench.py --impls 4 --reps 10 --epi --no-ref > gpurun_out/r2c/base.log 2>&1 || exit 1
grep -hv amdgpu gpurun_out/r2c/new.log gpurun_out/r2c/base.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r2c/bench.json 2> gpurun_out/r2c/bench.err || { tail -20 gpurun_out/r2c/bench.err; exit 1; }
cut -c1-300 gpurun_out/r2c/bench.json
