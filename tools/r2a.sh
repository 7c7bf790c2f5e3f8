mkdir -p gpurun_out/r2a
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -m gpu -p no:cacheprovider -k "gemm" -x > gpurun_out/r2a/k.log 2>&1 || { echo "kernel tests failed"; tail -30 gpurun_out/r2a/k.log; exit 1; }
tail -1 gpurun_out/r2a/k.log
SH="fwd qkv,fwd proj,fwd fc1,fwd fc2,dgrad fc2"
timeout -k 10 200 python tools/gemm_bench.py --impls 4 --reps 10 --epi --only "$SH" > gpurun_out/r2a/new.log 2>&1 || exit 1
VIT_HIP_LIB=$PWD/vision-transformer_amd/csrc/diag/lib_old.so timeout -k 10 200 python tools/gemm_bench.py --impls 4 --reps 10 --epi --no-ref --only "$SH" > gpurun_out/r2a/old.log 2>&1 || exit 1
grep -hv amdgpu gpurun_out/r2a/new.log gpurun_out/r2a/old.log
