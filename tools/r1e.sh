mkdir -p gpurun_out/r1e
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -m gpu -p no:cacheprovider -k "gemm" -x > gpurun_out/r1e/k.log 2>&1 || { echo "kernel tests failed"; tail -30 gpurun_out/r1e/k.log; exit 1; }
tail -1 gpurun_out/r1e/k.log
timeout -k 10 300 python tools/gemm_bench.py --impls 2,4 --reps 10 > gpurun_out/r1e/base.log 2>&1 || exit 1
SH="fwd qkv,fwd fc2,dgrad fc1,wgrad fc1"
for v in direct noepi; do
VIT_HIP_LIB=$PWD/vision-transformer_amd/csrc/diag/lib_$v.so timeout -k 10 200 python tools/gemm_bench.py --impls 4 --reps 10 --only "$SH" --no-ref > gpurun_out/r1e/$v.log 2>&1 || exit 1
done
grep -h -v amdgpu.ids gpurun_out/r1e/base.log gpurun_out/r1e/direct.log gpurun_out/r1e/noepi.log
