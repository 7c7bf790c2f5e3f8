mkdir -p gpurun_out/r1l
SH="fwd qkv,fwd fc1,dgrad fc2"
timeout -k 10 200 python tools/gemm_bench.py --impls 4 --reps 10 --only "$SH" --no-ref > gpurun_out/r1l/base.log 2>&1 || exit 1
VIT_HIP_LIB=$PWD/vision-transformer_amd/csrc/diag/lib_plain.so timeout -k 10 200 python tools/gemm_bench.py --impls 4 --reps 10 --only "$SH" --no-ref > gpurun_out/r1l/plain.log 2>&1 || exit 1
grep -hv amdgpu gpurun_out/r1l/base.log gpurun_out/r1l/plain.log
