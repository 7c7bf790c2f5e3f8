# round-2e: v4 ablations (no LDS-DMA / no MFMA) on three shapes
mkdir -p gpurun_out/r2e
SH="fwd qkv,fwd fc2,wgrad fc1"
timeout -k 10 200 python tools/gemm_bench.py --impls 4 --reps 10 --no-ref --only "$SH" > gpurun_out/r2e/base.log 2>&1 || exit 1
for v in NODMA NOMFMA; do
VIT_HIP_LIB=$PWD/vision-transformer_amd/csrc/diag/lib_$v.so timeout -k 10 200 python tools/gemm_bench.py --impls 4 --reps 10 --only "$SH" --no-ref > gpurun_out/r2e/$v.log 2>&1 || exit 1
done
grep -h -v amdgpu gpurun_out/r2e/base.log gpurun_out/r2e/NODMA.log gpurun_out/r2e/NOMFMA.log
