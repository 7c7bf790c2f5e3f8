# round-2f: v4 tile order inside an XCD (VIT_GEMM_GROUP tile rows per group, column-major inside) vs row-major
mkdir -p gpurun_out/r2f
SH="fwd qkv,fwd fc1,fwd fc2,dgrad fc2,dgrad fc1,wgrad fc1"
for G in 1 2 4 8 16; do
VIT_GEMM_GROUP=$G timeout -k 10 200 python tools/gemm_bench.py --impls 4 --reps 10 --no-ref --epi --only "$SH" > gpurun_out/r2f/g$G.log 2>&1 || exit 1
echo "== G=$G"; grep -v amdgpu gpurun_out/r2f/g$G.log
done
