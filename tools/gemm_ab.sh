# A/B of the in-tree library against variant builds on the C2 GEMM shapes (tools/gemm_ab.py, interleaved rounds).
# usage: bash tools/gemm_ab.sh TAG "VARIANT_SPECS" [SHAPES]  -> gpurun_out/TAG/ab.log
set -u
OUT=gpurun_out/$1; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/gemm_ab.py vision-transformer_amd/VisionTransformer/libvit_hip.so $2 \
  --shapes ${3:-fwd_qkv,fwd_proj,fwd_fc1m,fwd_fc2,dgrad_fc2m,dgrad_fc1,dgrad_qkv,dgrad_proj} > $OUT/ab.log 2>&1
