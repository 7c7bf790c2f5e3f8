set -u
OUT=gpurun_out/${1:-r4c}; mkdir -p $OUT
export TMPDIR=/tmp
L=vision-transformer_amd/VisionTransformer/libvit_hip.so
timeout -k 10 300 python -u tools/gemm_ab.py $L $L@gemm_impl=5 ${EXTRA_LIBS:-} --shapes ${SHAPES:-fwd_qkv,fwd_proj,fwd_fc1m,fwd_fc2,dgrad_fc2m,dgrad_fc1,dgrad_qkv,dgrad_proj} > $OUT/ab_v5.log 2>&1
