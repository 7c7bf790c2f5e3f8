set -u
OUT=gpurun_out/r4b; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k "v5_matches_v4 or kernels_exact" > $OUT/v5tests.log 2>&1
rc=$?; echo "v5tests rc=$rc" >> $OUT/status.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/gemm_ab.py vision-transformer_amd/VisionTransformer/libvit_hip.so vision-transformer_amd/VisionTransformer/libvit_hip.so@gemm_impl=5 --shapes fwd_qkv,fwd_proj,fwd_fc1m,fwd_fc2,dgrad_fc2m,dgrad_fc1,dgrad_qkv,dgrad_proj > $OUT/ab_v5.log 2>&1
rc=$?; echo "ab rc=$rc" >> $OUT/status.txt; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_check.sh r4a newtests bench
