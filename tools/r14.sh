#!/bin/bash
# round 6: attn_bwd_w16 kernel tests + isolated A/B vs attn_bwd_fused, then the GPU test files after test_gpu_kernels
set -u
OUT=gpurun_out/r14; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v -m gpu -p no:cacheprovider --timeout 120 \
  --timeout-method thread -k "w16 or ring_ragged" > $OUT/w16_tests.log 2>&1; rc=$?; echo "w16 tests rc=$rc" | tee -a $OUT/status.txt
[ $rc -ge 124 ] && exit $rc
for i in 1 2; do
  timeout -k 10 120 python -u tools/attn_bench.py > $OUT/attn_fused_$i.log 2>&1 || exit 1
  timeout -k 10 120 python -u tools/attn_bench.py --opt attn_bwd_w16=1 > $OUT/attn_w16_$i.log 2>&1 || exit 1
done
echo "bench ok" | tee -a $OUT/status.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_train.py -v -m gpu -p no:cacheprovider \
  --timeout 300 --timeout-method thread > $OUT/model_train.log 2>&1; echo "model/train rc=$?" | tee -a $OUT/status.txt
