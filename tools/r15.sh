#!/bin/bash
set -u
OUT=gpurun_out/r15; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v -m gpu -p no:cacheprovider --timeout 120 \
  --timeout-method thread -k "w16" > $OUT/w16_tests.log 2>&1; rc=$?; echo "w16 tests rc=$rc" | tee -a $OUT/status.txt
[ $rc -ge 124 ] && exit $rc
for i in 1 2; do
  timeout -k 10 120 python -u tools/attn_bench.py > $OUT/attn_fused_$i.log 2>&1 || exit 1
  timeout -k 10 120 python -u tools/attn_bench.py --opt attn_bwd_w16=1 > $OUT/attn_w16_$i.log 2>&1 || exit 1
done
echo "bench ok" | tee -a $OUT/status.txt
