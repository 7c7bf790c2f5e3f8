#!/bin/bash
set -u
OUT=gpurun_out/r18; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -v -m gpu -p no:cacheprovider \
  --timeout 200 --timeout-method thread -k "transpose or dgrad_transposed or row0_mode or two_stream" > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc" | tee -a $OUT/status.txt; [ $rc -ne 0 ] && exit $rc
bash tools/bench_ab.sh r18 3 "-" "--engine dgrad_wt=0" && echo "ab ok" | tee -a $OUT/status.txt
timeout -k 10 180 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-gemm-peak --engine fwd_streams=1 --engine concurrent_wgrad=0 > $OUT/inorder_wt.json 2>>$OUT/err.log
timeout -k 10 180 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-gemm-peak --engine fwd_streams=1 --engine concurrent_wgrad=0 --engine dgrad_wt=0 > $OUT/inorder_nowt.json 2>>$OUT/err.log
echo done | tee -a $OUT/status.txt
