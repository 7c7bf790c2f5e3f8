#!/bin/bash
set -u
OUT=gpurun_out/r19; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_dropin.py tests/test_gpu_train.py -x -v -m gpu -p no:cacheprovider \
  --timeout 300 --timeout-method thread -k "optimizer_in_backward or adamw or train or rccl or checkpoint or data_parallel" > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc" | tee -a $OUT/status.txt; [ $rc -ne 0 ] && exit $rc
bash tools/bench_ab.sh r19 3 "-" "--optimizer-in-backward 0" && echo "ab ok" | tee -a $OUT/status.txt
