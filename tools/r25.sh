#!/bin/bash
# r25: auto attention_probs + vectorized AdamW: the affected GPU tests, smoke, and the AdamW kernel time in the step
set -u
O=gpurun_out/r25; mkdir -p $O; export TMPDIR=/tmp
step() { local n=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "$n rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || exit $rc; }
step tests 400 python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu tests -k "probs or adamw" > $O/tests.log 2>&1
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step prof 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-gemm-peak --no-roofline > $O/bench.json 2> $O/bench.err
S=$(find $O/trace -name "*kernel_stats.csv" | head -1); cp "$S" $O/kernel_stats.csv; rm -rf $O/trace
