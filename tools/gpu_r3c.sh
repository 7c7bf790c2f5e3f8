# round 3 validation pass: full GPU tests, smoke, bench
set -u
OUT=gpurun_out/r3c; mkdir -p $OUT
timeout -k 10 240 rocprofv3 -L > $OUT/counters.txt 2>&1; echo "list rc=$?"
bash tools/gpu_check.sh r3c tests smoke bench
tail -5 $OUT/tests.log; grep -E "FAILED|ERROR" $OUT/tests.log | head -20; tail -3 $OUT/smoke.log; cat $OUT/bench.json
