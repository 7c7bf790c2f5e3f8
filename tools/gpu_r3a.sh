bash tools/gpu_check.sh r3b newtests || true
cat gpurun_out/r3b/status.txt; grep -E "PASS|FAIL|ERROR|exact-delta|worst" gpurun_out/r3b/newtests.log | tail -40
bash tools/gpu_check.sh r3b bench || exit 1
cat gpurun_out/r3b/bench.json; tail -5 gpurun_out/r3b/bench.err
