# round-2j: final validation of the round: all gpu tests, smoke, bench (default flags), kernel profile
bash tools/gpu_check.sh r2j tests smoke bench || exit 1
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r2j/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-gemm-peak > gpurun_out/r2j/prof.log 2>&1 || exit 1
cat gpurun_out/r2j/status.txt; tail -2 gpurun_out/r2j/tests.log; tail -3 gpurun_out/r2j/smoke.log; cat gpurun_out/r2j/bench.json
