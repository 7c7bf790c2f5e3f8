# round-2m: validation of the global_load_lds GEMM staging across the full stack: gpu tests, smoke, bench, kernel profile
bash tools/gpu_check.sh r2m tests smoke bench || exit 1
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r2m/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-gemm-peak > gpurun_out/r2m/prof.log 2>&1 || exit 1
cat gpurun_out/r2m/status.txt; tail -2 gpurun_out/r2m/tests.log; tail -3 gpurun_out/r2m/smoke.log; cat gpurun_out/r2m/bench.json
