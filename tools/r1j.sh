bash tools/gpu_check.sh r1j tests smoke bench prof || exit 1
cat gpurun_out/r1j/status.txt; tail -2 gpurun_out/r1j/tests.log; cat gpurun_out/r1j/bench.json
