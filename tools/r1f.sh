bash tools/gpu_check.sh r1f tests smoke bench prof || exit 1
timeout -k 10 300 python tools/gemm_bench.py --impls 2,4 --reps 10 > gpurun_out/r1f/gemm.log 2>&1
cat gpurun_out/r1f/status.txt; tail -3 gpurun_out/r1f/tests.log; cat gpurun_out/r1f/bench.json; grep -v amdgpu.ids gpurun_out/r1f/gemm.log
