# round-2zz: end-of-session validation (dK/dV at 2 waves/SIMD, 8-lane attn_delta): gpu tests, smoke, bench, ViT-L / 384^2 bench lines, kernel profiles
bash tools/gpu_check.sh r2zz tests smoke bench || exit 1
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r2zz/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-gemm-peak > gpurun_out/r2zz/prof.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --model large --batch 128 --steps 10 --warmup 3 --no-cpu-baseline --no-gemm-peak > gpurun_out/r2zz/bench_large.json 2> gpurun_out/r2zz/bench_large.err || exit 1
timeout -k 10 300 python bench.py --model base --img 384 --batch 64 --steps 10 --warmup 3 --no-cpu-baseline --no-gemm-peak > gpurun_out/r2zz/bench_384.json 2> gpurun_out/r2zz/bench_384.err || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r2zz/prof384 -o run --output-format csv -- python bench.py --model base --img 384 --batch 64 --steps 5 --warmup 2 --no-cpu-baseline --no-gemm-peak > gpurun_out/r2zz/prof384.log 2>&1 || exit 1
cat gpurun_out/r2zz/status.txt; tail -2 gpurun_out/r2zz/tests.log; tail -3 gpurun_out/r2zz/smoke.log; cat gpurun_out/r2zz/bench.json gpurun_out/r2zz/bench_large.json gpurun_out/r2zz/bench_384.json
