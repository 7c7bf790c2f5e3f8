# round-2y: attn_delta with 8 lanes per (row, head) (T > 256 path): kernel + model tests, 384^2 bench + profile
mkdir -p gpurun_out/r2y
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "attention" > gpurun_out/r2y/k.log 2>&1 || { tail -30 gpurun_out/r2y/k.log; exit 1; }
tail -1 gpurun_out/r2y/k.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -q -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread -k "long_sequence or full_size_configs" > gpurun_out/r2y/m.log 2>&1 || { tail -30 gpurun_out/r2y/m.log; exit 1; }
tail -1 gpurun_out/r2y/m.log
timeout -k 10 300 python bench.py --model base --img 384 --batch 64 --steps 10 --warmup 3 --no-cpu-baseline --no-gemm-peak > gpurun_out/r2y/bench_384.json 2> gpurun_out/r2y/bench_384.err || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r2y/prof384 -o run --output-format csv -- python bench.py --model base --img 384 --batch 64 --steps 5 --warmup 2 --no-cpu-baseline --no-gemm-peak > gpurun_out/r2y/prof384.log 2>&1 || exit 1
cat gpurun_out/r2y/bench_384.json
