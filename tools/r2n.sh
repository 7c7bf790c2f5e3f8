# round-2n: new long-sequence / full-size config tests; bench lines for BASELINE configs 4 (ViT-L/16 B=128) and 5 (ViT-B/16 384^2 B=64)
mkdir -p gpurun_out/r2n
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -v -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread -k "long_sequence or full_size_configs" > gpurun_out/r2n/tests.log 2>&1 || { tail -40 gpurun_out/r2n/tests.log; exit 1; }
tail -8 gpurun_out/r2n/tests.log
timeout -k 10 300 python bench.py --model large --batch 128 --steps 10 --warmup 3 --no-cpu-baseline --no-gemm-peak > gpurun_out/r2n/bench_large.json 2> gpurun_out/r2n/bench_large.err || exit 1
timeout -k 10 300 python bench.py --model base --img 384 --batch 64 --steps 10 --warmup 3 --no-cpu-baseline --no-gemm-peak > gpurun_out/r2n/bench_384.json 2> gpurun_out/r2n/bench_384.err || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r2n/prof384 -o run --output-format csv -- python bench.py --model base --img 384 --batch 64 --steps 5 --warmup 2 --no-cpu-baseline --no-gemm-peak > gpurun_out/r2n/prof384.log 2>&1 || exit 1
cat gpurun_out/r2n/bench_large.json gpurun_out/r2n/bench_384.json
