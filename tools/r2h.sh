# round-2h: attention tests + bench, bench with cpu baseline, kernel profile (committed as profiles/r2_*)
mkdir -p gpurun_out/r2h
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -x -p no:cacheprovider -k "attention" > gpurun_out/r2h/k.log 2>&1 || { echo "attention tests failed"; tail -30 gpurun_out/r2h/k.log; exit 1; }
tail -1 gpurun_out/r2h/k.log
timeout -k 10 200 python tools/attn_bench.py > gpurun_out/r2h/attn.log 2>&1 || exit 1
cat gpurun_out/r2h/attn.log
timeout -k 10 600 python bench.py > gpurun_out/r2h/bench.json 2> gpurun_out/r2h/bench.err || { tail -20 gpurun_out/r2h/bench.err; exit 1; }
cat gpurun_out/r2h/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r2h/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r2h/prof.log 2>&1 || exit 1
echo done
