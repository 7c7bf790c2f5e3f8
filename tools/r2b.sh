# round-2b GPU pass: all gpu tests, attention + GEMM A/B, bench (concurrent vs in-order wgrad), kernel profile
mkdir -p gpurun_out/r2b
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r2b/tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r2b/tests.log; exit 1; }
tail -2 gpurun_out/r2b/tests.log
timeout -k 10 200 python tools/attn_bench.py > gpurun_out/r2b/attn.log 2>&1 || exit 1
VIT_ATTN_FWD_SPLIT=1 timeout -k 10 200 python tools/attn_bench.py > gpurun_out/r2b/attn_split.log 2>&1 || exit 1
grep -h fwd gpurun_out/r2b/attn.log gpurun_out/r2b/attn_split.log
SH="fwd proj,fwd fc1,fwd fc2,dgrad fc2,dgrad fc1,dgrad qkv"
timeout -k 10 300 python tools/gemm_bench.py --impls 4 --reps 10 --epi --no-ref --only "$SH" > gpurun_out/r2b/gemm_tail.log 2>&1 || exit 1
VIT_GEMM_TAIL=0 timeout -k 10 300 python tools/gemm_bench.py --impls 4 --reps 10 --epi --no-ref --only "$SH" > gpurun_out/r2b/gemm_notail.log 2>&1 || exit 1
grep -hv amdgpu gpurun_out/r2b/gemm_tail.log gpurun_out/r2b/gemm_notail.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r2b/bench_conc.json 2> gpurun_out/r2b/bench_conc.err || { tail -20 gpurun_out/r2b/bench_conc.err; exit 1; }
VIT_CONCURRENT_WGRAD=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r2b/bench_seq.json 2> gpurun_out/r2b/bench_seq.err || exit 1
cat gpurun_out/r2b/bench_conc.json gpurun_out/r2b/bench_seq.json | cut -c1-400
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r2b/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r2b/prof.log 2>&1 || exit 1
echo done
