# round-2o: persistent attention backward (next item staged during the current one): kernel tests, timing vs one item per workgroup, model tests
mkdir -p gpurun_out/r2o
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "attention" > gpurun_out/r2o/k.log 2>&1 || { tail -30 gpurun_out/r2o/k.log; exit 1; }
tail -1 gpurun_out/r2o/k.log
timeout -k 10 120 python tools/attn_bench.py --reps 10 > gpurun_out/r2o/persist.log 2>&1 || exit 1
VIT_ATTN_BWD_GRID=1000000 timeout -k 10 120 python tools/attn_bench.py --reps 10 > gpurun_out/r2o/oneitem.log 2>&1 || exit 1
echo "== persistent"; grep -v amdgpu gpurun_out/r2o/persist.log; echo "== one item per workgroup"; grep -v amdgpu gpurun_out/r2o/oneitem.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_train.py -q -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread -s > gpurun_out/r2o/m.log 2>&1 || { tail -40 gpurun_out/r2o/m.log; exit 1; }
tail -1 gpurun_out/r2o/m.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-gemm-peak > gpurun_out/r2o/bench.json 2> gpurun_out/r2o/bench.err || exit 1
cat gpurun_out/r2o/bench.json
