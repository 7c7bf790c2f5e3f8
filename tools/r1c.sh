# v4 GEMM: exactness, then A/B timing; then the pending model/train tests
mkdir -p gpurun_out/r1c
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -m gpu -p no:cacheprovider -k "gemm" -x > gpurun_out/r1c/k.log 2>&1 || { echo "kernel tests failed rc=$?"; tail -30 gpurun_out/r1c/k.log; exit 1; }
tail -2 gpurun_out/r1c/k.log
timeout -k 10 300 python tools/gemm_bench.py --impls 2,4 --reps 10 > gpurun_out/r1c/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r1c/bench.log; exit 1; }
cat gpurun_out/r1c/bench.log
timeout -k 10 600 python -m pytest tests/test_gpu_train.py tests/test_gpu_model.py -q -m gpu -p no:cacheprovider -k "tiny or data_parallel or train_loop" > gpurun_out/r1c/t.log 2>&1
echo "model tests rc=$?"; tail -5 gpurun_out/r1c/t.log
