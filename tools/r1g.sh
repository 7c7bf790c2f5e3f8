mkdir -p gpurun_out/r1g
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -m gpu -p no:cacheprovider -k "attention" -x > gpurun_out/r1g/k.log 2>&1 || { echo "attn tests failed"; tail -30 gpurun_out/r1g/k.log; exit 1; }
tail -1 gpurun_out/r1g/k.log
timeout -k 10 300 python tools/attn_bench.py > gpurun_out/r1g/attn.log 2>&1 || { tail gpurun_out/r1g/attn.log; exit 1; }
cat gpurun_out/r1g/attn.log
