# round-3b: model-level tests through the T > 256 kernels after the attn_fwd_mfma occupancy change, and smoke
mkdir -p gpurun_out/r3b
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_train.py -q -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r3b/m.log 2>&1 || { tail -30 gpurun_out/r3b/m.log; exit 1; }
tail -1 gpurun_out/r3b/m.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2 || exit 1
