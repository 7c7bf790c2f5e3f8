set -u
O=gpurun_out/r7b; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/attn_bench.py --opt attn_fwd_ring=0 > $O/attn_old.log 2>&1; echo "attn_old rc=$?" >> $O/status.txt
timeout -k 10 300 python -u tools/attn_bench.py > $O/attn_new.log 2>&1; echo "attn_new rc=$?" >> $O/status.txt
timeout -k 10 600 python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "attention" > $O/kern_attn.log 2>&1; echo "kern rc=$?" >> $O/status.txt
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1; echo "tests rc=$?" >> $O/status.txt
timeout -k 10 600 python -u tools/diag_fp32_depth.py > $O/diag.log 2>&1; echo "diag rc=$?" >> $O/status.txt
timeout -k 10 600 python bench.py --no-cpu-baseline --no-gemm-peak > $O/bench.json 2> $O/bench.err; echo "bench rc=$?" >> $O/status.txt
