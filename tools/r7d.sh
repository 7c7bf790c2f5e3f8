set -u
O=gpurun_out/r7d; mkdir -p $O; export TMPDIR=/tmp
step() { local n=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "$n rc=$rc" >> $O/status.txt; [ $rc -lt 124 ] || exit $rc; }
step attn_base 300 python -u tools/attn_bench.py > $O/attn_base.log 2>&1
step attn_qbuf 300 env VIT_HIP_LIB=tools/variants/libvit_hip_qbuf.so python -u tools/attn_bench.py > $O/attn_qbuf.log 2>&1
step attn_ord3 300 env VIT_HIP_LIB=tools/variants/libvit_hip_ord3.so python -u tools/attn_bench.py > $O/attn_ord3.log 2>&1
step attn_base2 300 python -u tools/attn_bench.py > $O/attn_base2.log 2>&1
step attn_qbuf2 300 env VIT_HIP_LIB=tools/variants/libvit_hip_qbuf.so python -u tools/attn_bench.py > $O/attn_qbuf2.log 2>&1
step attn_ord32 300 env VIT_HIP_LIB=tools/variants/libvit_hip_ord3.so python -u tools/attn_bench.py > $O/attn_ord32.log 2>&1
step tests 900 python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
step fp32 600 python -u -m pytest -v -s -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_model.py -k "full_depth" > $O/fp32.log 2>&1
