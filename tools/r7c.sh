set -u
O=gpurun_out/r7c; mkdir -p $O; export TMPDIR=/tmp
step() { local n=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "$n rc=$rc" >> $O/status.txt; [ $rc -lt 124 ] || exit $rc; }
step gemm 600 python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "tail_split or persistent" > $O/gemm.log 2>&1
step tests 900 python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
step bench_on 600 python bench.py --no-cpu-baseline --no-gemm-peak > $O/bench_on.json 2> $O/bench_on.err
step bench_off 600 python bench.py --no-cpu-baseline --no-gemm-peak --opt gemm_tail_v2=0 > $O/bench_off.json 2> $O/bench_off.err
step bench_on2 600 python bench.py --no-cpu-baseline --no-gemm-peak > $O/bench_on2.json 2> $O/bench_on2.err
