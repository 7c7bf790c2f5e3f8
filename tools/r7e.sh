set -u
O=gpurun_out/r7e; mkdir -p $O; export TMPDIR=/tmp
step() { local n=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "$n rc=$rc" >> $O/status.txt; [ $rc -lt 124 ] || exit $rc; }
L=vision-transformer_amd/VisionTransformer/libvit_hip.so
V=tools/variants/libvit_hip_dmamfma.so
step gemmtest 600 env VIT_HIP_LIB=$V python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "gemm" > $O/gemmtest.log 2>&1
step ab 600 python -u tools/gemm_ab.py $L $V --reps 10 --shapes fwd_qkv,fwd_proj,fwd_fc1m,fwd_fc2,dgrad_fc2m,dgrad_fc1,dgrad_qkv,dgrad_proj,wgrad_fc1,wgrad_qkv > $O/ab.log 2>&1
step bench_base 600 python bench.py --no-cpu-baseline --no-gemm-peak > $O/bench_base.json 2> $O/bench_base.err
step bench_var 600 env VIT_HIP_LIB=$V python bench.py --no-cpu-baseline --no-gemm-peak > $O/bench_var.json 2> $O/bench_var.err
step bench_base2 600 python bench.py --no-cpu-baseline --no-gemm-peak > $O/bench_base2.json 2> $O/bench_base2.err
step bench_var2 600 env VIT_HIP_LIB=$V python bench.py --no-cpu-baseline --no-gemm-peak > $O/bench_var2.json 2> $O/bench_var2.err
