# split-major XCD mapping for split-K weight gradients: bitwise check, GEMM table, bench, wgrad PMC
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r3f; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; echo "tests rc=$?"; tail -3 $OUT/tests.log
timeout -k 10 300 python tools/gemm_bench.py --epi --reps 10 --no-ref > $OUT/gemm_bench.txt 2>&1; echo "gemm_bench rc=$?"; cat $OUT/gemm_bench.txt
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err; echo "bench rc=$?"; python -c "
import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['step_mfma_frac']); [print(k, v['ms_per_step'], v.get('tflops')) for k,v in d['roofline_families'].items()]"
P="python bench.py --steps 2 --warmup 1 --no-roofline --no-cpu-baseline --no-gemm-peak"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc1 -o run --output-format csv -- $P > $OUT/pmc1.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc2 -o run --output-format csv -- $P > $OUT/pmc2.log 2>&1 || exit 1
python tools/pmc_families.py base_224_b256_bf16 3 $OUT/pmc.json $OUT/pmc1 $OUT/pmc2 | grep -A4 "gemm_\""
