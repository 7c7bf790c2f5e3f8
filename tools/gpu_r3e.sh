# round 3: C2 parity re-check, kernel-trace profile of the bench step, PMC passes per kernel family, GEMM shape table
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r3e; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_dropin.py -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k base_width > $OUT/parity.log 2>&1; echo "parity rc=$?"
grep -E "PASS|FAIL|worst" $OUT/parity.log
B="python bench.py --steps 10 --warmup 3 --no-roofline --no-cpu-baseline --no-gemm-peak"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- $B > $OUT/prof.log 2>&1 || { echo "prof failed"; exit 1; }
P="python bench.py --steps 2 --warmup 1 --no-roofline --no-cpu-baseline --no-gemm-peak"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS" "GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $grp -d $OUT/pmc$i -o run --output-format csv -- $P > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
  echo "pmc pass $i ok"
done
python tools/pmc_families.py base_224_b256_bf16 3 $OUT/pmc_base_224_b256_bf16.json $OUT/pmc1 $OUT/pmc2 $OUT/pmc3 $OUT/pmc4 > $OUT/pmc_summary.txt 2>&1; cat $OUT/pmc_summary.txt | head -80
timeout -k 10 300 python tools/gemm_bench.py --epi --reps 10 > $OUT/gemm_bench.txt 2>&1; echo "gemm_bench rc=$?"; cat $OUT/gemm_bench.txt
timeout -k 10 300 python tools/gemm_sweep.py > $OUT/gemm_sweep.txt 2>&1; echo "sweep rc=$?"; cat $OUT/gemm_sweep.txt
