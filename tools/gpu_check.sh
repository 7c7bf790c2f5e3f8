#!/bin/bash
# One GPU-box pass: gpu tests, smoke, bench (+cpu baseline), rocprofv3 kernel stats of a short bench.
# Every GPU step has its own time limit; a crash/abort/timeout (exit >= 124 or signal) stops the script.
# usage: bash tools/gpu_check.sh TAG [tests|bench|prof ...]
set -u
TAG=${1:-run}; shift || true
STEPS=${*:-tests smoke bench prof}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { local rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; }
for s in $STEPS; do
  case $s in
    tests) timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 \
             --timeout-method thread > "$OUT/tests.log" 2>&1 ;;
    newtests) timeout -k 10 600 python -u -m pytest tests/test_gpu_dropin.py -v -m gpu -p no:cacheprovider \
             --timeout 300 --timeout-method thread > "$OUT/newtests.log" 2>&1 ;;
    kern) timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -v -m gpu -p no:cacheprovider \
             --timeout 120 --timeout-method thread > "$OUT/kern.log" 2>&1 ;;
    ab) timeout -k 10 300 python -u tools/gemm_ab.py vision-transformer_amd/VisionTransformer/libvit_hip.so \
          --shapes ${AB_SHAPES:-fwd_fc1,fwd_fc1m,dgrad_fc2,dgrad_fc2m} > "$OUT/ab.log" 2>&1 ;;
    model) timeout -k 10 900 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_dropin.py -x -v -m gpu \
             -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/model.log" 2>&1 ;;
    attn) timeout -k 10 300 python -u tools/attn_bench.py > "$OUT/attn.log" 2>&1 &&
          timeout -k 10 300 python -u tools/attn_bench.py --T 577 --batch 64 >> "$OUT/attn.log" 2>&1 ;;
    ln) timeout -k 10 300 python -u tools/ln_bench.py > "$OUT/ln.log" 2>&1 ;;
    lnab) for v in ${LN_VARIANTS:-}; do
            VIT_HIP_LIB=tools/variants/libvit_hip_$v.so timeout -k 10 120 python -u tools/ln_bench.py > "$OUT/ln_$v.log" 2>&1 || break
          done ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 ;;
    bench) timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" ;;
    prof) timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
            python bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/prof.log" 2>&1 ;;
    *) echo "unknown step $s"; continue ;;
  esac
  rc=$?
  echo "$s rc=$rc" | tee -a "$OUT/status.txt"
  if fatal $rc; then echo "stopping after fatal rc=$rc in $s"; exit $rc; fi
done
exit 0
