# A/B of the LayerNorm kernels (tools/ln_bench.py) across runtime switches: usage bash tools/ln_sweep.sh TAG "ENV1" "ENV2" ...
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for v in "$@"; do
  echo "== $v" >> gpurun_out/$TAG/ln.log
  env $v timeout -k 10 60 python -u tools/ln_bench.py >> gpurun_out/$TAG/ln.log 2>&1 || exit 1
done
