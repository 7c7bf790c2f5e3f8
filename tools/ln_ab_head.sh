# A/B of LayerNorm library variants (tools/build_variant.sh ... vit_norm): usage bash tools/ln_ab_head.sh TAG ROUNDS VARIANT...
# ("default" = the in-tree library)
TAG=$1; R=$2; shift 2
mkdir -p gpurun_out/$TAG
for i in $(seq 1 "$R"); do
  for v in "$@"; do
    echo "== $v" >> gpurun_out/$TAG/ln.log
    if [ "$v" = default ]; then lib=""; else lib="VIT_HIP_LIB=tools/variants/libvit_hip_$v.so"; fi
    env $lib timeout -k 10 60 python -u tools/ln_bench.py >> gpurun_out/$TAG/ln.log 2>&1 || exit 1
  done
done
