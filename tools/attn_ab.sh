# Attention A/B: tools/attn_bench.py on the in-tree library and on variant builds, alternating, on one box.
# usage: bash tools/attn_ab.sh TAG "variant1 variant2 ..."   (tools/variants/libvit_hip_<variant>.so)
set -u
OUT=gpurun_out/$1; mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  echo "== in-tree (round $r)" >> $OUT/attn_ab.log
  timeout -k 10 120 python -u tools/attn_bench.py --reps 30 >> $OUT/attn_ab.log 2>&1 || exit $?
  for v in $2; do
    echo "== $v (round $r)" >> $OUT/attn_ab.log
    VIT_HIP_LIB=tools/variants/libvit_hip_$v.so timeout -k 10 120 python -u tools/attn_bench.py --reps 30 >> $OUT/attn_ab.log 2>&1 || exit $?
  done
done
