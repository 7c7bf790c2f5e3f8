set -u
O=gpurun_out/r10b; mkdir -p $O
for r in 1 2; do
  for v in "-" "--opt gemm_tail=1"; do
    e=$v; [ "$e" = "-" ] && e=""
    for cfg in "--model large --batch 128" "--img 384 --batch 64"; do
      line=$(timeout -k 10 240 python bench.py --steps 15 --warmup 4 --no-cpu-baseline --no-gemm-peak --no-roofline $cfg $e 2>>$O/err.log) || exit 1
      echo "$r [$cfg] [$v] $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $O/ab.log
    done
  done
done
