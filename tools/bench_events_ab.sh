# Overhead of bench.py's per-launch HIP events (the live roofline) on the headline step time: 2 rounds, same box.
OUT=gpurun_out/${1:-evab}; mkdir -p "$OUT"
for r in 1 2; do
  for v in "" "--no-roofline"; do
    line=$(timeout -k 10 180 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-gemm-peak $v 2>>"$OUT/err.log") || exit 1
    echo "$r [$v] $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a "$OUT/ab.log"
  done
done
