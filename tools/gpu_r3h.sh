# GEMM memory-path diagnosis: L2 hit rate, L2 latency, TLB, TA, SQ waits per shape; tile-order grouping A/B
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r3h; mkdir -p $OUT
L=tools/variants/libvit_hip_steady.so
timeout -k 10 300 python tools/gemm_ab.py $L $L@VIT_GEMM_GROUP=2 $L@VIT_GEMM_GROUP=4 $L@VIT_GEMM_GROUP=8 --reps 6 > $OUT/group.txt 2>&1; echo "group rc=$?"; cat $OUT/group.txt
i=0
for grp in "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum" "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" "GRBM_GUI_ACTIVE" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $OUT/pmc$i -o run --output-format csv -- python tools/gemm_ab.py $L --reps 2 --shapes sq8192,fwd_qkv,fwd_fc1,dgrad_fc2,wgrad_fc1,fwd_proj > $OUT/pmc$i.log 2>&1 || { echo "pmc $i failed"; tail -3 $OUT/pmc$i.log; exit 1; }
  echo "pmc $i ok"
done
python - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for path in glob.glob("gpurun_out/r3h/pmc*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(path)):
        if "gemm_bf16_v4" not in r["Kernel_Name"] and "splitk" not in r["Kernel_Name"]: continue
        key = (r["Kernel_Name"].split("(")[0][-50:], r["Grid_Size"])
        agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for key, cs in agg.items():
    med = {c: sorted(v)[len(v)//2] for c, v in cs.items()}
    out = {}
    if "TCC_HIT_sum" in med: out["l2_hit"] = round(med["TCC_HIT_sum"] / max(1, med["TCC_HIT_sum"] + med["TCC_MISS_sum"]), 3)
    if "TCP_TCC_READ_REQ_sum" in med: out["l2_lat"] = round(med["TCP_TCC_READ_REQ_LATENCY_sum"] / max(1, med["TCP_TCC_READ_REQ_sum"]), 1)
    if "TCP_UTCL1_TRANSLATION_MISS_sum" in med: out["tlb_miss"] = med["TCP_UTCL1_TRANSLATION_MISS_sum"]; out["tcp_req"] = med["TCP_TCC_READ_REQ_sum"]
    if "TCP_PENDING_STALL_CYCLES_sum" in med: out["tcp_pend"] = med["TCP_PENDING_STALL_CYCLES_sum"]
    if "TA_BUSY_avr" in med: out["ta_busy"] = med["TA_BUSY_avr"]; out["ta_stall_tc"] = med["TA_ADDR_STALLED_BY_TC_CYCLES_sum"]
    if "SQ_WAVE_CYCLES" in med:
        w = med["SQ_WAVE_CYCLES"]; out["wait_any"] = round(med["SQ_WAIT_ANY"]/w, 3); out["wait_inst"] = round(med["SQ_WAIT_INST_ANY"]/w, 3); out["active"] = round(med["SQ_ACTIVE_INST_ANY"]/w, 3); out["lds_conf"] = med["SQ_LDS_BANK_CONFLICT"]
    if "SQ_VALU_MFMA_BUSY_CYCLES" in med and "GRBM_GUI_ACTIVE" in med: out["mfma_busy"] = round(med["SQ_VALU_MFMA_BUSY_CYCLES"]*8/(1024*med["GRBM_GUI_ACTIVE"]), 3)
    if "FETCH_SIZE" in med: out["fetch_MB_x2"] = round(med["FETCH_SIZE"]*2/1024, 1)
    print(key, out)
PY
