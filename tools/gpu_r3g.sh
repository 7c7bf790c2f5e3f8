# GEMM A/B: r2 baseline vs branch-free steady loop (+ split-major wgrad), ablations, deeper ring
set -u
OUT=gpurun_out/r3g; mkdir -p $OUT
V=tools/variants
timeout -k 10 400 python tools/gemm_ab.py $V/libvit_hip_r2.so $V/libvit_hip_steady.so $V/libvit_hip_lead8.so $V/libvit_hip_noepi.so $V/libvit_hip_nodma.so --reps 8 > $OUT/ab.txt 2>&1; echo "ab rc=$?"; cat $OUT/ab.txt
