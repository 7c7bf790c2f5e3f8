#!/bin/bash
# round 6 evidence at HEAD (end of round 6: AdamW chunks, GEMM setprio, ring Q buffer): tests, smoke, C2/C4/C5 bench lines, kernel traces (default and in-order schedules) and the
# PMC families under the in-order schedule the roofline step times (tools/gpu_profile.sh)
set -u
T=${1:-r61}
O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
step() { local n=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "$n rc=$rc" >> $O/status.txt; [ $rc -lt 124 ] || exit $rc; }
step tests 900 python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step bench 600 python bench.py > $O/bench.json 2> $O/bench.err
step c4 600 python bench.py --model large --batch 128 --no-cpu-baseline --no-gemm-peak > $O/c4.json 2> $O/c4.err
step c5 600 python bench.py --img 384 --batch 64 --no-cpu-baseline --no-gemm-peak > $O/c5.json 2> $O/c5.err
step profsteps 600 bash tools/gpu_prof_steps.sh $T/profsteps
step profsteps_inorder 600 bash tools/gpu_prof_steps.sh $T/profsteps_inorder --engine fwd_streams=1 --engine concurrent_wgrad=0
step pmc 1200 bash tools/gpu_profile.sh $T/prof
