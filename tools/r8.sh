set -u
T=${1:-r8}
O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
step() { local n=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "$n rc=$rc" >> $O/status.txt; [ $rc -lt 124 ] || exit $rc; }
step tests 900 python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step bench 900 python bench.py > $O/bench.json 2> $O/bench.err
step c4 600 python bench.py --model large --batch 128 --no-cpu-baseline --no-gemm-peak > $O/c4.json 2> $O/c4.err
step c5 600 python bench.py --img 384 --batch 64 --no-cpu-baseline --no-gemm-peak > $O/c5.json 2> $O/c5.err
step profsteps 600 bash tools/gpu_prof_steps.sh $T/profsteps
step pmc 1200 bash tools/gpu_profile.sh $T/prof
