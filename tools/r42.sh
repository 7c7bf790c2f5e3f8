#!/bin/bash
# r42: ring forward with the Q double buffer (RING_QBUF=1) — attention / model GPU tests, then whole-step A/B vs the
# previous library (tools/variants/libvit_hip_head.so)
set -u
O=gpurun_out/r42; mkdir -p $O; export TMPDIR=/tmp
step() { local n=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "$n rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || exit $rc; }
step tests 900 python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
step ab 900 bash tools/lib_ab.sh r42 3 tools/variants/libvit_hip_head.so
