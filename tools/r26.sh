#!/bin/bash
# r26: the whole GPU suite and smoke at HEAD (after the auto attention_probs default)
set -u
O=gpurun_out/r26; mkdir -p $O; export TMPDIR=/tmp
step() { local n=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "$n rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || exit $rc; }
step tests 900 python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
