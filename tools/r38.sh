#!/bin/bash
# r38: pair-hash dropout keep bits — BDR epilogue GEMM timing vs the previous library (masks differ by design: '!'),
# then the whole GPU suite and smoke
set -u
O=gpurun_out/r38; mkdir -p $O; export TMPDIR=/tmp
step() { local n=$1; shift; timeout -k 10 "$@"; local rc=$?; echo "$n rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || exit $rc; }
step gemm 300 python -u tools/gemm_ab.py vision-transformer_amd/VisionTransformer/libvit_hip.so tools/variants/libvit_hip_prevhash.so --shapes fwd_proj,fwd_fc2,fwd_proj_bdrm,fwd_fc2_bdrm,fwd_proj_br,fwd_fc2_br > $O/gemm_ab.log 2>&1
step tests 900 python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
