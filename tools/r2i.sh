mkdir -p gpurun_out/r2i
timeout -k 10 120 python tools/ln_bench.py > gpurun_out/r2i/new.log 2>&1 || exit 1
VIT_HIP_LIB=$PWD/vision-transformer_amd/csrc/diag/lib_lnold.so timeout -k 10 120 python tools/ln_bench.py > gpurun_out/r2i/old.log 2>&1 || exit 1
grep -hv amdgpu gpurun_out/r2i/new.log gpurun_out/r2i/old.log
