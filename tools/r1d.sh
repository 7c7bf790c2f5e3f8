# ablations of the v4 GEMM + counters
mkdir -p gpurun_out/r1d
SH="fwd qkv,fwd fc2,dgrad fc1,wgrad fc1"
timeout -k 10 200 python tools/gemm_bench.py --impls 2,4 --reps 10 --only "$SH" --no-ref > gpurun_out/r1d/base.log 2>&1 || exit 1
VIT_HIP_LIB=$PWD/vision-transformer_amd/csrc/diag/lib_nodma.so timeout -k 10 200 python tools/gemm_bench.py --impls 4 --reps 10 --only "$SH" --no-ref > gpurun_out/r1d/nodma.log 2>&1 || exit 1
VIT_HIP_LIB=$PWD/vision-transformer_amd/csrc/diag/lib_nomfma.so timeout -k 10 200 python tools/gemm_bench.py --impls 4 --reps 10 --only "$SH" --no-ref > gpurun_out/r1d/nomfma.log 2>&1 || exit 1
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d gpurun_out/r1d/pmc_sq -o run --output-format csv -- python tools/gemm_one.py 50432 2304 768 4 > gpurun_out/r1d/pmc_sq.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-trace -d gpurun_out/r1d/pmc_tcc -o run --output-format csv -- python tools/gemm_one.py 50432 2304 768 4 > gpurun_out/r1d/pmc_tcc.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VMEM --kernel-trace -d gpurun_out/r1d/pmc_mfma -o run --output-format csv -- python tools/gemm_one.py 50432 2304 768 4 > gpurun_out/r1d/pmc_mfma.log 2>&1 || echo "mfma pmc failed (ignored)"
head -50 gpurun_out/r1d/*.log
