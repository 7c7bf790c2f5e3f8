# round-2d: PMC counters of the QKV-forward GEMM (gemm_bf16_v4<kc,kc,bf16,PLAIN>, M=50432 N=2304 K=768, 5 launches);
# one counter group per rocprofv3 pass
mkdir -p gpurun_out/r2d
export TMPDIR=/tmp
P="python tools/gemm_one.py 50432 2304 768"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT -d gpurun_out/r2d/p1 -o run --output-format csv -- $P > gpurun_out/r2d/p1.log 2>&1 || { tail -5 gpurun_out/r2d/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE FETCH_SIZE -d gpurun_out/r2d/p2 -o run --output-format csv -- $P > gpurun_out/r2d/p2.log 2>&1 || { tail -5 gpurun_out/r2d/p2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA -d gpurun_out/r2d/p3 -o run --output-format csv -- $P > gpurun_out/r2d/p3.log 2>&1 || { tail -5 gpurun_out/r2d/p3.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r2d/kt -o run --output-format csv -- $P > gpurun_out/r2d/kt.log 2>&1 || exit 1
ls gpurun_out/r2d/*/
