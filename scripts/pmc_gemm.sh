# PMC counters of the weight-gradient GEMM at the c2 dW_hh shape (scripts/gemm_shapes.py dW_hh)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt -o run -- python3 scripts/gemm_shapes.py dW_hh > gpurun_out/kt.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/pmc1 -o run -- python3 scripts/gemm_shapes.py dW_hh > gpurun_out/pmc1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE SQ_ACTIVE_INST_MFMA SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc2 -o run -- python3 scripts/gemm_shapes.py dW_hh > gpurun_out/pmc2.log 2>&1
