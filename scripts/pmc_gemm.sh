# PMC counters of one GEMM route at a c2 hot-path shape (scripts/gemm_shapes.py names: xproj, offset-head, dW_hh, dW_ih)
# usage: bash scripts/pmc_gemm.sh <shape> [outdir]
set -e
SHAPE=${1:-dW_hh}
OUT=${2:-gpurun_out/pmc_$SHAPE}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 scripts/gemm_shapes.py $SHAPE > $OUT/kt.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $OUT/pmc1 -o run -- python3 scripts/gemm_shapes.py $SHAPE > $OUT/pmc1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE SQ_ACTIVE_INST_MFMA SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc2 -o run -- python3 scripts/gemm_shapes.py $SHAPE > $OUT/pmc2.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc3 -o run -- python3 scripts/gemm_shapes.py $SHAPE > $OUT/pmc3.log 2>&1
