# PMC counters of one kernel of the c2 step (bench.py, 3 timed steps), by regex
# usage: bash scripts/pmc_step_kernel.sh <kernel-regex> <outdir>
set -e
RX=$1
OUT=${2:-gpurun_out/pmc_step}
mkdir -p $OUT
export TMPDIR=/tmp
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --kernel-include-regex "$RX" --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $OUT/pmc1 -o run -- $B > $OUT/pmc1.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-include-regex "$RX" --pmc FETCH_SIZE SQ_ACTIVE_INST_MFMA SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc2 -o run -- $B > $OUT/pmc2.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-include-regex "$RX" --pmc WRITE_SIZE SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc3 -o run -- $B > $OUT/pmc3.log 2>&1
python3 scripts/pmc_summary.py $OUT
