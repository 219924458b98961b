# GPU box: one rocprofv3 PMC pass of MFMA utilisation over the c2 bench (all kernels)
# usage: bash scripts/gpu_pmc_mfma.sh <outdir> [config]
set -e
OUT=${1:-gpurun_out/pmc_mfma}
C=${2:-c2}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVE_CYCLES --output-format csv -d $OUT/pass -o run -- python3 bench.py --config $C --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing > $OUT/pass.log 2>&1
python3 scripts/pmc_mfma.py $OUT/pass $OUT/pmc_mfma.json $C
