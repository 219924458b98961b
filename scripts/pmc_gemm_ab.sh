# PMC passes of one GEMM shape under two env settings (scripts/gemm_shapes.py names)
# usage: bash scripts/pmc_gemm_ab.sh <shape> "<VAR=a>" "<VAR=b>"   (outputs gpurun_out/pmcab_<tag>/)
set -e
SHAPE=$1; shift
export TMPDIR=/tmp
for setting in "$@"; do
  tag=$(echo "$setting" | tr '= ' '__')
  OUT=gpurun_out/pmcab_$tag
  mkdir -p $OUT
  for pass in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
              "FETCH_SIZE SQ_ACTIVE_INST_MFMA SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES" \
              "WRITE_SIZE SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_WAVES GRBM_GUI_ACTIVE" \
              "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum SQ_INSTS_SALU"; do
    n=$(echo $pass | cut -c1-8 | tr -d ' ')
    ( export $setting; timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d $OUT/p_$n -o run -- python3 scripts/gemm_shapes.py $SHAPE > $OUT/p_$n.log 2>&1 ) || echo "pass $n failed"
  done
  python scripts/pmc_summary.py $OUT > $OUT/summary.txt
  echo "== $setting"; cat $OUT/summary.txt
done
