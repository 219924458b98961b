# GPU box: gemm_wg2 alone -- timing + f64 error at the c2 shape, then PMC passes
set -e
TAG=${1:-wg2b}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 120 python -u scripts/gemm_shapes.py wg2 dW_hh dW_ih > gpurun_out/$TAG/shapes.log 2>&1 || { cat gpurun_out/$TAG/shapes.log; exit 1; }
cat gpurun_out/$TAG/shapes.log
bash scripts/pmc_gemm.sh wg2 gpurun_out/$TAG/pmc
python scripts/pmc_summary.py gpurun_out/$TAG/pmc 2>&1 | tail -40 || true
