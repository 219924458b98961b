# GPU box: gemm_wg2 alone -- timing + f64 error at the c2 shape, its parity tests, then PMC passes
set -e
TAG=${1:-wg2b}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 120 python -u scripts/gemm_shapes.py wg2 > gpurun_out/$TAG/shapes.log 2>&1 || { cat gpurun_out/$TAG/shapes.log; exit 1; }
cat gpurun_out/$TAG/shapes.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_persist.py -k "wg2" -x -q --timeout 200 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { tail -40 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
bash scripts/pmc_gemm.sh wg2 gpurun_out/$TAG/pmc
python scripts/pmc_summary.py gpurun_out/$TAG/pmc 2>&1 | grep wg2 || true
