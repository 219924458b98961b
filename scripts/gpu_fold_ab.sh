# GPU box: the folded decoder BPTT (dec_bwd_fold) against the reference
# fixtures and the full-shape oracle test, then a same-box A/B with dec_bwd_sk
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
ABCD_DECBWD=fold timeout -k 10 900 python -u -m pytest tests/test_gpu_prod.py tests/test_gpu_fullshape.py tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_fold.log 2>&1 || { tail -40 gpurun_out/pytest_fold.log; exit 1; }
tail -1 gpurun_out/pytest_fold.log
bash scripts/ab_env.sh ABCD_DECBWD "sk fold"
timeout -k 10 600 python -u -m pytest tests/test_gpu_modules.py tests/test_gpu_x6.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_mod.log 2>&1 || { tail -40 gpurun_out/pytest_mod.log; exit 1; }
tail -1 gpurun_out/pytest_mod.log
