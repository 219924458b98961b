# GPU box: gemm_wg3 forms (ABCD_WG3W: 8 = 8x1, default 4x2) against gemm_wg2 (alone, c2 shape), wgrad parity
set -e
OUT=gpurun_out/wgdiag
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/wg_probe.py 0 1 0 1 2>&1 | grep -v amdgpu.ids > $OUT/probe.log
echo "8x1" >> $OUT/probe.log
ABCD_WG3W=8 timeout -k 10 200 python -u scripts/wg_probe.py 1 1 2>&1 | grep -v amdgpu.ids >> $OUT/probe.log
echo "4x2 no split" >> $OUT/probe.log
ABCD_WG3DIAG=1 timeout -k 10 200 python -u scripts/wg_probe.py 1 1 2>&1 | grep -v amdgpu.ids >> $OUT/probe.log
cat $OUT/probe.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_persist.py -x -q --timeout 240 --timeout-method thread -k "wgrad" > $OUT/pytest_wgrad.log 2>&1 || { tail -40 $OUT/pytest_wgrad.log; exit 1; }
tail -1 $OUT/pytest_wgrad.log
