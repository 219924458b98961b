# GPU box: gemm_wg3 at 4 and 8 waves against gemm_wg2 (alone, c2 shape), probes (ABCD_WG3DIAG), wgrad parity
set -e
OUT=gpurun_out/wgdiag
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/wg_probe.py 0 1 0 1 2>&1 | grep -v amdgpu.ids > $OUT/probe.log
echo "4 waves" >> $OUT/probe.log
ABCD_WG3W=4 timeout -k 10 200 python -u scripts/wg_probe.py 1 1 2>&1 | grep -v amdgpu.ids >> $OUT/probe.log
for dg in 1 2 3 4; do
  echo "8 waves DIAG $dg" >> $OUT/probe.log
  ABCD_WG3DIAG=$dg timeout -k 10 200 python -u scripts/wg_probe.py 1 1 2>&1 | grep -v amdgpu.ids >> $OUT/probe.log
done
cat $OUT/probe.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_persist.py -x -q --timeout 240 --timeout-method thread -k "wgrad" > $OUT/pytest_wgrad.log 2>&1 || { tail -40 $OUT/pytest_wgrad.log; exit 1; }
tail -1 $OUT/pytest_wgrad.log
