# GPU box: the full-shape and production parity tests under the non-default encoder weight-gradient forms
set -e
mkdir -p gpurun_out/forms
for f in "ABCD_WG3W=2" "ABCD_WG3W=8" "ABCD_WG3=0"; do
  env $f timeout -k 10 600 python -u -m pytest tests/test_gpu_fullshape.py tests/test_gpu_prod.py -x -q --timeout 240 --timeout-method thread -k "512 or prod" > gpurun_out/forms/p.log 2>&1 || { echo "$f"; tail -30 gpurun_out/forms/p.log; exit 1; }
  echo "$f: $(tail -1 gpurun_out/forms/p.log)"
done
