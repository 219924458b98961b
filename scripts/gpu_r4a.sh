set -e
mkdir -p gpurun_out/r4a
export TMPDIR=/tmp
timeout -k 10 60 python -u scripts/xcc_map.py > gpurun_out/r4a/xcc_map.log 2>&1; cat gpurun_out/r4a/xcc_map.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_trainer.py tests/test_gpu_feat.py tests/test_gpu_prod.py tests/test_gpu_fullshape.py -k "plain_checkpoint or op_surface or reference_toy_batch or gpu_featurize or timeout or c5-512 or c5gru-512" > gpurun_out/r4a/pytest_new.log 2>&1 || { tail -40 gpurun_out/r4a/pytest_new.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/r4a/pytest_new.log | tail -20
