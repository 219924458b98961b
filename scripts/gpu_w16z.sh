# GPU box: dec_bwd_w16's P1 dZ on two waves in x6 (default) vs four waves in fp32 (ABCD_W16Z=0):
# parity at the fixtures and full shape, same-box A/B, stamps
set -e
OUT=gpurun_out/w16z
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_prod.py tests/test_gpu_fullshape.py -x -q --timeout 240 --timeout-method thread -k "fused_step or c2-512 or c5gru-512" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash scripts/ab_env.sh ABCD_W16Z "0 1" > $OUT/ab.log 2>&1; cat $OUT/ab.log
timeout -k 10 240 python -u scripts/persist_stamps.py > $OUT/persist_phase_stamps.log 2>&1 || echo "stamps failed"
grep -A12 "^dec_bwd" $OUT/persist_phase_stamps.log || true
echo w16z done
