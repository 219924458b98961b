# GPU box: nt-load hand-off gathers (ABCD_NTLD=1) -- parity (prod fixtures, c2 / c5gru full shape), same-box A/B
set -e
OUT=gpurun_out/nt
mkdir -p $OUT
export TMPDIR=/tmp
ABCD_NTLD=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_prod.py tests/test_gpu_fullshape.py -x -q --timeout 240 --timeout-method thread -k "c2-512 or c5gru-512 or c4-512" > $OUT/pytest_nt.log 2>&1 || { tail -40 $OUT/pytest_nt.log; exit 1; }
tail -1 $OUT/pytest_nt.log
bash scripts/ab_env.sh ABCD_NTLD "0 1" > $OUT/ab.log 2>&1; cat $OUT/ab.log
ABCD_NTLD=1 timeout -k 10 240 python -u scripts/persist_stamps.py > $OUT/persist_phase_stamps.log 2>&1 || echo "stamps failed"
grep -B1 -A3 "median ns" $OUT/persist_phase_stamps.log || true
echo nt done
