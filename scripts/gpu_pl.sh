# GPU box: plain-load mlp / emit gathers in dec_fwd_x6 (ABCD_PLLD=1): parity twice at c2 / c4 / c5 / c5gru
# full shape (8 row groups), same-box A/B
set -e
OUT=gpurun_out/pl
mkdir -p $OUT
export TMPDIR=/tmp
for k in 1 2; do
ABCD_PLLD=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_fullshape.py -x -q --timeout 240 --timeout-method thread -k "512" > $OUT/pytest_$k.log 2>&1 || { tail -40 $OUT/pytest_$k.log; exit 1; }
tail -1 $OUT/pytest_$k.log
done
bash scripts/ab_env.sh ABCD_PLLD "0 1" > $OUT/ab.log 2>&1; cat $OUT/ab.log
echo pl done
