# GPU box: dec_fwd_x6 EK emit (all 32 members, K split in two) -- the -m gpu suite, same-box A/B, stamps
set -e
OUT=gpurun_out/ek
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
bash scripts/ab_env.sh ABCD_DECFWD_EK "0 1" > $OUT/ab.log 2>&1; cat $OUT/ab.log
timeout -k 10 240 python -u scripts/persist_stamps.py > $OUT/persist_phase_stamps.log 2>&1; grep -A9 "^dec_fwd" $OUT/persist_phase_stamps.log
