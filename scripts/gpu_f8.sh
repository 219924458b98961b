# GPU box: enc_fwd_w8 (32-row groups of 8 members) -- the -m gpu suite, same-box A/B against enc_fwd_persist, stamps
set -e
OUT=gpurun_out/f8
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
bash scripts/ab_env.sh ABCD_ENCFWD "p w" > $OUT/ab.log 2>&1; cat $OUT/ab.log
timeout -k 10 240 python -u scripts/persist_stamps.py > $OUT/persist_phase_stamps.log 2>&1; grep -A5 "^enc_fwd" $OUT/persist_phase_stamps.log
