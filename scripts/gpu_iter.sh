# GPU box, one build -> measure iteration:
#   1. the production-shape parity tests (reference fixtures + full-shape oracle) on the default path
#   2. a same-box A/B of one environment switch on the c2 bench (alternating, 2 pairs)
#   3. optionally the persistent-kernel phase stamps and the contention probe
# usage: bash scripts/gpu_iter.sh <tag> <VAR> "<v_a> <v_b>" [stamps]
set -e
TAG=$1; VAR=$2; VALS=$3
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_prod.py tests/test_gpu_fullshape.py tests/test_gpu_persist.py \
  -x -q --timeout 120 --timeout-method thread --durations=10 -rA > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
grep -E "passed|failed" $OUT/pytest.log | tail -1
for rep in 1 2; do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/b_$v.json 2> $OUT/b_$v.err
    python -c "import json;d=json.load(open('$OUT/b_$v.json'));print('$VAR=$v', d['ms_per_step'], {k:v['avg_launch_us'] for k,v in d['roofline']['all_kernels'].items()})"
  done
done
if [ "$4" = "stamps" ]; then
  timeout -k 10 240 python -u scripts/persist_stamps.py > $OUT/persist_phase_stamps.log 2>&1
  timeout -k 10 300 python -u scripts/contention_probe.py > $OUT/contention_probe.log 2>&1
  echo stamps done
fi
