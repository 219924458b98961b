# GPU box, one build -> measure iteration:
#   1. the production-shape parity tests (reference fixtures + full-shape oracle) on the default path
#   2. a same-box A/B of environment settings on the c2 bench (alternating, 2 rounds); "-" = the defaults
#   3. with STAMPS=1: the persistent-kernel phase stamps and the contention probe
# usage: [STAMPS=1] bash scripts/gpu_iter.sh <tag> "-" "VAR=a" "VAR=b OTHER=c" ...
set -e
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_prod.py tests/test_gpu_fullshape.py tests/test_gpu_persist.py} \
  -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
grep -E "passed|failed" $OUT/pytest.log | tail -1
for rep in 1 2; do
  k=0
  for setting in "$@"; do
    k=$((k + 1))
    e=$setting; [ "$e" = "-" ] && e=""
    env $e timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/b_$k.json 2> $OUT/b_$k.err
    python -c "import json;d=json.load(open('$OUT/b_$k.json'));print('[$setting]', d['ms_per_step'], {k:v['avg_launch_us'] for k,v in d['roofline']['all_kernels'].items()})"
  done
done
if [ "$STAMPS" = "1" ]; then
  timeout -k 10 240 python -u scripts/persist_stamps.py > $OUT/persist_phase_stamps.log 2>&1
  timeout -k 10 300 python -u scripts/contention_probe.py > $OUT/contention_probe.log 2>&1
  echo stamps done
fi
