# GPU box: a chosen subset of the -m gpu tests, then a same-box A/B of an
# environment setting on the c2 bench step.
# usage: bash scripts/gpu_ab_tests.sh "<test files>" VAR "v0 v1"
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest $1 -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1 || { tail -40 gpurun_out/pytest_ab.log; exit 1; }
tail -1 gpurun_out/pytest_ab.log
if [ -n "$2" ]; then bash scripts/ab_env.sh $2 "$3"; fi
