# GPU box: a subset of the -m gpu tests, then ab_multi.sh over the given settings
# usage: bash scripts/gpu_tests_ab.sh "<test files>" "VAR=a" "VAR=b" ...
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
T="$1"; shift
timeout -k 10 900 python -u -m pytest $T -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1 || { tail -40 gpurun_out/pytest_ab.log; exit 1; }
tail -1 gpurun_out/pytest_ab.log
bash scripts/ab_multi.sh "$@"
