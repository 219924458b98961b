# GPU box: the whole -m gpu suite, smoke(), one c2 bench line
# usage: bash scripts/gpu_suite.sh <tag>
set -e
TAG=${1:-suite}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1
tail -1 gpurun_out/$TAG/smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/$TAG/bench_c2.json 2> gpurun_out/$TAG/bench_c2.err
cat gpurun_out/$TAG/bench_c2.json
