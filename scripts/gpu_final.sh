# GPU box, end of a round: the whole -m gpu suite, smoke(), then the profile set
# (bench lines of every config, c2 rocprofv3 stats, PMC traffic, one-step timeline, phase stamps)
# usage: bash scripts/gpu_final.sh <tag>
set -e
TAG=${1:-final}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$TAG/smoke.log 2>&1
tail -1 gpurun_out/$TAG/smoke.log
bash scripts/gpu_profile.sh $TAG
bash scripts/gpu_timeline.sh ${TAG}tl
timeout -k 10 240 python -u scripts/persist_stamps.py > gpurun_out/$TAG/persist_phase_stamps.log 2>&1
timeout -k 10 300 python -u scripts/contention_probe.py > gpurun_out/$TAG/contention_probe.log 2>&1
echo final done
