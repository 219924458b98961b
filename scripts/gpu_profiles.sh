# GPU box, end of a round (tests already run): smoke(), bench lines of every
# config, c2 rocprofv3 kernel stats, PMC traffic, one-step timeline, phase stamps
# usage: bash scripts/gpu_profiles.sh <tag>
set -e
TAG=${1:-final}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$TAG/smoke.log 2>&1
tail -1 gpurun_out/$TAG/smoke.log
bash scripts/gpu_profile.sh $TAG
bash scripts/gpu_timeline.sh ${TAG}tl
timeout -k 10 240 python -u scripts/persist_stamps.py > gpurun_out/$TAG/persist_phase_stamps.log 2>&1
echo profiles done
