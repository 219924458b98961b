# GPU box: the gemm_wg2 encoder weight-gradient route -- timing alone, its tests,
# the full-shape c2 oracle test, then c2 bench lines with and without it (same box)
set -e
TAG=${1:-wg2}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 120 python -u scripts/gemm_shapes.py wg2 > gpurun_out/$TAG/shapes.log 2>&1 || { cat gpurun_out/$TAG/shapes.log; exit 1; }
cat gpurun_out/$TAG/shapes.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_persist.py -k "wg2 or bench_size" tests/test_gpu_fullshape.py -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { tail -40 gpurun_out/$TAG/pytest.log; exit 1; }
tail -3 gpurun_out/$TAG/pytest.log
for v in 1 0 1 0; do
ABCD_WG2=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/$TAG/b$v.json 2> gpurun_out/$TAG/b$v.err
python -c "import json;d=json.load(open('gpurun_out/$TAG/b$v.json'));print('WG2=$v', d['ms_per_step'], d['value'])"
done
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/kt -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/$TAG/kt.log 2>&1
echo done
