# GPU box: the production-shape parity tests + persistent-vs-per-step tests, then the c2 bench (no CPU leg)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sampler_head.py tests/test_gpu_prod.py tests/test_gpu_persist.py tests/test_gpu_parity.py tests/test_gpu_dp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_quick.log 2>&1 || { tail -30 gpurun_out/pytest_quick.log; exit 1; }
tail -1 gpurun_out/pytest_quick.log
for k in 1 2; do
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bq.json 2> gpurun_out/bq.err
python -c "import json;d=json.load(open('gpurun_out/bq.json'));print(d['ms_per_step'], {k:v['avg_launch_us'] for k,v in d['roofline']['all_kernels'].items()})"
done
