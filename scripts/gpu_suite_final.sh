# GPU box: the whole -m gpu suite and smoke() on the final tree
set -e
mkdir -p gpurun_out/fin
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/fin/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/fin/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/fin/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/fin/smoke.log 2>&1
tail -2 gpurun_out/fin/smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/fin/bench.json 2> gpurun_out/fin/bench.err
python -c "import json;d=json.load(open('gpurun_out/fin/bench.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
