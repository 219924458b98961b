# GPU box: the whole -m gpu suite, the c2 bench line, the persistent-kernel phase stamps
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err
python -c "import json;d=json.load(open('gpurun_out/bench.json'));print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['parity']['recon_loss_rel_delta'], d['parity']['argmax_equal'])"
timeout -k 10 240 python -u scripts/persist_stamps.py > gpurun_out/persist_phase_stamps.log 2>&1
echo stamps done
if [ $# -gt 0 ]; then bash scripts/ab_multi.sh "$@"; fi
