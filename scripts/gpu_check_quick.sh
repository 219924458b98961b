# GPU box: persistent-kernel + production parity tests, two c2 bench lines, one timeline without kernel timing
set -e
TAG=${1:-q}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_persist.py tests/test_gpu_prod.py tests/test_gpu_trainer.py tests/test_gpu_fullshape.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for k in 1 2; do
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/b$k.json 2> $OUT/b$k.err
python -c "import json;d=json.load(open('$OUT/b$k.json'));print(d['ms_per_step'], d['value'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-kernel-timing > /dev/null 2> $OUT/prof.err
python scripts/step_timeline.py $(find $OUT/prof -name "run_kernel_trace.csv" | head -1) > $OUT/timeline.txt
grep -n "persist_reset\|_persist<\|dec_fwd_x6\|dec_bwd_fold\|enc_bwd_sk" $OUT/timeline.txt | head -10
