# GPU box: the -m gpu suite on the current defaults, then the dec_bwd_w16 P1 sub-phase stamps
# (a library built with -DABCD_STAMP_DIAG) and a c2 bench line
set -e
OUT=gpurun_out/r4b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error" $OUT/pytest_gpu.log | head -20; tail -3 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
ABCD_STAMP_DIAG=1 ABCD_HIP_LIB=$PWD/seq2seq_abcd-vae_amd/libabcd_diag.so timeout -k 10 240 python -u scripts/persist_stamps.py > $OUT/stamps_diag.log 2>&1
grep -A12 "^dec_bwd" $OUT/stamps_diag.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $OUT/bench_c2.json 2> $OUT/bench_c2.err
python -c "import json;d=json.load(open('$OUT/bench_c2.json'));print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], {k:v['avg_launch_us'] for k,v in d['roofline']['all_kernels'].items()})"
