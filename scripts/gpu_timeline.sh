# GPU box: c2 bench twice + one rocprofv3 kernel trace -> one step's timeline
# usage: bash scripts/gpu_timeline.sh <tag>   (outputs under gpurun_out/<tag>/)
set -e
TAG=${1:-tl}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for k in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bq$k.json 2> $OUT/bq$k.err
  python -c "import json;d=json.load(open('$OUT/bq$k.json'));print(d['ms_per_step'], {k:v['avg_launch_us'] for k,v in d['roofline']['all_kernels'].items()})"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/prof.err
python scripts/step_timeline.py $(find $OUT/prof -name "run_kernel_trace.csv" | head -1) > $OUT/timeline.txt
echo timeline done
