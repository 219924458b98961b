# GPU box: same-box A/B of one env knob on the c2 bench (alternating, 3 pairs) + one timeline without kernel timing
# usage: bash scripts/gpu_ab_env.sh <tag> <VAR> <a> <b>
set -e
TAG=$1; VAR=$2; A=$3; B=$4
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for k in 1 2 3; do
for v in $A $B; do
env $VAR=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-kernel-timing > $OUT/b_$v.json 2> $OUT/b_$v.err
python -c "import json;d=json.load(open('$OUT/b_$v.json'));print('$VAR=$v', d['ms_per_step'])"
done
done
for v in $A $B; do
env $VAR=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_$v -o run -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-kernel-timing > /dev/null 2> $OUT/prof_$v.err
python scripts/step_timeline.py $(find $OUT/prof_$v -name "run_kernel_trace.csv" | head -1) > $OUT/timeline_$v.txt
done
echo done
