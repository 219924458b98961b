# same-box A/B over several environment settings of the c2 step (two rounds):
# bash scripts/ab_multi.sh "VAR=a" "VAR=b OTHER=c" ...
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for setting in "$@"; do
    env $setting timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > /tmp/ab.json 2> /tmp/ab.err
    python -c "import json;d=json.load(open('/tmp/ab.json'));print('$setting', d['ms_per_step'], {k:v['avg_launch_us'] for k,v in d['roofline']['all_kernels'].items()})"
  done
done
