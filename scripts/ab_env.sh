# A/B of an environment setting on the c2 step: bash scripts/ab_env.sh VAR "v0 v1" [config]
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
C=${3:-c2}
for rep in 1 2; do
  for v in $2; do
    env $1=$v timeout -k 10 200 python -u bench.py --config $C --steps 20 --warmup 3 --no-cpu-baseline > /tmp/ab.json 2> /tmp/ab.err
    python -c "import json;d=json.load(open('/tmp/ab.json'));print('$1=$v', d['ms_per_step'], {k:v['avg_launch_us'] for k,v in d['roofline']['all_kernels'].items()})"
  done
done
