# A/B timing of an experiment bit: bash scripts/ab_exp.sh <bits> [config]
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
C=${2:-c2}
for k in 0 $1 0 $1; do
  ABCD_EXP=$k timeout -k 10 200 python -u bench.py --config $C --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_$k.json 2>gpurun_out/ab_$k.err
  python -c "import json;d=json.load(open('gpurun_out/ab_$k.json'));print('EXP=$k', d['ms_per_step'], {k:v['avg_launch_us'] for k,v in d['roofline']['all_kernels'].items()})"
done
