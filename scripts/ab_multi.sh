# A/B timing of several experiment-bit settings: bash scripts/ab_multi.sh "0 2 4 8 14" [config]
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
C=${2:-c2}
for rep in 1 2; do
for k in $1; do
  ABCD_EXP=$k timeout -k 10 200 python -u bench.py --config $C --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_$k.json 2>gpurun_out/ab_$k.err
  python -c "import json;d=json.load(open('gpurun_out/ab_$k.json'));print('EXP=$k', d['ms_per_step'], {k:v['avg_launch_us'] for k,v in d['roofline']['all_kernels'].items()})"
done
done
