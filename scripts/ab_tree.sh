# A/B of the c2 step: the tree under _ab/ (an older commit, built) against this one, alternating
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
for k in 1 2; do
  for t in _ab .; do
    (cd $t && timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > /tmp/ab.json 2> /tmp/ab.err)
    python -c "import json;d=json.load(open('/tmp/ab.json'));print('$t', d['ms_per_step'], {k:v['avg_launch_us'] for k,v in d['roofline']['all_kernels'].items()})"
  done
done
