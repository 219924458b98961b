# Same-box A/B of library builds on the c2 step: bash scripts/ab_libs.sh lib1.so lib2.so ...
# (each run loads its library through ABCD_HIP_LIB; two alternating rounds)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
for k in 1 2; do
  for lib in "$@"; do
    ABCD_HIP_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > /tmp/ab.json 2> /tmp/ab.err
    python -c "import json;d=json.load(open('/tmp/ab.json'));print('$lib', d['ms_per_step'], {k:v['avg_launch_us'] for k,v in d['roofline']['all_kernels'].items()})"
  done
done
