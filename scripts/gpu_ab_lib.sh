# GPU box: same-box A/B of two builds of the library on the c2 bench (alternating, 3 pairs), one
# kernel-trace timeline per build, and (optional) a pytest selection run against build B
# usage: bash scripts/gpu_ab_lib.sh <tag> <libA.so> <libB.so> [pytest -k expression]
# (library file names inside seq2seq_abcd-vae_amd/)
set -e
TAG=$1; A=$2; B=$3; K=$4
OUT=gpurun_out/$TAG
PKG=$(pwd)/seq2seq_abcd-vae_amd
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$K" ]; then
  KS=(); [ "$K" != all ] && KS=(-k "$K")
  ABCD_HIP_LIB=$PKG/$B timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    "${KS[@]}" > $OUT/pytest_B.txt 2>&1
  tail -3 $OUT/pytest_B.txt
fi
for k in 1 2 3; do
for v in $A $B; do
ABCD_HIP_LIB=$PKG/$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/b_${v}_$k.json 2> $OUT/b_${v}_$k.err
python -c "import json;d=json.load(open('$OUT/b_${v}_$k.json'));print('$v', d['ms_per_step'], d.get('kernels', {}) if 0 else '')"
done
done
for v in $A $B; do
ABCD_HIP_LIB=$PKG/$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$v -o run -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-kernel-timing > /dev/null 2> $OUT/prof_$v.err
python scripts/step_timeline.py $(find $OUT/prof_$v -name "run_kernel_trace.csv" | head -1) > $OUT/timeline_$v.txt
done
echo done
