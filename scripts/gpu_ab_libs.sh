# GPU box: same-box A/B of several builds of the library on the c2 bench
# (alternating, 3 rounds), one kernel-trace timeline per build
# usage: bash scripts/gpu_ab_libs.sh <tag> <lib1.so> <lib2.so> [lib3.so ...]   (names inside seq2seq_abcd-vae_amd/)
set -e
TAG=$1; shift
OUT=gpurun_out/$TAG
PKG=$(pwd)/seq2seq_abcd-vae_amd
mkdir -p $OUT
export TMPDIR=/tmp
for k in 1 2 3; do
for v in "$@"; do
ABCD_HIP_LIB=$PKG/$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/b_${v}_$k.json 2> $OUT/b_${v}_$k.err
python -c "import json;d=json.load(open('$OUT/b_${v}_$k.json'));print('$v', d['ms_per_step'], {k:round(v['avg_launch_us']) for k,v in d['roofline']['all_kernels'].items()})"
done
done
for v in "$@"; do
ABCD_HIP_LIB=$PKG/$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$v -o run -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-kernel-timing > /dev/null 2> $OUT/prof_$v.err
python scripts/step_timeline.py $(find $OUT/prof_$v -name "run_kernel_trace.csv" | head -1) > $OUT/timeline_$v.txt
done
echo done
