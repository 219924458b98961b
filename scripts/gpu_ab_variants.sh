# GPU box: same-box A/B of library builds and environment settings on the c2 bench
# (alternating, 3 rounds), one kernel-trace timeline per variant
# usage: bash scripts/gpu_ab_variants.sh <tag> <name>=<lib.so>[,VAR=VAL...] ...   (libs inside seq2seq_abcd-vae_amd/)
set -e
TAG=$1; shift
OUT=gpurun_out/$TAG
PKG=$(pwd)/seq2seq_abcd-vae_amd
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name spec cmd...
  local name=$1 spec=$2; shift 2
  local lib=${spec%%,*} envs=""
  [ "$lib" != "$spec" ] && envs=${spec#*,}
  env ABCD_HIP_LIB=$PKG/$lib ${envs//,/ } "$@"
}
for k in 1 2 3; do
for v in "$@"; do
name=${v%%=*}; spec=${v#*=}
run $name $spec timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/b_${name}_$k.json 2> $OUT/b_${name}_$k.err
python -c "import json;d=json.load(open('$OUT/b_${name}_$k.json'));print('$name', d['ms_per_step'], {k:round(v['avg_launch_us']) for k,v in d['roofline']['all_kernels'].items()})"
done
done
for v in "$@"; do
name=${v%%=*}; spec=${v#*=}; lib=${spec%%,*}; envs=""; [ "$lib" != "$spec" ] && envs=${spec#*,}
export ABCD_HIP_LIB=$PKG/$lib
for e in ${envs//,/ }; do export "$e"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$name -o run -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-kernel-timing > /dev/null 2> $OUT/prof_$name.err
for e in ${envs//,/ }; do unset "${e%%=*}"; done
python scripts/step_timeline.py $(find $OUT/prof_$name -name "run_kernel_trace.csv" | head -1) > $OUT/timeline_$name.txt
done
echo done
