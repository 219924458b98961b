# GPU box: rocprofv3 kernel stats of the c2 bench step under each environment setting given
# usage: bash scripts/prof_ab.sh "" "ABCD_X6R=0" ...   (summaries: gpurun_out/profab_<k>/)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
k=0
for envs in "$@"; do
  k=$((k + 1))
  OUT=gpurun_out/profab_$k
  mkdir -p $OUT
  env $envs timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing > $OUT/bench.json 2> $OUT/err.log
  echo "== [$envs]"
  python3 scripts/kstats.py $OUT
done
