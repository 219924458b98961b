# GPU box: bench lines of every config, rocprofv3 kernel stats of c2, PMC traffic + MFMA passes of c2 / c5 / c5gru.
# usage: bash scripts/gpu_profile.sh <tag>     (outputs under gpurun_out/<tag>/)
set -e
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for c in c2 c4 c5 c5gru; do
  timeout -k 10 400 python -u bench.py --config $c --steps 20 --warmup 3 > $OUT/bench_$c.json 2> $OUT/bench_$c.err
  echo "bench $c done"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2 -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_prof_c2.json 2> $OUT/prof_c2.err
echo "rocprof c2 done"
# PMC: HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) and MFMA utilisation, per config
for c in c2 c5 c5gru; do
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_$c -o run -- python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing > /dev/null 2> $OUT/pmc_fetch_$c.err
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write_$c -o run -- python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing > /dev/null 2> $OUT/pmc_write_$c.err
  python scripts/pmc_traffic.py $OUT/pmc_fetch_$c $OUT/pmc_write_$c $OUT/traffic_$c.json $c > /dev/null
  bash scripts/gpu_pmc_mfma.sh $OUT/mfma_$c $c > $OUT/mfma_$c.log 2>&1 && cp $OUT/mfma_$c/pmc_mfma.json $OUT/pmc_mfma_$c.json
  echo "pmc $c done"
done
cp $OUT/traffic_c2.json $OUT/traffic.json && cp $OUT/pmc_mfma_c2.json $OUT/pmc_mfma.json
