# GPU box, end of a round, in two parts (each fits one gpurun call):
#   part 1: the whole -m gpu suite, smoke(), the bench lines of every config,
#           rocprofv3 kernel stats of c2 and a one-step kernel timeline
#   part 2: PMC traffic + MFMA passes (c2 / c5 / c5gru), phase stamps, contention probe
# usage: bash scripts/gpu_final.sh <tag> [1|2]      (outputs under gpurun_out/<tag>/)
set -e
TAG=${1:-final}
PART=${2:-1}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$PART" = "1" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
  tail -1 $OUT/smoke.log
  for c in c2 c4 c5 c5gru; do
    timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 3 > $OUT/bench_$c.json 2> $OUT/bench_$c.err
    echo "bench $c done"
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2 -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_prof_c2.json 2> $OUT/prof_c2.err
  python scripts/step_timeline.py $(find $OUT/prof_c2 -name "run_kernel_trace.csv" | head -1) > $OUT/step_timeline_c2.txt
  python scripts/queue_gaps.py $(find $OUT/prof_c2 -name "run_kernel_trace.csv" | head -1) > $OUT/queue_gaps_c2.txt
  echo "part 1 done"
else
  # PMC: HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) and MFMA utilisation, per config
  for c in c2 c4 c5 c5gru; do
    timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_$c -o run -- python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing > /dev/null 2> $OUT/pmc_fetch_$c.err
    timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write_$c -o run -- python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing > /dev/null 2> $OUT/pmc_write_$c.err
    python scripts/pmc_traffic.py $OUT/pmc_fetch_$c $OUT/pmc_write_$c $OUT/traffic_$c.json $c > /dev/null
    bash scripts/gpu_pmc_mfma.sh $OUT/mfma_$c $c > $OUT/mfma_$c.log 2>&1
    cp $OUT/mfma_$c/pmc_mfma.json $OUT/pmc_mfma_$c.json
    echo "pmc $c done"
  done
  timeout -k 10 240 python -u scripts/persist_stamps.py > $OUT/persist_phase_stamps.log 2>&1
  timeout -k 10 240 python -u scripts/persist_stamps.py c5 > $OUT/persist_phase_stamps_c5.log 2>&1
  timeout -k 10 300 python -u scripts/contention_probe.py > $OUT/contention_probe.log 2>&1
  echo "part 2 done"
fi
