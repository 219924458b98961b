# GPU box: gemm_wg3 wave forms in the c2 step (ABCD_WG3W: 8 = 8x1, 2 = 4x2 default), fullshape parity
set -e
OUT=gpurun_out/wg3ab
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_fullshape.py -x -q --timeout 240 --timeout-method thread -k "512" > $OUT/pytest_full.log 2>&1 || { tail -40 $OUT/pytest_full.log; exit 1; }
tail -1 $OUT/pytest_full.log
bash scripts/ab_env.sh ABCD_WG3W "8 2" > $OUT/ab.log 2>&1; cat $OUT/ab.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/prof.err
grep -h "gemm_wg" $OUT/prof/run_kernel_stats.csv | cut -c1-200 || true
