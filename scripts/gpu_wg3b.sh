# GPU box: gemm_wg3b (ABCD_WG3W=b): wgrad + fullshape parity with it, same-box A/B in the c2 step against the 4x2 wg3
set -e
OUT=gpurun_out/wg3b
mkdir -p $OUT
export TMPDIR=/tmp
ABCD_WG3W=b timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_persist.py -x -q --timeout 240 --timeout-method thread -k "wgrad and not 3w8" > $OUT/pytest_wgrad.log 2>&1 || { tail -40 $OUT/pytest_wgrad.log; exit 1; }
tail -1 $OUT/pytest_wgrad.log
ABCD_WG3W=b timeout -k 10 500 python -u -m pytest tests/test_gpu_fullshape.py -x -q --timeout 240 --timeout-method thread -k "512" > $OUT/pytest_full.log 2>&1 || { tail -40 $OUT/pytest_full.log; exit 1; }
tail -1 $OUT/pytest_full.log
bash scripts/ab_env.sh ABCD_WG3W "2 b" > $OUT/ab.log 2>&1; cat $OUT/ab.log
ABCD_WG3W=b timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/prof.err
grep -h "gemm_wg" $OUT/prof/run_kernel_stats.csv | cut -c1-200 || true
