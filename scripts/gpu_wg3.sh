# GPU box: gemm_wg3 (pre-split planes, transposed LDS reads, 8 waves) parity and same-box A/B against gemm_wg2
set -e
OUT=gpurun_out/wg3
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_persist.py -x -q --timeout 240 --timeout-method thread -k "wgrad" > $OUT/pytest_wgrad.log 2>&1 || { tail -40 $OUT/pytest_wgrad.log; exit 1; }
tail -1 $OUT/pytest_wgrad.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_fullshape.py -x -q --timeout 240 --timeout-method thread -k "512" > $OUT/pytest_full.log 2>&1 || { tail -40 $OUT/pytest_full.log; exit 1; }
tail -1 $OUT/pytest_full.log
bash scripts/ab_env.sh ABCD_WG3 "0 1" > $OUT/ab.log 2>&1; cat $OUT/ab.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/prof.err
python scripts/step_timeline.py $(find $OUT/prof -name "run_kernel_trace.csv" | head -1) > $OUT/timeline.txt
grep -h "gemm_wg" $OUT/prof/run_kernel_stats.csv | cut -c1-200 || true
tail -30 $OUT/timeline.txt | cut -c1-110
echo wg3 done
