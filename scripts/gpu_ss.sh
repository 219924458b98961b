# GPU box: the sampler's parameter GEMMs on a stream of their own (ABCD_SAMPSIDE=1): timeline + same-box A/B
set -e
OUT=gpurun_out/ss
mkdir -p $OUT
export TMPDIR=/tmp
ABCD_SAMPSIDE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-kernel-timing > $OUT/b.json 2> $OUT/prof.err
python scripts/step_timeline.py $(find $OUT/prof -name "run_kernel_trace.csv" | head -1) > $OUT/timeline.txt
grep -n "samp_head_bwd\|enc_bwd\|gemm_ks\|persist_reset\|gemm_wg3\|sq_pass1" $OUT/timeline.txt | cut -c1-110 | tail -14
bash scripts/ab_env.sh ABCD_SAMPSIDE "0 1" > $OUT/ab.log 2>&1; cat $OUT/ab.log
