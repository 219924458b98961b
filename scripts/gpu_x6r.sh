# GPU box: gemm_x6r with 48-row wave blocks (ABCD_X6R_MR=3) against 32 (default): alone, parity, in the step
set -e
OUT=gpurun_out/x6r
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/gemm_bench.py 2>&1 | grep -v amdgpu.ids > $OUT/gb.log
ABCD_X6R_MR=3 timeout -k 10 200 python -u scripts/gemm_bench.py 2>&1 | grep -v amdgpu.ids >> $OUT/gb.log
cat $OUT/gb.log
ABCD_X6R_MR=3 timeout -k 10 500 python -u -m pytest tests/test_gpu_fullshape.py tests/test_gpu_kernels.py -x -q --timeout 240 --timeout-method thread -k "512 or x6r or gemm" > $OUT/p.log 2>&1 || { tail -30 $OUT/p.log; exit 1; }
tail -1 $OUT/p.log
bash scripts/ab_env.sh ABCD_X6R_MR "2 3" > $OUT/ab.log 2>&1; cat $OUT/ab.log
