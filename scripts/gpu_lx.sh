# GPU box: XCD-local decoder-BPTT exchange (ABCD_LX): parity at c2 full shape and the
# B=72 fixtures, then same-box A/B of the c2 bench and the PMC traffic of both arms
set -e
OUT=gpurun_out/lx
mkdir -p $OUT
export TMPDIR=/tmp
ABCD_LX=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_fullshape.py tests/test_gpu_prod.py tests/test_gpu_trainer.py -x -q --timeout 200 --timeout-method thread -k "c2 or lstm_k128 or gru or plain_checkpoint" > $OUT/pytest_lx.log 2>&1 || { tail -30 $OUT/pytest_lx.log; exit 1; }
tail -2 $OUT/pytest_lx.log
bash scripts/ab_env.sh ABCD_LX "0 1" > $OUT/ab.log 2>&1; cat $OUT/ab.log
for v in 0 1; do
ABCD_LX=$v timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_$v -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing > /dev/null 2> $OUT/pmc_fetch_$v.err
ABCD_LX=$v timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write_$v -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing > /dev/null 2> $OUT/pmc_write_$v.err
python scripts/pmc_traffic.py $OUT/pmc_fetch_$v $OUT/pmc_write_$v $OUT/traffic_$v.json
done
echo lx done
