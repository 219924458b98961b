# GPU box: enc_bwd_w8 (ABCD_ENCBWD=w8) -- parity at the B=72 fixtures and c2 / c5gru
# full shape, then same-box A/B against enc_bwd_sk, stamps and PMC traffic of w8
set -e
OUT=gpurun_out/w8
mkdir -p $OUT
export TMPDIR=/tmp
ABCD_ENCBWD=w8 timeout -k 10 500 python -u -m pytest tests/test_gpu_prod.py tests/test_gpu_fullshape.py -x -q --timeout 240 --timeout-method thread -k "fused_step or module_surface or c2-512 or c5gru-128" > $OUT/pytest_w8.log 2>&1 || { tail -40 $OUT/pytest_w8.log; exit 1; }
tail -1 $OUT/pytest_w8.log
bash scripts/ab_env.sh ABCD_ENCBWD "sk w8" > $OUT/ab.log 2>&1; cat $OUT/ab.log
bash scripts/ab_env.sh ABCD_ENCBWD "sk w8" c5gru > $OUT/ab_c5gru.log 2>&1; cat $OUT/ab_c5gru.log
ABCD_ENCBWD=w8 timeout -k 10 240 python -u scripts/persist_stamps.py > $OUT/persist_phase_stamps.log 2>&1 || echo "stamps failed"
grep -A5 "^enc_bwd" $OUT/persist_phase_stamps.log || true
ABCD_ENCBWD=w8 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing > /dev/null 2> $OUT/pmc_fetch.err
ABCD_ENCBWD=w8 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing > /dev/null 2> $OUT/pmc_write.err
python scripts/pmc_traffic.py $OUT/pmc_fetch $OUT/pmc_write $OUT/traffic.json > /dev/null
python -c "import json;d=json.load(open('$OUT/traffic.json'));print({k:(round(v['hbm_bytes_per_launch']/1e9,2), round(v['write_bytes']/1e9,2)) for k,v in d['kernels'].items()})"
echo w8 done
