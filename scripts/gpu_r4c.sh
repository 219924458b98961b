# GPU box: sampler parameter GEMMs on the side stream (ABCD_SAMPSIDE) A/B at c2, then the contention probe.
set -e
OUT=gpurun_out/r4c
mkdir -p $OUT
export TMPDIR=/tmp
bash scripts/ab_env.sh ABCD_SAMPSIDE "0 1" > $OUT/ab_sampside.log 2>&1; cat $OUT/ab_sampside.log
timeout -k 10 300 python -u scripts/contention_probe.py > $OUT/contention_probe.log 2>&1; cat $OUT/contention_probe.log
echo r4c done
