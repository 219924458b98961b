# GPU box: gemm_wg3b (256-row tiles, ABCD_WG3W=b) correctness map and timing against the 4x2 wg3
set -e
OUT=gpurun_out/wg3b
mkdir -p $OUT
: > $OUT/d.log
for k in 64 2048 16384; do
ABCD_WG3W=b timeout -k 10 120 python -u scripts/wg_debug.py $k 2>&1 | grep -v amdgpu.ids | head -1 >> $OUT/d.log
done
cat $OUT/d.log
timeout -k 10 200 python -u scripts/wg_probe.py 1 1 2>&1 | grep -v amdgpu.ids > $OUT/probe.log
echo "wg3b" >> $OUT/probe.log
ABCD_WG3W=b timeout -k 10 200 python -u scripts/wg_probe.py 1 1 1 2>&1 | grep -v amdgpu.ids >> $OUT/probe.log
cat $OUT/probe.log
