set -e
mkdir -p gpurun_out/wgdebug
: > gpurun_out/wgdebug/d.log
for k in 2048 16384; do
timeout -k 10 120 python -u scripts/wg_debug.py $k 2>&1 | grep -v amdgpu.ids | head -1 >> gpurun_out/wgdebug/d.log
done
cat gpurun_out/wgdebug/d.log
bash scripts/gpu_wgdiag.sh
