set -e
mkdir -p gpurun_out/wgt
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_persist.py tests/test_gpu_fullshape.py -x -q --timeout 240 --timeout-method thread -k "wgrad or 512" > gpurun_out/wgt/p.log 2>&1 || { tail -30 gpurun_out/wgt/p.log; exit 1; }
tail -1 gpurun_out/wgt/p.log
