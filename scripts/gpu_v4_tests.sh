mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_v4.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_v4.log 2>&1
rc=$?
tail -30 gpurun_out/gpu_v4.log
exit $rc
