set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_v4.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_v4.log 2>&1 || { tail -30 gpurun_out/gpu_v4.log; exit 1; }
tail -2 gpurun_out/gpu_v4.log
rm -f gpurun_out/ab_v4.jsonl
bash scripts/ab_v4.sh gpurun_out/ab_v4.jsonl "1920 1080 8 8 equirect" default default
bash scripts/ab_v4.sh gpurun_out/ab_v4.jsonl "1920 1080 8 8 none" default
cut -c1-160 gpurun_out/ab_v4.jsonl
