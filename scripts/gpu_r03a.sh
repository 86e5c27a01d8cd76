#!/usr/bin/env bash
# Round-3 GPU check (run via gpurun from the repo root): the -m gpu suite, the default bench, the
# configs[4] strong-scaling workload on one GPU, and its N-rank path rehearsed on one GPU.
set -euo pipefail
TAG=${1:-r03a}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
tail -3 "$OUT/gpu_tests.log"
timeout -k 10 300 python bench.py > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err"
tail -c 400 "$OUT/bench_c2.json"
timeout -k 10 300 python bench.py --workload c5_8k --no-cpu-baseline > "$OUT/bench_c5_n1.json" 2> "$OUT/bench_c5_n1.err"
tail -c 300 "$OUT/bench_c5_n1.json"
for n in ${RANKS:-2 4 8}; do
    PT_BENCH_REHEARSE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" \
        --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus "$n" --workload c5_8k \
        --steps 3 --warmup 1 --device-warmup-ms 0 > "$OUT/rehearse_c5_n$n.json" 2> "$OUT/rehearse_c5_n$n.err"
    tail -c 300 "$OUT/rehearse_c5_n$n.json"
done
