#!/usr/bin/env bash
# The N-rank bench paths rehearsed on one GPU (gpurun): every rank on cuda:0, gloo through host
# memory; rank 0 checks the gathered image against a single-rank render (verified.bit_exact).
#   bash scripts/gpu_rehearse.sh TAG   -> gpurun_out/TAG/rehearse_{c5,c2}_n*.json
set -euo pipefail
TAG=${1:-rehearse}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for n in ${RANKS:-2 4 8}; do
    PT_BENCH_REHEARSE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" \
        --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus "$n" --workload c5_8k \
        --steps 3 --warmup 1 --device-warmup-ms 0 > "$OUT/rehearse_c5_n$n.json" 2> "$OUT/rehearse_c5_n$n.err"
    tail -c 300 "$OUT/rehearse_c5_n$n.json"
done
PT_BENCH_REHEARSE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29600 bench.py --gpus 2 \
    --steps 10 --warmup 2 --device-warmup-ms 0 > "$OUT/rehearse_c2_n2.json" 2> "$OUT/rehearse_c2_n2.err"
tail -c 300 "$OUT/rehearse_c2_n2.json"
