#!/usr/bin/env bash
# Round 5, first GPU call: the bench-regime / grid-alternation parity tests, then the 2-rank c2
# rehearsal (PT_MI355_CT_WAVES=0, default device warm-up: the round-4 failing condition) twice.
#   bash scripts/gpu_r05a.sh TAG   -> gpurun_out/TAG/
set -euo pipefail
TAG=${1:-r05a}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_regime.py tests/test_gpu_output.py "tests/test_gpu_configs.py::test_ct_occupancy_variants_match_oracle" \
    > "$OUT/tests.log" 2>&1
tail -3 "$OUT/tests.log"
timeout -k 10 300 python bench.py --cpu-seconds 2 > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err"
tail -c 600 "$OUT/bench_c2.json"
for i in 1 2; do
    PT_MI355_CT_WAVES=0 PT_BENCH_REHEARSE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29600 + i)) bench.py --gpus 2 \
        --no-cpu-baseline > "$OUT/reh0_$i.json" 2> "$OUT/reh0_$i.err"
    tail -c 400 "$OUT/reh0_$i.json"
done
