#!/usr/bin/env bash
# Second PMC pass (dev tool): hardware FLOP counts, lane-cycles, LDS behaviour, instruction fetch.
set -euo pipefail
TAG=${1:-dev}
OUT=$PWD/gpurun_out/pmc/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
CMD=(python3 "$PWD/scripts/quick_perf.py")
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP64 SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_IFETCH SQ_INSTS_BRANCH --output-format csv -d "$OUT/c" -o run -- "${CMD[@]}" > "$OUT/c.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 --output-format csv -d "$OUT/d" -o run -- "${CMD[@]}" > "$OUT/d.log" 2>&1
python3 "$PWD/scripts/pmc_summary.py" "$OUT"
