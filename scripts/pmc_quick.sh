#!/usr/bin/env bash
# Quick PMC pass over scripts/quick_perf.py (dev tool): VALU/SALU/LDS instruction counts and
# stall cycles of the render kernel.  Usage: scripts/pmc_quick.sh TAG
set -euo pipefail
TAG=${1:-dev}
OUT=$PWD/gpurun_out/pmc/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
CMD=(python3 "$PWD/scripts/quick_perf.py")
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/a" -o run -- "${CMD[@]}" > "$OUT/a.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU_TRANS_F32 --output-format csv -d "$OUT/b" -o run -- "${CMD[@]}" > "$OUT/b.log" 2>&1 || \
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY --output-format csv -d "$OUT/b" -o run -- "${CMD[@]}" > "$OUT/b.log" 2>&1
python3 "$PWD/scripts/pmc_summary.py" "$OUT"
