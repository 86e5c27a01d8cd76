#!/usr/bin/env bash
# GPU-box profiling of the benchmark command (run via gpurun from the repo root).
#   pass 1: rocprofv3 --kernel-trace --stats  (per-kernel durations)
#   pass 2/3: PMC FETCH_SIZE / WRITE_SIZE in separate passes (HBM traffic, MI355X_MICROARCH.md §HBM)
#   pass 4: SQ instruction/cycle counters (VALU mix)
# Output under gpurun_out/prof/<tag>/ ; scripts/summarize_profile.py turns it into profiles/.
set -euo pipefail
TAG=${1:-r01}
WORKLOAD=${WORKLOAD:-c2_1080p}
STEPS=${STEPS:-10}
OUT=$PWD/gpurun_out/prof/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
# (--no-configs4: the default line's configs[4] leg would add 8K launches of the same kernel instance)
CMD=(python3 "$PWD/bench.py" --workload "$WORKLOAD" --steps "$STEPS" --warmup 2 --no-cpu-baseline --no-configs4)
# The kernel trace runs the bench as it is timed (the diffuse steps chained: consecutive launches
# overlap).  The PMC passes run it with --no-chain: counter collection serialises the
# dispatches, and a chained launch held back behind its successor would make the successor's waves wait
# out their bounded polls; the counters of one launch (instructions, bytes) do not depend on the overlap.
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- "${CMD[@]}" > "$OUT/trace.log" 2>&1
echo "trace done" >> "$OUT/progress"
CMD+=(--no-chain)
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- "${CMD[@]}" > "$OUT/fetch.log" 2>&1
echo "fetch done" >> "$OUT/progress"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- "${CMD[@]}" > "$OUT/write.log" 2>&1
echo "write done" >> "$OUT/progress"
[ "${TRACE_ONLY:-0}" = 1 ] && exit 0
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/sq" -o run -- "${CMD[@]}" > "$OUT/sq.log" 2>&1
echo "sq done" >> "$OUT/progress"
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY --output-format csv -d "$OUT/sq2" -o run -- "${CMD[@]}" > "$OUT/sq2.log" 2>&1 || echo "sq2 pass failed (counter names?)"
echo "sq2 done" >> "$OUT/progress"
# L2 hit / miss of the render kernel's loads (texel gathers vs accumulator, round 4): 2 TCC counters
[ "${TCC:-0}" = 1 ] && { timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/tcc" -o run -- "${CMD[@]}" > "$OUT/tcc.log" 2>&1 || echo "tcc pass failed"; }
find "$OUT" -name '*.csv' | head -50
