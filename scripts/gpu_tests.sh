#!/usr/bin/env bash
# The -m gpu suite on the GPU box (run via gpurun from the repo root): gpurun_out/<tag>/gpu_tests.log
set -euo pipefail
TAG=${1:-gpu}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf "$@" > "$OUT/gpu_tests.log" 2>&1 || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -3 "$OUT/gpu_tests.log"
