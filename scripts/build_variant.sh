#!/usr/bin/env bash
# Dev tool: build the working tree's libpt_mi355.so with extra -D defines into build/libpt_NAME.so
# (test / A/B builds loaded with PT_MI355_LIB):  bash scripts/build_variant.sh NAME -DX=1 ...
set -euo pipefail
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/build"
cd "$ROOT" && python3 -c "
import sys, subprocess
from cpuperformanceraytracer_amd import build as b
cmd = [b.hipcc(), f'--offload-arch={b.ARCH}', '-O3', '-std=c++17', '-fPIC', '-shared', *b.PARITY_FLAGS, *b.PERF_FLAGS,
       f'-I{b.ROOT / \"include\"}', f'-I{b.CSRC}', '-Wno-unused-function', *sys.argv[1:], *[str(b.CSRC / s) for s in b.SOURCES],
       '-o', '$ROOT/build/libpt_$NAME.so']
subprocess.run(cmd, check=True)
" "$@"
ls -la "$ROOT/build/libpt_$NAME.so"
