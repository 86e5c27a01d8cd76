#!/usr/bin/env bash
# Dev tool: build libpt_mi355.so of git revision REV into build/libpt_NAME.so (for A/B runs with
# PT_MI355_LIB; the revision's C ABI must match the working tree's Python side).
#   bash scripts/build_rev.sh REV NAME
set -euo pipefail
REV=$1; NAME=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=/tmp/pt_wt_$NAME
rm -rf "$WT"; git -C "$ROOT" worktree prune
git -C "$ROOT" worktree add -f "$WT" "$REV" > /dev/null
mkdir -p "$ROOT/build"
(cd "$WT" && python3 -c "
import sys; sys.path.insert(0, '.')
from cpuperformanceraytracer_amd import build as b
import subprocess
cmd = [b.hipcc(), f'--offload-arch={b.ARCH}', '-O3', '-std=c++17', '-fPIC', '-shared', *b.PARITY_FLAGS, *b.PERF_FLAGS,
       f'-I{b.ROOT / \"include\"}', f'-I{b.CSRC}', '-Wno-unused-function', *[str(b.CSRC / s) for s in b.SOURCES],
       '-o', '$ROOT/build/libpt_$NAME.so']
subprocess.run(cmd, check=True)
")
git -C "$ROOT" worktree remove --force "$WT"
ls -la "$ROOT/build/libpt_$NAME.so"
