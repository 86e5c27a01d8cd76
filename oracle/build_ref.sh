#!/usr/bin/env bash
# oracle/build_ref.sh -- TEST INFRASTRUCTURE ONLY.
#
# Builds the reference's own scalar path tracer (unmodified, compiled where it lies under
# /root/reference) into oracle/_ref/ so it can (a) generate the golden fixtures in tests/golden
# and (b) serve as the "reference" CPU baseline in bench.py.  Nothing from the reference is
# copied into the repository: the one generated header (a selection of mathlib.h's own scalar
# lines, see below) lives in a temporary directory that is deleted on exit, and only the
# compiled binary/.so land in oracle/_ref/ (git-ignored).
#
# Why a generated header: the reference's full mathlib.h only compiles under MSVC (it overloads
# operators on __m256 and calls SVML).  demofox_path_tracing_scalar.cpp only needs mathlib.h's
# scalar f32xN subset, so we extract exactly those line ranges and add
# `using std::{sqrt,abs,cos,sin,tan};`: MSVC's <cmath> declares the float overloads of these in
# the global namespace, so the reference's unqualified calls on f32 (scalar.cpp:46-48,122,126,
# 169,173,338) are sqrtf/fabsf/cosf/sinf/tanf under MSVC.  libstdc++'s <cmath> only has the double
# versions globally: without the using-declarations GCC binds abs(float) to abs(int) (5 pixels
# differ) and cos/sin/tan to double precision (a different rounding of x, y and
# the camera distance).  The float overloads here resolve to glibc's sinf/cosf/tanf.
# `-I-` stops GCC from searching the reference directory first for "mathlib.h".
#
# Flags: -O2 -ffp-contract=off  (MSVC /fp:precise does not contract a*b+c).
set -euo pipefail
REF=${REF:-/root/reference/CPUPerformanceRayTracer}
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
OUT="$HERE/_ref"
if [ ! -f "$REF/demofox_path_tracing_scalar.cpp" ]; then
    echo "build_ref.sh: reference not present at $REF -- skipping (prebuilt files are used)" >&2
    exit 0
fi
mkdir -p "$OUT"
GEN="$(mktemp -d "${TMPDIR:-/tmp}/ptref.XXXXXX")"
trap 'rm -rf "$GEN"' EXIT
M="$REF/mathlib.h"
{
    echo '#pragma once'
    echo '#include "utils.h"'
    echo '#include <cmath>'
    echo 'using std::sqrt; using std::abs; using std::cos; using std::sin; using std::tan;'
    awk 'NR>=12&&NR<=72' "$M"              # f32x2/3/4 structs + add/sub/mul/div/dot/fmadd
    awk 'NR==415||NR==436||NR==437' "$M"   # (comment) + sroot/rsroot(f32)
    awk 'NR>=582&&NR<=619' "$M"            # scalar operator+ - * /
    awk 'NR>=723&&NR<=726' "$M"            # len(f32xN)
    awk 'NR>=729&&NR<=731' "$M"            # (comments)
    awk 'NR>=749&&NR<=751' "$M"            # normalize(f32xN)
    awk 'NR==763||NR==768' "$M"            # lerp, cross(f32x3)
} > "$GEN/mathlib.h"
CXX=${CXX:-g++}
FLAGS="-std=c++17 -O2 -ffp-contract=off -fPIC -w"
INC="-I$GEN -I- -I$GEN -I$REF"
$CXX $FLAGS $INC -c "$REF/demofox_path_tracing_scalar.cpp" -o "$GEN/scalar.o" 2>/dev/null
$CXX $FLAGS -c "$HERE/ref_driver.cpp" -o "$GEN/drv.o"
$CXX $FLAGS -DREF_DRIVER_MAIN -c "$HERE/ref_driver.cpp" -o "$GEN/drv_main.o"
$CXX -shared -o "$OUT/libref_scalar.so" "$GEN/scalar.o" "$GEN/drv.o" -lm
$CXX -o "$OUT/ref_scalar" "$GEN/scalar.o" "$GEN/drv_main.o" -lm

# --- c_numBounces = 8 (BASELINE configs[1]-[4]) ----------------------------------------------------
# The reference's own line 19 reads `const int c_numBounces = 4; //8`: the value it annotates as the
# alternative.  A temporary copy of the file (in $GEN, deleted on exit, never in the repository) with
# ONLY that constant changed is compiled exactly like the unmodified file.  The script checks that
# the copy differs from the original in that one line and records both sha256s and the diff in
# oracle/_ref/b8_patch.json (make_golden.py copies it into tests/golden/manifest.json).
SRC="$REF/demofox_path_tracing_scalar.cpp"
B8="$GEN/b8"
mkdir -p "$B8"
cp "$REF/demofox_path_tracing_scalar.h" "$B8/"
sed '19s/^const int c_numBounces = 4; \/\/8\r\{0,1\}$/const int c_numBounces = 8; \/\/8/' "$SRC" > "$B8/demofox_path_tracing_scalar.cpp"
NDIFF=$(diff "$SRC" "$B8/demofox_path_tracing_scalar.cpp" | grep -c '^[<>]' || true)
if [ "$NDIFF" != "2" ]; then
    echo "build_ref.sh: c_numBounces patch did not change exactly line 19 ($NDIFF diff lines)" >&2
    exit 1
fi
DIFF_TXT=$(diff "$SRC" "$B8/demofox_path_tracing_scalar.cpp" | tr -d '\r' || true)
python3 - "$SRC" "$B8/demofox_path_tracing_scalar.cpp" "$DIFF_TXT" > "$OUT/b8_patch.json" <<'PY'
import hashlib, json, sys
orig, patched, diff = sys.argv[1], sys.argv[2], sys.argv[3]
h = lambda p: hashlib.sha256(open(p, "rb").read()).hexdigest()
print(json.dumps({"file": "demofox_path_tracing_scalar.cpp", "line": 19,
                  "sha256_original": h(orig), "sha256_patched": h(patched), "diff": diff}, indent=1))
PY
$CXX $FLAGS -I"$GEN" -I- -I"$B8" -I"$GEN" -I"$REF" -c "$B8/demofox_path_tracing_scalar.cpp" -o "$GEN/scalar_b8.o" 2>/dev/null
$CXX -o "$OUT/ref_scalar_b8" "$GEN/scalar_b8.o" "$GEN/drv_main.o" -lm

# --- config 4's miss term: EquirectangularTextureSample's per-lane body --------------------------
# texture.cpp:101-139 is an m256x3 (MSVC __m256) function whose per-lane body, :111-135, is plain
# scalar f32 code on f32x2/f32x3 (+ TexelFetch, :6-14, and struct texture, texture.h:6-12).  Those
# line ranges are extracted into a temporary file and compiled, with the same mathlib.h subset as
# above plus `using std::atan2; using std::asin;` (MSVC's float overloads, as for sqrt/cos above),
# inside ref_env.cpp's per-direction wrapper.  No arithmetic is added.
T="$REF/texture.cpp"
{
    echo '#include "mathlib.h"'
    echo 'using std::atan2; using std::asin;'
    awk 'NR>=6&&NR<=12' "$REF/texture.h"     # struct texture
    awk 'NR>=6&&NR<=14' "$T"                 # TexelFetch
} > "$GEN/ref_texture_fetch.inc"
awk 'NR>=111&&NR<=135' "$T" > "$GEN/ref_env_lane_body.inc"
$CXX $FLAGS -I"$GEN" -I"$HERE" -I"$REF" "$HERE/ref_env.cpp" -o "$OUT/ref_env" -lm
# LoadTexture's decoder (config 4): the reference's vendored stb_image.h, compiled where it lies
$CXX -std=c++17 -O2 -w -I"$REF" "$HERE/ref_hdr.cpp" -o "$OUT/ref_hdr" -lm
# WriteImage's encoder (output stage): the reference's vendored stb_image_write.h, where it lies
$CXX -std=c++17 -O2 -w -I"$REF" "$HERE/ref_bmp.cpp" -o "$OUT/ref_bmp" -lm
echo "build_ref.sh: built $OUT/libref_scalar.so, $OUT/ref_scalar, $OUT/ref_scalar_b8, $OUT/ref_env, $OUT/ref_hdr and $OUT/ref_bmp"
