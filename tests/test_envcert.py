"""The certified env-texel cells (csrc/pt_envcert.h, both kernels' miss term) against the exact
glibc restatements they fall back to (csrc/pt_invtrig.h): the polynomial angles' intervals hold
atanf_glibc for EVERY f32 q in [2^-40, 2^40] and asinf_glibc for every f32 in [0, 1 - 2^-20]
(exhaustive), the atan2 sign glue holds on random domain pairs, and every certified cell of the v4
random-jitter sampler and of the config-4 nearest sampler equals the exact pipeline's on random unit
directions.  The GPU computes the same bits (f32 add/mul/fma, correctly rounded 1/x, a/b, sqrt), and
the GPU env / v4 parity tests stay bit-exact against the oracle."""
from __future__ import annotations

import re
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def test_envcert_contains_glibc_and_cells_match(tmp_path):
    cxx = shutil.which("g++")
    if not cxx:
        pytest.skip("no g++")
    exe = tmp_path / "check_envcert"
    subprocess.run([cxx, "-std=c++17", "-O2", "-ffp-contract=off", str(ROOT / "tests/native/check_envcert.cpp"),
                    "-o", str(exe), "-lm", "-lpthread"], check=True)
    out = subprocess.run([str(exe), "10000000"], capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stdout
    assert out.stdout.count("violations 0") == 5, out.stdout
    assert "atan checked 671088641" in out.stdout and "asin checked 1065353201" in out.stdout
    rate = float(re.search(r"uniform directions only: fallback_rate (\S+)", out.stdout).group(1))
    assert rate < 1e-3, out.stdout
