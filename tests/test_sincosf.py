"""The product's sin/cos (csrc/pt_sincosf.h, compiled here for the host) equals the host libm's
sinf/cosf -- the functions the reference and the oracle call -- on EVERY f32 of the domain the
path tracer uses, a = Randomf3201 * 2*pi in [0, 2*pi] (demofox_path_tracing_scalar.cpp:45).
The device compiles the same header; its double ops (mul, fma) are IEEE on gfx950, so the GPU
result is the same bit pattern (confirmed end-to-end by the bit-exact GPU parity tests)."""
from __future__ import annotations

import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    cxx = shutil.which("g++") or shutil.which("c++")
    if not cxx:
        pytest.skip("no host C++ compiler")
    exe = tmp_path_factory.mktemp("sincos") / "check_sincosf"
    subprocess.run([cxx, "-std=c++17", "-O2", "-ffp-contract=off", str(ROOT / "tests/native/check_sincosf.cpp"),
                    "-o", str(exe), "-lm", "-lpthread"], check=True)
    return exe


def test_sincosf_exhaustive_on_0_2pi(checker):
    out = subprocess.run([str(checker)], check=False, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout + out.stderr
    n = int(out.stdout.split()[1])
    assert n > 1_000_000_000          # every f32 in [0, 2*pi*1.0001]
    assert "mismatches 0" in out.stdout


def test_sincosf_negative_range(checker):
    """Same algorithm for negative arguments (odd/even symmetry through the reduction), -0
    excluded: glibc returns sinf(-0) = -0, the straight-line form +0 (its callers' arguments
    Randomf * 2*pi are never -0; pt_sincosf.h states the domain)."""
    out = subprocess.run([str(checker), "-6.2832", "-1e-45"], check=False, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout
