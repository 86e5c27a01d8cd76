"""The product's glibc restatements (csrc/pt_libmf.h, compiled here for the host) equal the host
libm's expf / powf -- what the oracle calls where the reference calls SVML exp_ps / pow_ps under
USE_FAST_APPROXIMATE_EXP 0 / USE_FAST_APPROXIMATE_GAMMA 0 (global_preprocessor_flags.h:62,64).
The device compiles the same header; its double ops (mul, add, fma) are IEEE on gfx950, so the GPU
gives the same bits (confirmed end-to-end by tests/test_gpu_flags.py)."""
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
    exe = tmp_path_factory.mktemp("libmf") / "check_libmf"
    subprocess.run([cxx, "-std=c++17", "-O2", "-ffp-contract=off", str(ROOT / "tests/native/check_libmf.cpp"),
                    "-o", str(exe), "-lm", "-lpthread"], check=True)
    return exe


@pytest.mark.parametrize("args,minimum", [(["exp"], 1 << 32), (["pow_gamma"], 75_000_000),
                                          (["pow_random", "20000000"], 9_000_000)])
def test_libm_restatement(checker, args, minimum):
    out = subprocess.run([str(checker), *args], check=False, capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stdout + out.stderr
    assert int(out.stdout.split()[1]) >= minimum
    assert "mismatches 0" in out.stdout
