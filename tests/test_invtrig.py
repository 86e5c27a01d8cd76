"""The product's atan2f / asinf (csrc/pt_invtrig.h, compiled here for the host) equal the host libm
-- what the reference's EquirectangularTextureSample calls (texture.cpp:112) -- on every f32 of
asinf's domain, every non-negative f32 for atanf, and 2e8 random atan2f pairs.  The device build
runs the same f32 operations with IEEE '/' and sqrt (bit-exact GPU env-map tests)."""
from __future__ import annotations

import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def test_invtrig_matches_host_libm(tmp_path):
    cxx = shutil.which("g++")
    if not cxx:
        pytest.skip("no g++")
    exe = tmp_path / "check_invtrig"
    subprocess.run([cxx, "-std=c++17", "-O2", "-ffp-contract=off", str(ROOT / "tests/native/check_invtrig.cpp"),
                    "-o", str(exe), "-lm", "-lpthread"], check=True)
    out = subprocess.run([str(exe), "100000000"], capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stdout
    assert out.stdout.count("mismatches 0") == 3
