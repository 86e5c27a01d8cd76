"""GPU check of the kernel's fast correctly-rounded f32 reciprocal / division / square root
(csrc/pt_exactmath.h) against the compiler's IEEE sequences: exhaustive for rcp_rn (all 2^32
bit patterns in range) and sqrt_rn (all 2^31 non-negative patterns in range), 3 x 2^32
pseudo-random operand pairs for div_rn.  Built with the product's parity flags."""
from __future__ import annotations

import subprocess
from pathlib import Path

import pytest

from cpuperformanceraytracer_amd.build import ARCH, PARITY_FLAGS, hipcc

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def test_exactmath_probe(tmp_path):
    exe = tmp_path / "exactmath_probe"
    subprocess.run([hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", *PARITY_FLAGS,
                    str(ROOT / "tests/native/exactmath_probe.hip"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    print(out.stdout)
    assert out.returncode == 0, out.stdout + out.stderr
    lines = [l for l in out.stdout.splitlines() if "checked=" in l]
    assert len(lines) == 5
    for l in lines:
        checked = int(l.split("checked=")[1].split()[0])
        assert checked > 1_000_000_000, l
        assert l.endswith("mismatches=0"), l
