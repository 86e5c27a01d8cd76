"""The closest-sphere stage of both kernels (pt_kernel.hip spheres_closest, pt_v4.hip trace<DEF>)
rests on one geometric claim: for pairwise-disjoint spheres, of the spheres that pass the
reference's early tests (TestSphereTrace, demofox_path_tracing_scalar.cpp:145-184 / v4 :641-695)
the one with the largest b is the only one whose distance can be the accepted minimum.
tests/native/check_sphere_closest.cpp compiles both arithmetic flavours for the host (the
reference's f32 operations, -ffp-contract=off) and compares the stage with the sequential tests on
random rays, rays grazing two neighbouring spheres, origins just off a surface and origins inside a
sphere -- bit for bit.  The GPU parity tests check the kernels on whole images, also with every
candidate forced onto the fallback path."""
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
    exe = tmp_path_factory.mktemp("sphere_closest") / "check_sphere_closest"
    subprocess.run([cxx, "-std=c++17", "-O2", "-ffp-contract=off", str(ROOT / "tests/native/check_sphere_closest.cpp"),
                    "-o", str(exe), "-lm"], check=True)
    return exe


@pytest.mark.parametrize("seed", ["0x9e3779b97f4a7c15", "12345"])
def test_closest_sphere_equals_sequential(checker, seed):
    out = subprocess.run([str(checker), "200000", seed], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-2000:]
    assert "disagreements 0" in out.stdout
    # the interesting case is exercised: rays with more than one sphere past the early tests
    for line in out.stdout.splitlines():
        if line.startswith(("diffuse", "v4")):
            assert int(line.split(">1 candidate")[1].split()[0]) > 10_000, line
