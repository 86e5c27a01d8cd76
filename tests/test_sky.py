"""The diffuse kernel's sky test (csrc/pt_kernel.hip sky_ray): a tile whose camera rays all have
|D.x| > 0.51 D.z or |D.y| > 0.51 D.z skips their TestSceneTrace and takes the reference's miss.
tests/native/check_sky.cpp checks the predicate against the oracle's TestSceneTrace
(demofox_path_tracing_scalar.cpp:186-287) on every camera ray of four images and on dense direction
grids across both thresholds: no sky direction hits, and the steepest direction that hits stays
below the threshold (0.504, the floor's and ceiling's x extent at the box's front edge).  The v4
kernel's test (pt_v4.hip sky_ray_v4, InitializeScene seen from (0, 0, 40)) is checked the same way
against the v4 oracle's TestSceneTrace, with jittered camera rays and slope grids around each
threshold."""
from __future__ import annotations

import re
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def test_sky_rays_miss_everything(tmp_path):
    cxx = shutil.which("g++") or shutil.which("c++")
    if not cxx:
        pytest.skip("no host C++ compiler")
    lib = ROOT / "oracle" / "liboracle.so"
    if not lib.exists():
        subprocess.run(["make", "-C", str(ROOT / "oracle"), "-s", "liboracle.so"], check=True)
    exe = tmp_path / "check_sky"
    subprocess.run([cxx, "-std=c++17", "-O2", "-ffp-contract=off", str(ROOT / "tests/native/check_sky.cpp"), "-o",
                    str(exe), f"-L{ROOT / 'oracle'}", "-loracle", f"-Wl,-rpath,{ROOT / 'oracle'}", "-lm"], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-2000:]
    m = re.search(r"classified sky (\d+)\s+sky rays that hit (\d+)\s+largest hitting slope ([0-9.]+)", out.stdout)
    assert m and int(m.group(1)) > 10_000_000 and int(m.group(2)) == 0 and float(m.group(3)) < 0.505, out.stdout
    # the v4 kernel's test (pt_v4.hip sky_ray_v4) against the v4 oracle's TestSceneTrace
    m = re.search(r"v4 directions \d+\s+classified sky (\d+)\s+sky rays that hit (\d+)", out.stdout)
    assert m and int(m.group(1)) > 5_000_000 and int(m.group(2)) == 0, out.stdout
