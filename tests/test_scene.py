"""The kernel's compile-time scene (DemofoxScene in csrc/pt_scene.h) equals the host-built scene
(pt_build_demofox_scene, the reference's TestSceneTrace constants through the reference's own f32
operations) bit for bit -- including the quad normals written out as literals."""
from __future__ import annotations

import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def test_constexpr_scene_matches_host_scene(tmp_path):
    cxx = shutil.which("g++")
    if not cxx:
        pytest.skip("no g++")
    exe = tmp_path / "check_scene"
    subprocess.run([cxx, "-std=c++17", "-O2", "-ffp-contract=off", str(ROOT / "tests/native/check_scene.cpp"),
                    str(ROOT / "cpuperformanceraytracer_amd/csrc/pt_scene.cpp"), "-o", str(exe), "-lm"], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout
