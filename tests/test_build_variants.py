"""The compile-time variants the kernels keep (diagnostic and test builds) still compile for gfx950
(hipcc, device code only -- no GPU needed), so they cannot rot:

  PT_DIAG=1 / PT_DIAG=2 (+ PT_DIAG_WAVES_ONLY, PT_DIAG_NOATOMIC)   per-wave / per-tile timelines,
                                    per-phase cycle counters (scripts/diag_timeline.py), and the C ABI
                                    side that dumps them (pt_capi.cpp)
  PT_SPHERE_FORCE_SEQ=1, PT_V4_SPHERE_FORCE_SEQ=1   every closest-sphere candidate takes the
                                    sequential fallback (the fallback's own parity run)
  PT_EC_FORCE_EXACT=1               every env texel cell takes the exact inverse-trig fallback
                                    (pt_envcert.h; the fallback's own parity run)
  PT_AMBIENT_WAVES=4, PT_V4_WAVES=5  occupancy A/B builds
  PT_RING_MIN=9                     every MULTI launch on the ring pool (its parity run: all 130 GPU
                                    tests bit-exact, profiles/r03x_gpu_tests.txt)
  PT_CHECKED=1                      the bounds-guarded build (pt_guard.h; build.build_checked)
Every other alternate measured slower was removed from the sources (DESIGN.md records the numbers).
"""
from __future__ import annotations

import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "cpuperformanceraytracer_amd" / "csrc"

VARIANTS = [
    ("pt_kernel.hip", ["PT_DIAG=1"]),
    ("pt_kernel.hip", ["PT_DIAG=2"]),
    ("pt_kernel.hip", ["PT_DIAG=1", "PT_DIAG_WAVES_ONLY=1", "PT_DIAG_NOATOMIC=1"]),
    ("pt_kernel.hip", ["PT_SPHERE_FORCE_SEQ=1"]),
    ("pt_kernel.hip", ["PT_AMBIENT_WAVES=4"]),
    ("pt_v4.hip", ["PT_V4_SPHERE_FORCE_SEQ=1"]),
    ("pt_v4.hip", ["PT_V4_WAVES=5"]),
    ("pt_kernel.hip", ["PT_EC_FORCE_EXACT=1"]),
    ("pt_kernel.hip", ["PT_RING_MIN=9"]),
    ("pt_v4.hip", ["PT_EC_FORCE_EXACT=1"]),
    ("pt_capi.cpp", ["PT_DIAG=1"]),
    ("pt_kernel.hip", ["PT_CHECKED=1"]),
    ("pt_v4.hip", ["PT_CHECKED=1"]),
]


def _compile(src: str, defines: list[str], out: Path) -> subprocess.CompletedProcess:
    from cpuperformanceraytracer_amd.build import PARITY_FLAGS, PERF_FLAGS, hipcc
    cmd = [hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", *PARITY_FLAGS, *PERF_FLAGS,
           f"-I{ROOT / 'include'}", f"-I{CSRC}", "-Wno-unused-function", *[f"-D{d}" for d in defines], "-c",
           str(CSRC / src), "-o", str(out)]
    if src.endswith(".hip"):
        cmd.insert(1, "--cuda-device-only")
    return subprocess.run(cmd, capture_output=True, text=True, timeout=600)


def test_kept_variants_compile(tmp_path):
    if not (shutil.which("hipcc") or Path("/opt/rocm/bin/hipcc").exists()):
        pytest.skip("hipcc not available")
    with ThreadPoolExecutor(max_workers=4) as ex:
        futs = [ex.submit(_compile, src, d, tmp_path / f"v{i}.o") for i, (src, d) in enumerate(VARIANTS)]
        results = [f.result() for f in futs]
    bad = [(VARIANTS[i], r.stderr[-2000:]) for i, r in enumerate(results) if r.returncode != 0]
    assert not bad, bad


def test_no_removed_alternates_left():
    """The measured-slower switches are gone from the product sources (one code path each)."""
    removed = ["PT_AXIS_FROM_LDS", "PT_TRACE_UNROLL", "PT_AXIS_ASM", "PT_AXIS_EARLY", "PT_FLIP_FOLD", "PT_QUAD_CULL",
               "PT_ENV_CULL", "PT_CULL_SPHERES_FIRST", "PT_SPHERE_CLOSEST", "PT_SKY_SKIP", "PT_PRIO", "PT_CHUNK",
               "PT_OWN_LAST", "PT_PIXEL_MAJOR", "PT_AMBIENT_BLOCK_WAVES", "PT_ENV_DEFER", "PT_UNIT_COST",
               "PT_V4_BLOCK_WAVES", "PT_V4_CHUNK", "PT_V4_ENV_DEFER", "PT_V4_PIXEL_MAJOR", "PT_V4_ENV_Q",
               "PT_V4_IEEE_DIV", "PT_V4_SPHERE_CLOSEST", "PT_V4_SPHERE_ORDER", "PT_V4_UNIFIED_DIR",
               "PT_V4_SKY_SKIP", "PT_V4_FORCE_GENERIC", "PT_SQRT_MARKSTEIN", "PT_SCHED_REBUILD", "PT_RING_PM",
               "PT_RING_ANY", "PT_RING_FOLDK", "PT_X_ENV_AMB", "PT_X_ENV_SPHC", "PT_V4_T_NOENV", "PT_V4_T_NOTRIG",
               "PT_V4_T_FLAGS", "PT_V4_CT_DFL_WAVES", "PT_CT_SLOT_ALIAS"]
    import re
    for f in list(CSRC.glob("*.hip")) + list(CSRC.glob("*.h")) + list(CSRC.glob("*.cpp")):
        text = f.read_text()
        for name in removed:
            assert not re.search(rf"\b{name}\b", text), (f.name, name)
