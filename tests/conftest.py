"""Shared fixtures.  `-m gpu` tests need a real MI355X and call the product through its C ABI;
everything else runs on CPU (oracle vs golden fixtures, host logic, ABI exports, gloo sharding)."""
from __future__ import annotations

import json
import os
import lzma
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
GOLDEN = ROOT / "tests" / "golden"
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


# The suite's launches rebuild the tile schedule every 64 launches (the library's default is 256,
# pt_capi.cpp kSchedRebuildDefault): the 66-70-launch series of test_gpu_regime / test_gpu_configs /
# test_gpu_v4 / test_gpu_chain then cover a rebuild.  Set before any test initialises the library.
os.environ.setdefault("PT_MI355_SCHED_REBUILD", "64")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD GPU (MI355X, gfx950) and libpt_mi355.so")


@pytest.fixture(scope="session")
def manifest() -> dict:
    return json.loads((GOLDEN / "manifest.json").read_text())


def load_golden(name: str) -> np.ndarray:
    """A golden image (H x W x 3); a case with "rows" holds only rows start::stride of it."""
    m = json.loads((GOLDEN / "manifest.json").read_text())["cases"][name]
    raw = lzma.decompress((GOLDEN / f"{name}.f32.xz").read_bytes())
    nrows = m["rows"]["count"] if "rows" in m else m["height"]
    return np.frombuffer(raw, dtype="<f4").reshape(nrows, m["width"], 3).copy()


GOLDEN_B4 = ["g1_256x256_f1", "g2_256x256_f8", "g3_200x120_f3", "g4_64x64_f32"]
GOLDEN_B8 = ["g5_256x256_f8_b8", "g6_1920x1080_f2_b8", "g7_96x64_f53_b8"]


@pytest.fixture(scope="session")
def golden():
    return load_golden


def bits_equal(a: np.ndarray, b: np.ndarray) -> bool:
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


def mismatch_report(a: np.ndarray, b: np.ndarray) -> str:
    a = np.asarray(a, np.float32).reshape(-1, 3)
    b = np.asarray(b, np.float32).reshape(-1, 3)
    bad = np.nonzero((a.view(np.uint32) != b.view(np.uint32)).any(1))[0]
    if len(bad) == 0:
        return "identical"
    d = np.abs(a[bad].astype(np.float64) - b[bad]).max(1)
    return f"{len(bad)} of {len(a)} pixels differ; first {bad[:5].tolist()}, max |d| {d.max():.3g}"


@pytest.fixture(autouse=True)
def _device_errors_after_gpu_test(request):
    """After every -m gpu test: synchronise the device and read the kernels' error words
    (pt_check_device_errors).  An asynchronous fault is then reported by the test whose work caused it,
    not by whichever later test synchronises first (the round-5 r05z3 illegal address surfaced in the
    test after the pinned work-queue tests), and a launch whose pool or bounds guards fired fails its
    own test even when its image was not compared."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    from cpuperformanceraytracer_amd import _native as N
    if getattr(N, "_lib", None) is None:
        return
    import torch
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    rc = N.load().pt_check_device_errors()
    if rc != N.PT_OK:
        pytest.fail(f"device error words after the test: {N.load().pt_last_error().decode(errors='replace')}")
