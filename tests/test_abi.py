"""The drop-in boundary: libpt_mi355.so builds for gfx950, loads, and exports every symbol the
public headers declare -- the C ABI (include/pt_mi355.h) and the reference-named C++ entry points
(include/demofox_path_tracing_mi355.h).  Without a GPU the product must fail loudly (no CPU
fallback); no compute call is made here."""
from __future__ import annotations

import ctypes
import re
import shutil
import subprocess
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def lib_path():
    from cpuperformanceraytracer_amd import build
    try:
        return build.build_lib()
    except (RuntimeError, subprocess.CalledProcessError) as e:   # pragma: no cover - toolchain missing
        pytest.skip(f"cannot build libpt_mi355.so: {e}")


def header_functions() -> set[str]:
    text = (ROOT / "include" / "pt_mi355.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return set(re.findall(r"^\s*(?:int|int32_t|void|uint32_t|const char\*|pt_work_queue\*)\s+(pt_\w+)\s*\(", text,
                          flags=re.M))


def test_header_declares_the_abi():
    from cpuperformanceraytracer_amd._native import EXPORTED_SYMBOLS
    assert header_functions() == set(EXPORTED_SYMBOLS)


def test_every_declared_symbol_is_exported(lib_path):
    L = ctypes.CDLL(str(lib_path))
    for name in header_functions():
        assert hasattr(L, name), name


def test_reference_named_cpp_entry_points_exported(lib_path):
    nm = shutil.which("nm")
    if not nm:
        pytest.skip("nm not available")
    out = subprocess.run([nm, "-D", "-C", "--defined-only", str(lib_path)], capture_output=True, text=True,
                         check=True).stdout
    for sig in ("DemofoxRenderScalar(float*, int, int, int)",
                "DemofoxRenderSimd(float*, int, int, int)",
                "DemofoxRenderSimdTiled(float*, int, int, int, int, int, int, int)",
                "RenderTile(RenderBufferInfo&, RenderTileInfo&)"):
        assert sig in out, sig


def test_gfx950_code_object_embedded(lib_path):
    data = lib_path.read_bytes()
    assert b"gfx950" in data
    assert b"pt_render_kernel" in data


def test_no_gpu_fails_loudly(lib_path):
    """On a machine without a GPU every render returns an error -- never a silent CPU result."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from cpuperformanceraytracer_amd import _native
    L = _native.load()
    buf = np.zeros((4, 8, 3), np.float32)
    rc = L.pt_render_scalar(buf.ctypes.data, 8, 4, 3)
    assert rc == _native.PT_EHIP
    assert b"device" in L.pt_last_error()
    assert not buf.any()
    import cpuperformanceraytracer_amd as pt
    with pytest.raises(_native.PtError):
        pt.DemofoxRenderScalar(buf, 8, 4, 3)


def test_image_side_limit(lib_path):
    """mainImage's pixel coordinates are f32: sides above 2^24 are rejected before any GPU work."""
    from cpuperformanceraytracer_amd import _native
    L = _native.load()
    buf = np.zeros(8, np.float32)   # never touched: the size check fails first
    rc = L.pt_render_scalar(buf.ctypes.data, (1 << 24) + 8, 1, 3)
    assert rc == _native.PT_EINVAL
    assert b"2^24" in L.pt_last_error()


def test_struct_layouts_match_header():
    """ctypes mirrors of the POD structs have the C sizes the header implies."""
    from cpuperformanceraytracer_amd import _native as N
    assert ctypes.sizeof(N.PtConfig) == 4 * 4 + 3 * 4 + 4 + 4 * N.PT_MAX_DEVICES
    assert ctypes.sizeof(N.PtV4Config) == 9 * 4
    assert ctypes.sizeof(N.PtBufferInfo) == 8 + 3 * 4 + 4      # pointer + 3 ints (+ tail pad)
    assert ctypes.sizeof(N.PtTileInfo) == 8 * 4
    assert ctypes.sizeof(N.PtDeviceJob) == 8 + 9 * 4 + 4
    assert ctypes.sizeof(N.PtWorkCounts) == 8 * 8


def test_reference_shaped_host_compiles_and_links(tmp_path):
    """examples/reference_host.cpp uses only the reference's names (demofox_path_tracing_mi355.h)
    and links libpt_mi355.so (running it needs a GPU: tests/test_gpu_host.py)."""
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    from cpuperformanceraytracer_amd.build import build_examples
    exe = build_examples()
    assert exe.exists()
