"""The drop-in boundary exercised as a real C++ link: examples/reference_host.cpp is a
reference-shaped host (Application.cpp:400-477 call sequence) that uses only the reference's names
from include/demofox_path_tracing_mi355.h and links libpt_mi355.so.  Its accumulator must equal the
oracle's image bit for bit; CopyOutputToFile + WriteImage must produce the 24-bit BMP."""
from __future__ import annotations

import subprocess
from pathlib import Path

import numpy as np
import pytest

from conftest import bits_equal, mismatch_report
from layouts import tiled_to_interleaved
from oracle import pyoracle as po

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]
EXE = ROOT / "examples" / "reference_host"


@pytest.fixture(scope="module")
def exe():
    if not EXE.exists():
        from cpuperformanceraytracer_amd.build import build_examples
        build_examples()
    return EXE


def _texture(w=128, h=64):
    i = np.arange(w * h * 3, dtype=np.uint64)
    t = ((i * 2654435761) % (1 << 32)).astype(np.uint32).astype(np.float32) * np.float32(4.0 / 4294967296.0)
    return (t + np.float32(0.01)).astype(np.float32).reshape(h, w, 3)


def _run(exe, tmp_path, renderer, w, h, frames, bmp=True):
    out = tmp_path / f"{renderer}.f32"
    args = [str(exe), renderer, str(w), str(h), str(frames), str(out)]
    if bmp:
        args.append(str(tmp_path / f"{renderer}.bmp"))
    r = subprocess.run(args, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return np.fromfile(out, np.float32)


def test_host_v4(exe, tmp_path):
    w, h, frames = 320, 240, 3
    buf = _run(exe, tmp_path, "v4", w, h, frames)
    got = tiled_to_interleaved(buf, w, h, w // 10, h // 15)
    ref = po.render4(w, h, nframes=frames, env=_texture())
    assert bits_equal(got, ref), mismatch_report(got, ref)
    bmp = (tmp_path / "v4.bmp").read_bytes()
    assert bmp[:2] == b"BM" and len(bmp) == 54 + w * h * 3
    # CopyOutputToFile's pixels are the oracle's tonemap of the same accumulator (bytes R, G, B)
    px = po.tonemap(ref, po.PIXEL_RGBA8).view(np.uint8).reshape(h, w, 4)[..., :3]
    rows = np.frombuffer(bmp[54:], np.uint8).reshape(h, w, 3)[::-1, :, ::-1]   # bottom-up, BGR
    assert np.array_equal(rows, px)


@pytest.mark.parametrize("renderer", ["tiled", "scalar"])
def test_host_diffuse(exe, tmp_path, renderer):
    w, h, frames = 160, 120, 2
    buf = _run(exe, tmp_path, renderer, w, h, frames, bmp=False)
    got = tiled_to_interleaved(buf, w, h, w // 10, h // 15) if renderer == "tiled" else buf.reshape(h, w, 3)
    ref = po.render(w, h, nframes=frames, num_bounces=4)   # no pt_init: the reference defaults
    assert bits_equal(got, ref), mismatch_report(got, ref)
