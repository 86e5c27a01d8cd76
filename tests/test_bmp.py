"""WriteImage (asset_loading.cpp:48-54, stbi_write_bmp) -> pt_write_bmp (csrc/pt_texture.cpp).

Pinned byte for byte against stb_image_write v1.15 compiled from the reference's own sources
(oracle/_ref/ref_bmp, built by oracle/build_ref.sh where /root/reference exists), for every row
padding, 1-4 components (4: alpha compositing over pink), empty images; and against an
independent restatement of the header in this file.  Host code in libpt_mi355.so: no GPU needed.
"""
from __future__ import annotations

import struct
import subprocess
from pathlib import Path

import numpy as np
import pytest

import cpuperformanceraytracer_amd as pt
from cpuperformanceraytracer_amd import _native as N

ROOT = Path(__file__).resolve().parents[1]
REF_BMP = ROOT / "oracle" / "_ref" / "ref_bmp"


def _lib_or_skip():
    try:
        N.load()
    except (OSError, FileNotFoundError) as e:
        pytest.skip(f"libpt_mi355.so not loadable here: {e}")


def _expected(px: np.ndarray, w: int, h: int, comp: int) -> bytes:
    pad = (-w * 3) & 3
    out = bytearray(b"BM" + struct.pack("<IHHI", 54 + (w * 3 + pad) * h, 0, 0, 54) +
                    struct.pack("<IiiHH6I", 40, w, h, 1, 24, 0, 0, 0, 0, 0, 0))
    d = px.reshape(h, w, comp).astype(np.int64) if w and h else px
    for j in range(h - 1, -1, -1):
        for i in range(w):
            p = d[j, i]
            if comp <= 2:
                bgr = (p[0], p[0], p[0])
            elif comp == 3:
                bgr = (p[2], p[1], p[0])
            else:
                bg = (255, 0, 255)
                c = [int(bg[k] + int((p[k] - bg[k]) * p[3] / 255)) for k in range(3)]   # C: truncation
                bgr = (c[2], c[1], c[0])
            out += bytes(int(v) & 0xFF for v in bgr)
        out += b"\0" * pad
    return bytes(out)


@pytest.mark.parametrize("w,h,comp", [(1, 1, 3), (2, 3, 3), (3, 2, 4), (4, 4, 1), (5, 3, 2), (7, 5, 4), (13, 9, 3),
                                      (0, 4, 3), (4, 0, 4)])
def test_bmp_bytes(tmp_path, w, h, comp):
    _lib_or_skip()
    rng = np.random.default_rng(w * 100 + h * 10 + comp)
    px = rng.integers(0, 256, w * h * comp, dtype=np.uint8)
    if comp == 4 and w * h:
        px.reshape(-1, 4)[::3, 3] = 255   # opaque pixels next to translucent ones
    f = tmp_path / "o.bmp"
    pt.WriteImage(f, w, h, comp, px)
    got = f.read_bytes()
    assert got == _expected(px, w, h, comp)
    if REF_BMP.exists():
        raw = tmp_path / "in.raw"
        raw.write_bytes(px.tobytes())
        ref = tmp_path / "ref.bmp"
        subprocess.run([str(REF_BMP), str(raw), str(w), str(h), str(comp), str(ref)], check=True)
        assert got == ref.read_bytes()


def test_bmp_of_file_pixels(tmp_path):
    """The reference's output path: 32-bit file pixels (R, G, B, 255) written with 4 components."""
    _lib_or_skip()
    rng = np.random.default_rng(5)
    rgba = rng.integers(0, 256, (6, 10, 4), dtype=np.uint8)
    rgba[..., 3] = 255
    f = tmp_path / "img.bmp"
    pt.WriteImage(f, 10, 6, 4, rgba)
    data = f.read_bytes()
    assert len(data) == 54 + (10 * 3 + 2) * 6
    row0 = data[54:54 + 30]                      # bottom row first, BGR
    assert row0 == bytes(rgba[5, :, [2, 1, 0]].T.reshape(-1))


def test_bmp_errors(tmp_path):
    _lib_or_skip()
    with pytest.raises(N.PtError):
        pt.WriteImage(tmp_path / "x.bmp", 2, 2, 5, np.zeros(20, np.uint8))
    with pytest.raises(N.PtError):
        pt.WriteImage(tmp_path / "no_such_dir" / "x.bmp", 1, 1, 3, np.zeros(3, np.uint8))
