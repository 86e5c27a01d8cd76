"""LoadTexture (asset_loading.cpp:9-16) -> csrc/pt_texture.cpp, the RGBE .hdr decoder of config 4.

Pinned against the reference's vendored stb_image v2.26, compiled from the reference's sources
by oracle/build_ref.sh (oracle/_ref/ref_hdr): bit-identical texels on every texture the reference
ships (when /root/reference is present) and on synthetic files covering each scanline encoding
stb accepts.  The decoder is host code inside libpt_mi355.so, so these run without a GPU.
"""
from __future__ import annotations

import hashlib
import subprocess
from pathlib import Path

import numpy as np
import pytest

import cpuperformanceraytracer_amd as pt
from cpuperformanceraytracer_amd import _native as N
from cpuperformanceraytracer_amd.renderer import DecodeHdr

ROOT = Path(__file__).resolve().parents[1]
REF_TEXTURES = Path("/root/reference/Textures")
REF_HDR = ROOT / "oracle" / "_ref" / "ref_hdr"
# sha256 of the f32 texels stb_image decodes from HDR_040_Field_Env.hdr (512 x 256 x 3, flipped)
FIELD_ENV_SHA256 = "e1b72594c8b294b1905bc941249b40a9f9da0ab5a7a1df79cc8bc63eda50ea5c"


def _lib_or_skip():
    try:
        N.load()
    except (OSError, FileNotFoundError) as e:
        pytest.skip(f"libpt_mi355.so not loadable here: {e}")


def _stb(path: Path, tmp_path: Path) -> np.ndarray:
    out = tmp_path / "stb.bin"
    subprocess.run([str(REF_HDR), str(path), str(out)], check=True, capture_output=True)
    w, h, c = np.fromfile(out, dtype=np.int32, count=3)
    return np.fromfile(out, dtype=np.float32, offset=12).reshape(h, w, c)


def _header(w: int, h: int, sig: bytes = b"#?RADIANCE") -> bytes:
    return sig + b"\n# made by tests/test_texture.py\nFORMAT=32-bit_rle_rgbe\nEXPOSURE=1.0\n\n" + \
        f"-Y {h} +X {w}\n".encode()


def _rle_plane(vals: np.ndarray) -> bytes:
    """One channel of a new-style RLE scanline: alternate runs (>=3 equal bytes) and dumps."""
    out, i, n = bytearray(), 0, len(vals)
    while i < n:
        j = i
        while j < n and vals[j] == vals[i] and j - i < 127:
            j += 1
        if j - i >= 3:
            out += bytes([128 + (j - i), int(vals[i])])
            i = j
            continue
        k = i
        while k < n and k - i < 128 and not (k + 2 < n and vals[k] == vals[k + 1] == vals[k + 2]):
            k += 1
        out += bytes([k - i]) + bytes(int(v) for v in vals[i:k])
        i = k
    return bytes(out)


def _expected(rgbe: np.ndarray) -> np.ndarray:
    """stbi__hdr_convert + vertical flip, restated: c * 2^(e-136), e == 0 -> 0."""
    e = rgbe[..., 3].astype(np.int32)
    scale = np.where(e != 0, np.ldexp(np.float32(1.0), e - 136), 0).astype(np.float32)
    out = rgbe[..., :3].astype(np.float32) * scale[..., None]
    return out[::-1].copy()


def _random_rgbe(h: int, w: int, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    px = rng.integers(0, 256, (h, w, 4), dtype=np.uint8)
    px[..., 3] = rng.choice(np.array([0, 1, 100, 128, 136, 140, 255], np.uint8), (h, w))
    px[:, : w // 3] = px[:, :1]              # runs
    return px


def _encode(px: np.ndarray, mode: str, sig: bytes = b"#?RADIANCE") -> bytes:
    h, w, _ = px.shape
    body = bytearray()
    if mode == "flat":
        body += px.tobytes()
    elif mode == "rle":
        for j in range(h):
            body += bytes([2, 2, w >> 8, w & 255])
            for k in range(4):
                body += _rle_plane(px[j, :, k])
    elif mode == "rle_then_flat":            # first scanline RLE, the second not -> stb goes flat
        body += bytes([2, 2, w >> 8, w & 255])
        for k in range(4):
            body += _rle_plane(px[0, :, k])
        body += px.tobytes()                 # restarts at pixel 0 of row 0 (stb's goto)
    return _header(w, h, sig) + bytes(body)


@pytest.mark.parametrize("mode,w,h", [("flat", 5, 3), ("flat", 7, 9), ("rle", 8, 4), ("rle", 300, 7),
                                      ("rle", 1000, 2), ("flat", 40, 6)])
def test_synthetic_encodings(tmp_path, mode, w, h):
    _lib_or_skip()
    px = _random_rgbe(h, w, seed=w * 7 + h)
    if mode == "flat" and w >= 8:
        px[:, 0, 0] = 200                    # first bytes are not the 2,2 RLE marker
    data = _encode(px, mode)
    t = DecodeHdr(data)
    assert (t.Width, t.Height, t.Components) == (w, h, 3)
    assert np.array_equal(t.Data.view(np.uint32), _expected(px).view(np.uint32))
    if REF_HDR.exists():
        f = tmp_path / "x.hdr"
        f.write_bytes(data)
        assert np.array_equal(t.Data.view(np.uint32), _stb(f, tmp_path).view(np.uint32))


def test_rle_then_flat_quirk(tmp_path):
    """stb: a scanline without the RLE marker switches to flat decoding from pixel 1 of row 0."""
    _lib_or_skip()
    w, h = 16, 3
    px = _random_rgbe(h, w, seed=11)
    px[:, 0, 0] = 200
    data = _encode(px, "rle_then_flat", sig=b"#?RGBE")
    # after the RLE row, the flat stream's first pixel becomes (0,0), the rest continue from (0,1)
    t = DecodeHdr(data)
    assert np.array_equal(t.Data.view(np.uint32), _expected(px).view(np.uint32))
    if REF_HDR.exists():
        f = tmp_path / "q.hdr"
        f.write_bytes(data)
        assert np.array_equal(t.Data.view(np.uint32), _stb(f, tmp_path).view(np.uint32))


@pytest.mark.parametrize("bad", [
    b"#?RADIANCEX\nFORMAT=32-bit_rle_rgbe\n\n-Y 1 +X 1\n\x01\x01\x01\x80",      # signature
    b"#?RADIANCE\nFORMAT=32-bit_rle_xyze\n\n-Y 1 +X 1\n\x01\x01\x01\x80",       # format
    b"#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n+Y 1 +X 1\n\x01\x01\x01\x80",       # orientation
    b"#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n-Y 2 +X 2\n\x01\x01\x01\x80",       # truncated
    b"#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n-Y 1 +X 8\n\x02\x02\x00\x09",       # scanline length
    b"#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n-Y 1 +X 8\n\x02\x02\x00\x08\x8a\x01",  # run > width
])
def test_malformed_files_raise(bad):
    _lib_or_skip()
    with pytest.raises(N.PtError) as e:
        DecodeHdr(bad)
    assert e.value.code == N.PT_EINVAL


def test_missing_file_raises(tmp_path):
    _lib_or_skip()
    with pytest.raises(N.PtError):
        pt.LoadTexture(tmp_path / "nope.hdr")


@pytest.mark.skipif(not (REF_TEXTURES / "HDR_040_Field_Env.hdr").exists(), reason="reference textures absent")
def test_field_env_kat():
    """The config-4 parity texture of the reference decodes to stb's texels (sha256 recorded)."""
    _lib_or_skip()
    t = pt.LoadTexture(REF_TEXTURES / "HDR_040_Field_Env.hdr")
    assert (t.Width, t.Height, t.Components) == (512, 256, 3)
    assert hashlib.sha256(t.Data.tobytes()).hexdigest() == FIELD_ENV_SHA256


@pytest.mark.skipif(not REF_HDR.exists() or not REF_TEXTURES.exists(), reason="stb reference build absent")
@pytest.mark.parametrize("name", ["HDR_040_Field_Env", "px", "nx", "py", "ny", "pz", "nz"])
def test_reference_textures_match_stb(tmp_path, name):
    _lib_or_skip()
    t = pt.LoadTexture(REF_TEXTURES / f"{name}.hdr")
    ref = _stb(REF_TEXTURES / f"{name}.hdr", tmp_path)
    assert t.Data.shape == ref.shape
    assert np.array_equal(t.Data.view(np.uint32), ref.view(np.uint32))


def test_texture_struct_layout():
    """pt_texture {float* data; int32 width, height, components} -- 24 bytes on LP64."""
    import ctypes
    assert ctypes.sizeof(N.PtTexture) == 24
    assert [f[0] for f in N.PtTexture._fields_] == ["data", "width", "height", "components"]
