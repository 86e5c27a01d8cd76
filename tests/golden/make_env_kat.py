#!/usr/bin/env python3
"""Regenerate tests/golden/env_kat.npz: known answers of config 4's env miss term, produced by the
reference's OWN code -- texture.cpp:111-135 (the per-lane body of EquirectangularTextureSample,
called at demofox_path_tracing_simt_textured.cpp:408) with TexelFetch (texture.cpp:6-14), compiled
from the reference's line ranges by oracle/build_ref.sh into oracle/_ref/ref_env.

Requires /root/reference (this container only); the fixture (directions, texture shapes, expected
texels) is data and travels, the reference does not.

Textures are index-coded: texel (row, col) = (row, col, 1 + row*W + col) as f32 (exact below 2^24),
so an expected texel names the cell the reference picked; an all-zero texel is the reference's
"uv outside [0, 1)" branch (:130-135).  Directions: the poles, the +-x seam (atan2's +-pi branch
cut, signed zeros), atan2's quadrant edges and x = z diagonals, |y| one ulp above 1 (asin NaN),
denormal components, f32 directions on both sides of every 64th column boundary of the 2048 x 1024
map and every 16th row boundary (the (W-1) / (H-1) scaling of :123-124), and normalised random
directions as the renderer produces them.
"""
from __future__ import annotations

import sys
import tempfile
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path.insert(0, str(ROOT))

SHAPES = [(2048, 1024), (512, 256), (1, 1), (1, 9), (9, 1), (3, 5), (2, 2)]   # (W, H)


def index_texture(w: int, h: int) -> np.ndarray:
    r, c = np.meshgrid(np.arange(h, dtype=np.float32), np.arange(w, dtype=np.float32), indexing="ij")
    return np.stack([r, c, 1.0 + r * w + c], axis=-1).astype(np.float32)


def _normalize(v: np.ndarray) -> np.ndarray:
    """f32 normalize as the renderer does it (scalar.cpp normalize: v * (1 / sqrt(dot)))."""
    v = v.astype(np.float32)
    d = (v[:, 0] * v[:, 0] + v[:, 1] * v[:, 1]) + v[:, 2] * v[:, 2]
    inv = np.float32(1.0) / np.sqrt(d)
    return (v * inv[:, None]).astype(np.float32)


def _neighbours(v: np.ndarray, axis: int, k: int = 3) -> list[np.ndarray]:
    out = []
    for d in v:
        x = np.float32(d[axis])
        lo = hi = x
        for _ in range(k):
            lo = np.nextafter(lo, np.float32(-np.inf), dtype=np.float32)
            hi = np.nextafter(hi, np.float32(np.inf), dtype=np.float32)
            for y in (lo, hi):
                e = d.copy()
                e[axis] = y
                out.append(e)
        out.append(d.copy())
    return out


def directions() -> np.ndarray:
    f = np.float32
    tiny, den = f(1e-30), f(1e-40)
    one_up = np.nextafter(f(1), f(2), dtype=np.float32)
    edge = [
        (0, 1, 0), (0, -1, 0), (tiny, 1, 0), (-tiny, -1, tiny), (0, one_up, 0), (0, -one_up, 0),
        (-1, 0, 0), (-1, 0, -0.0), (-1, 0, tiny), (-1, 0, -tiny), (-1, 0, den), (-1, 0, -den),
        (-1, 0.5, 0.0), (-1, 0.5, -0.0), (-0.0, 0, -0.0), (0.0, 0, 0.0), (-0.0, 0.3, 0.0), (0.0, -0.3, -0.0),
        (1, 0, 0), (0, 0, 1), (0, 0, -1), (-0.0, 0, 1), (-0.0, 0, -1), (den, 0, den), (-den, 0, -den),
        (1, 0, 1), (-1, 0, 1), (-1, 0, -1), (1, 0, -1), (1, 1, 1), (-1, -1, -1),
    ]
    dirs = [np.array(e, np.float32) for e in edge]
    dirs += list(_normalize(np.array([e for e in edge[25:]], np.float32)))
    # column boundaries of the 2048-wide map: u * 2047 = k  =>  atan2 = (k / 2047 - 0.5) / 0.1591
    for k in range(0, 2048, 64):
        th = (k / 2047.0 - 0.5) / 0.1591
        v = np.array([[np.cos(th), 0.0, np.sin(th)]], np.float32)
        dirs += _neighbours(v, 2) + _neighbours(v, 0, 1)
    # row boundaries of the 1024-high map: v * 1023 = k  =>  asin(y) = (k / 1023 - 0.5) / 0.3183
    for k in range(0, 1024, 16):
        ph = (k / 1023.0 - 0.5) / 0.3183
        if abs(ph) >= np.pi / 2:
            continue
        v = np.array([[np.cos(ph), np.sin(ph), 0.25]], np.float32)
        dirs += _neighbours(v, 1)
    rng = np.random.default_rng(0xE17)
    dirs += list(_normalize(rng.normal(size=(8192, 3)).astype(np.float32)))
    return np.stack(dirs).astype(np.float32)


def main() -> None:
    from oracle import pyoracle
    import subprocess
    subprocess.run([str(ROOT / "oracle" / "build_ref.sh")], check=True)
    dirs = directions()
    out = {"dirs": dirs, "shapes": np.array(SHAPES, np.int32)}
    with tempfile.TemporaryDirectory() as td:
        for w, h in SHAPES:
            out[f"texels_{w}x{h}"] = pyoracle.ref_env_sample(index_texture(w, h), dirs, Path(td))
    np.savez_compressed(HERE / "env_kat.npz", **out)
    hit = (out["texels_2048x1024"] != 0).any(1)
    print(f"env_kat.npz: {len(dirs)} directions x {len(SHAPES)} textures; {hit.mean():.4f} in-range on 2048x1024")


if __name__ == "__main__":
    main()
