"""CPU checks of the v4 oracle (oracle/pt_oracle_v4.c), the checker for the v4 GPU kernel.

The reference's v4 file (demofox_path_tracing_optimization_v4.cpp) is Win32 + SVML code and
cannot be built here, so these pin the restatement piecewise: its RNG against the scalar oracle's
wang hash (itself pinned to the reference's goldens), Randomf3201_ps / the camera / the env lookups
against independent numpy + libm restatements of mathutils.h and texture.cpp, the scene tables of
InitializeScene, and the renderer's structural invariants (row shards, frame splits, pixel
independence).  Parity of the whole v4 image against a reference run is unpinned.
"""
from __future__ import annotations

import ctypes
import ctypes.util

import numpy as np
import pytest

from conftest import bits_equal
from oracle import pyoracle as po

libm = ctypes.CDLL(ctypes.util.find_library("m"))
for _f in ("tanf", "atan2f", "asinf", "floorf"):
    getattr(libm, _f).restype = ctypes.c_float
libm.tanf.argtypes = [ctypes.c_float]
libm.asinf.argtypes = [ctypes.c_float]
libm.floorf.argtypes = [ctypes.c_float]
libm.atan2f.argtypes = [ctypes.c_float, ctypes.c_float]
f32 = np.float32


def _wang(x: int) -> int:   # mathutils.h:8-16
    x = ((x ^ 61) ^ (x >> 16)) & 0xFFFFFFFF
    x = (x * 9) & 0xFFFFFFFF
    x = x ^ (x >> 4)
    x = (x * 0x27D4EB2D) & 0xFFFFFFFF
    return x ^ (x >> 15)


def test_randomf_matches_mathutils():
    """Randomf3201_ps: cvtepi32_ps(h & 0x7FFFFFFF) / 2147483648.0f (mathutils.h:18-26)."""
    for seed in (1, 2392335, 0xDEADBEEF, 12345 | 1):
        s = ctypes.c_uint32(seed)
        x = seed
        for _ in range(64):
            x = _wang(x)
            want = f32(f32(x & 0x7FFFFFFF) / f32(2147483648.0))
            got = po._load4().pto4_randomf(ctypes.byref(s))
            assert f32(got) == want
        assert s.value == x
    # the same hash as the scalar oracle (pinned to the reference's own scalar build)
    assert po.wang_hash_sequence(1, 4) == [663891101, 1738326990, 801461103, 3205955024]


def test_camera_distance_is_one():
    """InitializeCamera (v4 :1500): 1 / tan(c_FOVDegrees * 0.5 * c_pi / 180) in f32 == 1.0f (the
    kernel uses the constant)."""
    a = f32(f32(f32(f32(90.0) * f32(0.5)) * f32(3.14159265359)) / f32(180.0))
    assert f32(f32(1.0) / f32(libm.tanf(a))) == f32(1.0)


def test_default_scene_tables():
    t = po.scene4_tables()
    quads = t[:18 * 4].reshape(4, 6, 3)
    mats = t[18 * 4:].reshape(12, 17)
    # floor V0 translated by (0,0,10); normal +y; stripes quad untranslated (z = 5)
    assert quads[0, 0].tolist() == [-25.0, -12.5, 15.0] and quads[0, 1].tolist() == [0.0, 1.0, 0.0]
    assert quads[1, 0].tolist() == [-25.0, -1.5, 5.0]
    # AddMaterialToScene copies albedo.x into all three channels (v4 :1370-1372)
    assert np.all(mats[4:11, 0:3] == f32(0.9))
    assert mats[3, 3:6].tolist() == [20.0, 18.0, 14.0]            # light emissive (1,.9,.7)*20
    assert np.all(mats[0:4, 11] == 0.0)                            # quads: IOR 0 (SceneMaterial{0})
    assert mats[4:11, 11].tolist() == [f32(1.1)] * 7
    r = [f32(f32(f32(i) / f32(6.0)) * f32(0.5)) for i in range(7)]
    assert mats[4:11, 7].tolist() == r and mats[4:11, 13].tolist() == r   # spec / refr roughness
    assert np.all(mats[11] == 0.0)


def _equirect_random_np(env, d, seed):
    """EquirectangularTextureSampleRandom (texture.cpp:186-203) + TexelSampleRandom (:78-86),
    restated independently (numpy f32 + libm); fma via exact float64 products (a*b exact in f64)."""
    def fma(a, b, c):
        return f32(np.float64(a) * np.float64(b) + np.float64(c)) if abs(np.float64(a) * np.float64(b)) < 2**60 else None
    s = seed
    u = f32(libm.atan2f(f32(-d[2]), f32(-d[0])))
    v = f32(libm.asinf(f32(d[1])))
    u = fma(f32(0.1591), u, f32(0.5))
    v = fma(f32(0.3183), v, f32(0.5))
    u = f32(u - f32(libm.floorf(u)))
    v = f32(v - f32(libm.floorf(v)))
    u = min(max(u, f32(0)), f32(1))
    v = min(max(v, f32(0)), f32(1))
    H, W = env.shape[0], env.shape[1]
    row = fma(v, f32(H), -v)
    col = fma(u, f32(W), -u)
    s = _wang(s)
    rr = f32(np.floor(f32(row + f32(f32(s & 0x7FFFFFFF) / f32(2**31)))))
    s = _wang(s)
    rc = f32(np.floor(f32(col + f32(f32(s & 0x7FFFFFFF) / f32(2**31)))))
    lin = int(np.rint(fma(rr, f32(W), rc)))
    lin = min(max(lin, 0), W * H - 1)
    return env.reshape(-1, 3)[lin], s


def test_env_sample_equirect_random_independent():
    rng = np.random.default_rng(4)
    env = rng.random((37, 53, 3), dtype=np.float32)
    dirs = rng.normal(size=(200, 3)).astype(np.float32)
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    got = po.env_sample4(env, po.ENV_EQUIRECT, True, dirs, seed_value=99)
    s = 99
    for i, d in enumerate(dirs):
        want, s = _equirect_random_np(env, d, s)
        assert np.array_equal(got[i], want), (i, d, got[i], want)


def test_ambient_without_env():
    out = po.env_sample4(None, po.ENV_NONE, True, np.array([[0, 0, -1]], np.float32))
    assert out[0].tolist() == [f32(0.11), f32(0.1), f32(0.15)]


def test_cubemap_face_offsets():
    """Six constant 16x16 faces stacked (LoadCubemapTexture): the axis directions land in faces
    px nx py ny pz nz (texture.cpp:283-331), with both texel samplers."""
    env = np.repeat(np.arange(6, dtype=np.float32), 16 * 16 * 3).reshape(6 * 16, 16, 3)
    axes = np.array([[1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1]], np.float32)
    for jitter in (False, True):
        got = po.env_sample4(env, po.ENV_CUBEMAP, jitter, axes)
        assert got[:, 0].tolist() == [0, 1, 2, 3, 4, 5]


def test_row_shards_and_frame_split():
    env = np.random.default_rng(2).random((32, 64, 3), dtype=np.float32)
    w, h = 64, 40
    full = po.render4(w, h, nframes=5, env=env)
    part = po.render4(w, h, nframes=5, env=env, row_start=3, row_stride=4, nrows=(h - 3 + 3) // 4)
    assert bits_equal(part, full[3::4])
    split = po.render4(w, h, nframes=2, env=env)
    split = po.render4(w, h, frame_first=3, nframes=3, env=env, buf=split)
    assert bits_equal(split, full)
    # thread count never changes a pixel
    assert bits_equal(po.render4(w, h, nframes=5, env=env, nthreads=1), full)


def test_counts_and_scene_limits():
    _, c = po.render4(48, 32, nframes=2, env=None, counts=True)
    assert c["samples"] == 48 * 32 * 2 and c["segments"] >= c["samples"] and c["escaped"] <= c["samples"]
    s = po.default_scene4()
    s.nspheres = 9   # 4 quads + 9 spheres > MAX_OBJECTS
    with pytest.raises(ValueError):
        po.render4(8, 8, scene=s)


def test_counted_render_equals_plain_render():
    """Instrumentation never changes a pixel (counting on/off, threads)."""
    env = np.random.default_rng(8).random((16, 32, 3), dtype=np.float32)
    a, _ = po.render4(64, 48, nframes=3, env=env, counts=True)
    b = po.render4(64, 48, nframes=3, env=env, nthreads=4)
    assert bits_equal(a, b)
    assert (b != 0).any() and len(np.unique(b.reshape(-1, 3), axis=0)) > 100   # the scene is traced
