"""oracle/pyoracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes binding of oracle/liboracle.so (the from-scratch CPU restatement, pt_oracle.c) and of the
reference's own scalar build oracle/_ref/ (build_ref.sh).  Importable only by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg -- never by the product package.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "liboracle.so"
REF_BIN = HERE / "_ref" / "ref_scalar"
REF_LIB = HERE / "_ref" / "libref_scalar.so"


class Env(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("width", ctypes.c_int32), ("height", ctypes.c_int32)]


class Params(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("row_start", ctypes.c_int32),
                ("row_stride", ctypes.c_int32), ("nrows", ctypes.c_int32), ("frame_first", ctypes.c_uint32),
                ("nframes", ctypes.c_int32), ("num_bounces", ctypes.c_int32), ("ambient", ctypes.c_float * 3),
                ("env", ctypes.POINTER(Env)), ("nthreads", ctypes.c_int32)]


class Counts(ctypes.Structure):
    _fields_ = [("samples", ctypes.c_uint64), ("segments", ctypes.c_uint64), ("flops_sample", ctypes.c_uint64),
                ("flops_segment", ctypes.c_uint64), ("transcendentals", ctypes.c_uint64),
                ("escaped", ctypes.c_uint64), ("segments_primary", ctypes.c_uint64),
                ("flops_segment_primary", ctypes.c_uint64), ("flops_shared", ctypes.c_uint64)]


_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


def load() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        L = ctypes.CDLL(str(LIB))
        L.pto_render.argtypes = [ctypes.c_void_p, ctypes.POINTER(Params)]
        L.pto_render.restype = ctypes.c_int
        L.pto_render_counted.argtypes = [ctypes.c_void_p, ctypes.POINTER(Params), ctypes.POINTER(Counts)]
        L.pto_render_counted.restype = ctypes.c_int
        L.pto_wang_hash.argtypes = [ctypes.POINTER(ctypes.c_uint32)]
        L.pto_wang_hash.restype = ctypes.c_uint32
        L.pto_randomf.argtypes = [ctypes.POINTER(ctypes.c_uint32)]
        L.pto_randomf.restype = ctypes.c_float
        L.pto_random_unit_vector.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_float)]
        L.pto_seed.argtypes = [ctypes.c_uint32] * 3
        L.pto_seed.restype = ctypes.c_uint32
        L.pto_env_sample.argtypes = [ctypes.POINTER(Env), ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]
        L.pto_tonemap_channel.restype = ctypes.c_uint32
        L.pto_tonemap_channel.argtypes = [ctypes.c_float]
        L.pto_tonemap.restype = None
        L.pto_tonemap.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p]
        L.pto_tonemap_ex.restype = None
        L.pto_tonemap_ex.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                     ctypes.c_int32, ctypes.c_void_p]
        L.pto_tonemap_channel_ex.restype = ctypes.c_uint32
        L.pto_tonemap_channel_ex.argtypes = [ctypes.c_float, ctypes.c_int32, ctypes.c_int32]
        _lib = L
    return _lib


def _params(width, height, row_start, row_stride, nrows, frame_first, nframes, num_bounces, ambient, env, nthreads):
    p = Params(width, height, row_start, row_stride, nrows, frame_first, nframes, num_bounces,
               (ctypes.c_float * 3)(*ambient), None, nthreads)
    keep = None
    if env is not None:
        env = np.ascontiguousarray(env, dtype=np.float32)
        keep = (env, Env(env.ctypes.data, env.shape[1], env.shape[0]))
        p.env = ctypes.pointer(keep[1])
    return p, keep


def render(width: int, height: int, *, frame_first: int = 1, nframes: int = 1, num_bounces: int = 4,
           row_start: int = 0, row_stride: int = 1, nrows: int | None = None, ambient=(0.1, 0.1, 0.1),
           env: np.ndarray | None = None, nthreads: int | None = None, buf: np.ndarray | None = None) -> np.ndarray:
    """Accumulate frames [frame_first, frame_first+nframes) into buf (nrows x width x 3, interleaved)."""
    nrows = height if nrows is None else nrows
    if buf is None:
        buf = np.zeros((nrows, width, 3), np.float32)
    assert buf.dtype == np.float32 and buf.flags["C_CONTIGUOUS"] and buf.size >= nrows * width * 3
    nthreads = nthreads if nthreads is not None else min(os.cpu_count() or 1, 16)
    p, keep = _params(width, height, row_start, row_stride, nrows, frame_first, nframes, num_bounces, ambient, env,
                      nthreads)
    rc = load().pto_render(buf.ctypes.data, ctypes.byref(p))
    del keep
    if rc:
        raise ValueError("pto_render rejected the parameters")
    return buf


def render_counted(width: int, height: int, **kw) -> tuple[np.ndarray, dict]:
    nrows = kw.pop("nrows", None)
    nrows = height if nrows is None else nrows
    buf = np.zeros((nrows, width, 3), np.float32)
    p, keep = _params(width, height, kw.pop("row_start", 0), kw.pop("row_stride", 1), nrows,
                      kw.pop("frame_first", 1), kw.pop("nframes", 1), kw.pop("num_bounces", 4),
                      kw.pop("ambient", (0.1, 0.1, 0.1)), kw.pop("env", None), 1)
    assert not kw, kw
    c = Counts()
    rc = load().pto_render_counted(buf.ctypes.data, ctypes.byref(p), ctypes.byref(c))
    del keep
    if rc:
        raise ValueError("pto_render_counted rejected the parameters")
    return buf, {k: getattr(c, k) for k, _ in Counts._fields_}


def wang_hash_sequence(seed: int, n: int) -> list[int]:
    s = ctypes.c_uint32(seed)
    return [int(load().pto_wang_hash(ctypes.byref(s))) for _ in range(n)]


def seed(x: int, y: int, frame: int) -> int:
    return int(load().pto_seed(x, y, frame))


def random_unit_vector(seed_value: int, n: int) -> np.ndarray:
    s = ctypes.c_uint32(seed_value)
    out = np.zeros((n, 3), np.float32)
    v = (ctypes.c_float * 3)()
    for i in range(n):
        load().pto_random_unit_vector(ctypes.byref(s), v)
        out[i] = list(v)
    return out


def env_sample(env: np.ndarray, dirs: np.ndarray) -> np.ndarray:
    """pto_env_sample (texture.cpp:101-139's per-lane body) of every direction: N x 3 texels."""
    env = np.ascontiguousarray(env, dtype=np.float32)
    e = Env(env.ctypes.data, env.shape[1], env.shape[0])
    d = np.ascontiguousarray(dirs, dtype=np.float32).reshape(-1, 3)
    out = np.zeros_like(d)
    L = load()
    fp = ctypes.POINTER(ctypes.c_float)
    for i in range(d.shape[0]):
        L.pto_env_sample(ctypes.byref(e), d[i].ctypes.data_as(fp), out[i].ctypes.data_as(fp))
    return out


REF_BIN_B8 = HERE / "_ref" / "ref_scalar_b8"
REF_ENV = HERE / "_ref" / "ref_env"


def ref_available(num_bounces: int = 4) -> bool:
    return (REF_BIN if num_bounces == 4 else REF_BIN_B8).exists()


def ref_render(width: int, height: int, frames: int, tmpdir: Path, num_bounces: int = 4) -> np.ndarray:
    """Run the reference's own scalar code (fresh process => iFrame starts at 0).  num_bounces 8
    runs the build whose only change is c_numBounces = 8 (scalar.cpp:19, oracle/build_ref.sh)."""
    if num_bounces not in (4, 8):
        raise ValueError("the reference builds have c_numBounces 4 (as shipped) or 8 (its //8)")
    out = Path(tmpdir) / f"ref_{width}x{height}_{frames}_b{num_bounces}.f32"
    exe = REF_BIN if num_bounces == 4 else REF_BIN_B8
    subprocess.run([str(exe), str(width), str(height), str(frames), str(out)], check=True)
    return np.fromfile(out, np.float32).reshape(height, width, 3)


def ref_env_available() -> bool:
    return REF_ENV.exists()


def ref_env_sample(env: np.ndarray, dirs: np.ndarray, tmpdir: Path) -> np.ndarray:
    """The reference's own texture.cpp:111-135 (+ TexelFetch :6-14) on every direction (ref_env)."""
    env = np.ascontiguousarray(env, dtype=np.float32)
    d = np.ascontiguousarray(dirs, dtype=np.float32).reshape(-1, 3)
    tdir = Path(tmpdir)
    env.tofile(tdir / "env_tex.f32")
    d.tofile(tdir / "env_dirs.f32")
    subprocess.run([str(REF_ENV), str(tdir / "env_tex.f32"), str(env.shape[1]), str(env.shape[0]),
                    str(tdir / "env_dirs.f32"), str(tdir / "env_out.f32")], check=True)
    return np.fromfile(tdir / "env_out.f32", np.float32).reshape(-1, 3)


PIXEL_RGBA8 = 0   # PTO_PIXEL_RGBA8 (OutputToFile)
PIXEL_XRGB8 = 1   # PTO_PIXEL_XRGB8 (OutputToScreen)


def tonemap(rgb: np.ndarray, fmt: int = PIXEL_RGBA8, fast_aces: bool = True, fast_gamma: bool = True) -> np.ndarray:
    """Output stage of v4 (oracle/pt_oracle_output.c) on an interleaved H x W x 3 accumulator;
    fast_aces / fast_gamma: USE_FAST_APPROXIMATE_ACES_TONEMAP / _GAMMA (global_preprocessor_flags.h:62-63)."""
    a = np.ascontiguousarray(rgb, dtype=np.float32)
    h, w = a.shape[0], a.shape[1]
    out = np.empty((h, w), np.uint32)
    load().pto_tonemap_ex(a.ctypes.data, w, h, fmt, int(not fast_aces), int(not fast_gamma), out.ctypes.data)
    return out


def tonemap_channel(v: float, fast_aces: bool = True, fast_gamma: bool = True) -> int:
    return int(load().pto_tonemap_channel_ex(float(v), int(not fast_aces), int(not fast_gamma)))


# ---- v4 renderer (pt_oracle_v4.c) -----------------------------------------------------------------
ENV_NONE, ENV_EQUIRECT, ENV_CUBEMAP = 0, 1, 2
MAX_OBJECTS = 12


class Material4(ctypes.Structure):
    _fields_ = [("albedo", ctypes.c_float * 3), ("emissive", ctypes.c_float * 3), ("spec_chance", ctypes.c_float),
                ("spec_rough", ctypes.c_float), ("spec_color", ctypes.c_float * 3), ("ior", ctypes.c_float),
                ("refr_chance", ctypes.c_float), ("refr_rough", ctypes.c_float), ("refr_color", ctypes.c_float * 3)]


class Scene4(ctypes.Structure):
    _fields_ = [("nquads", ctypes.c_int32), ("nspheres", ctypes.c_int32), ("nmat", ctypes.c_int32),
                ("quad", ctypes.c_float * 3 * 4 * MAX_OBJECTS), ("sphere", ctypes.c_float * 4 * MAX_OBJECTS),
                ("mat", Material4 * MAX_OBJECTS)]


class Params4(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("row_start", ctypes.c_int32),
                ("row_stride", ctypes.c_int32), ("nrows", ctypes.c_int32), ("frame_first", ctypes.c_uint32),
                ("nframes", ctypes.c_int32), ("num_bounces", ctypes.c_int32), ("env_mode", ctypes.c_int32),
                ("random_jitter", ctypes.c_int32), ("rejection", ctypes.c_int32), ("env", ctypes.POINTER(Env)),
                ("nthreads", ctypes.c_int32), ("no_accumulate", ctypes.c_int32), ("exact_exp", ctypes.c_int32)]


class Counts4(ctypes.Structure):
    _fields_ = [("samples", ctypes.c_uint64), ("segments", ctypes.c_uint64), ("escaped", ctypes.c_uint64),
                ("flops", ctypes.c_uint64), ("transcendentals", ctypes.c_uint64)]


def _load4() -> ctypes.CDLL:
    L = load()
    if not getattr(L, "_v4", False):
        L.pto4_default_scene.argtypes = [ctypes.POINTER(Scene4)]
        L.pto4_render.argtypes = [ctypes.c_void_p, ctypes.POINTER(Params4), ctypes.POINTER(Scene4),
                                  ctypes.POINTER(Counts4)]
        L.pto4_render.restype = ctypes.c_int
        L.pto4_scene_tables.argtypes = [ctypes.POINTER(Scene4), ctypes.c_void_p, ctypes.c_int32]
        L.pto4_scene_tables.restype = ctypes.c_int
        L.pto4_randomf.argtypes = [ctypes.POINTER(ctypes.c_uint32)]
        L.pto4_randomf.restype = ctypes.c_float
        L.pto4_random_unit_vector.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.c_int,
                                              ctypes.POINTER(ctypes.c_float)]
        L.pto4_env_sample.argtypes = [ctypes.POINTER(Env), ctypes.c_int32, ctypes.c_int32,
                                      ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_uint32),
                                      ctypes.POINTER(ctypes.c_float)]
        L._v4 = True
    return L


def default_scene4() -> Scene4:
    s = Scene4()
    _load4().pto4_default_scene(ctypes.byref(s))
    return s


def render4(width: int, height: int, *, frame_first: int = 1, nframes: int = 1, num_bounces: int = 8,
            row_start: int = 0, row_stride: int = 1, nrows: int | None = None, env_mode: int = ENV_EQUIRECT,
            env: np.ndarray | None = None, random_jitter: bool = True, rejection: bool = True,
            scene: Scene4 | None = None, nthreads: int | None = None, buf: np.ndarray | None = None,
            counts: bool = False, accumulate: bool = True, fast_exp: bool = True):
    """v4 renderer (DemofoxRenderOptV4): accumulate frames [frame_first, +nframes) into buf
    (nrows x width x 3, interleaved).  env None => ambient (USE_ENV_MAP 0).  counts=True returns
    (buf, {samples, segments, escaped}) and renders single-threaded.  accumulate / fast_exp:
    ACCUMULATE_FRAMES / USE_FAST_APPROXIMATE_EXP (global_preprocessor_flags.h:60,64)."""
    nrows = height if nrows is None else nrows
    if buf is None:
        buf = np.zeros((nrows, width, 3), np.float32)
    assert buf.dtype == np.float32 and buf.flags["C_CONTIGUOUS"] and buf.size >= nrows * width * 3
    nthreads = nthreads if nthreads is not None else min(os.cpu_count() or 1, 16)
    p = Params4(width, height, row_start, row_stride, nrows, frame_first, nframes, num_bounces,
                env_mode if env is not None else ENV_NONE, int(random_jitter), int(rejection), None, nthreads,
                int(not accumulate), int(not fast_exp))
    keep = None
    if env is not None:
        env = np.ascontiguousarray(env, dtype=np.float32)
        keep = (env, Env(env.ctypes.data, env.shape[1], env.shape[0]))
        p.env = ctypes.pointer(keep[1])
    c = Counts4()
    rc = _load4().pto4_render(buf.ctypes.data, ctypes.byref(p), ctypes.byref(scene) if scene is not None else None,
                              ctypes.byref(c) if counts else None)
    del keep
    if rc:
        raise ValueError("pto4_render rejected the parameters")
    if counts:
        return buf, {k: int(getattr(c, k)) for k, _ in Counts4._fields_}
    return buf


def scene4_tables(scene: Scene4 | None = None) -> np.ndarray:
    out = np.zeros(18 * MAX_OBJECTS + 17 * MAX_OBJECTS, np.float32)
    n = _load4().pto4_scene_tables(ctypes.byref(scene) if scene is not None else None, out.ctypes.data, out.size)
    if n < 0:
        raise ValueError("invalid scene")
    return out[:n]


def env_sample4(env: np.ndarray | None, env_mode: int, random_jitter: bool, dirs: np.ndarray, seed_value: int = 1):
    """Per-direction env lookups (v4 :769-784), one RNG state threaded through all of them."""
    keep = None
    ep = None
    if env is not None:
        env = np.ascontiguousarray(env, dtype=np.float32)
        keep = (env, Env(env.ctypes.data, env.shape[1], env.shape[0]))
        ep = ctypes.pointer(keep[1])
    s = ctypes.c_uint32(seed_value)
    d = np.ascontiguousarray(dirs, dtype=np.float32).reshape(-1, 3)
    out = np.zeros_like(d)
    o = (ctypes.c_float * 3)()
    for i in range(d.shape[0]):
        v = (ctypes.c_float * 3)(*d[i])
        _load4().pto4_env_sample(ep, env_mode, int(random_jitter), v, ctypes.byref(s), o)
        out[i] = list(o)
    del keep
    return out


# ---- CPU baseline: AVX2 port of demofox_path_tracing_simt_pooled.cpp (pt_cpu_simd.c) -----------------
SIMD_LIB = HERE / "libcpusimd.so"
_simd = None


def simd_load():
    global _simd
    if _simd is None:
        if not SIMD_LIB.exists():
            build()
        L = ctypes.CDLL(str(SIMD_LIB))
        L.ptc_simd_supported.restype = ctypes.c_int
        L.ptc_render_simd_tiled.restype = ctypes.c_int
        L.ptc_render_simd_tiled.argtypes = [ctypes.c_void_p] + [ctypes.c_int32] * 4 + [ctypes.c_uint32] + \
            [ctypes.c_int32] * 3
        _simd = L
    return _simd


def simd_supported() -> bool:
    return bool(simd_load().ptc_simd_supported())


def render_simd_tiled(width: int, height: int, num_tiles_x: int, num_tiles_y: int, *, frame_first: int = 1,
                      nframes: int = 1, num_bounces: int = 8, nthreads: int | None = None,
                      buf: np.ndarray | None = None) -> np.ndarray:
    """The AVX2 simt_pooled port: accumulate frames into buf (tile-major planar8 layout)."""
    if buf is None:
        buf = np.zeros(width * height * 3, np.float32)
    nthreads = nthreads if nthreads is not None else min(os.cpu_count() or 1, 16)
    rc = simd_load().ptc_render_simd_tiled(buf.ctypes.data, width, height, num_tiles_x, num_tiles_y, frame_first,
                                           nframes, num_bounces, nthreads)
    if rc:
        raise ValueError(f"ptc_render_simd_tiled failed ({rc})")
    return buf


def sky_skipped(width: int, height: int, *, row_start: int = 0, row_stride: int = 1, nrows: int | None = None,
                slope: float = 0.51) -> tuple[int, int]:
    """(camera rays, their TestSceneTrace flops) that the diffuse kernel's sky tiles skip (pto_sky_skipped)."""
    nrows = height if nrows is None else nrows
    p, keep = _params(width, height, row_start, row_stride, nrows, 1, 1, 8, (0.1, 0.1, 0.1), None, 1)
    fl = ctypes.c_uint64(0)
    L = load()
    L.pto_sky_skipped.restype = ctypes.c_uint64
    L.pto_sky_skipped.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.POINTER(ctypes.c_uint64)]
    n = L.pto_sky_skipped(ctypes.byref(p), slope, ctypes.byref(fl))
    del keep
    return int(n), int(fl.value)


def trace4(P, D) -> tuple[float, int, int]:
    """v4 TestSceneTrace of one ray in the default scene: (distance, material, reference flops)
    (pto4_trace_scene_flops)."""
    L = load()
    f3 = ctypes.c_float * 3
    L.pto4_trace_scene_flops.restype = ctypes.c_float
    L.pto4_trace_scene_flops.argtypes = [ctypes.c_void_p, f3, f3, ctypes.POINTER(ctypes.c_int),
                                         ctypes.POINTER(ctypes.c_uint64)]
    mat, fl = ctypes.c_int(-1), ctypes.c_uint64(0)
    d = L.pto4_trace_scene_flops(None, f3(*P), f3(*D), ctypes.byref(mat), ctypes.byref(fl))
    return float(d), int(mat.value), int(fl.value)
