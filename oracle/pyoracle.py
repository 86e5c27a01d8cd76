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


def ref_available() -> bool:
    return REF_BIN.exists()


def ref_render(width: int, height: int, frames: int, tmpdir: Path) -> np.ndarray:
    """Run the reference's own scalar code (fresh process => iFrame starts at 0)."""
    out = Path(tmpdir) / f"ref_{width}x{height}_{frames}.f32"
    subprocess.run([str(REF_BIN), str(width), str(height), str(frames), str(out)], check=True)
    return np.fromfile(out, np.float32).reshape(height, width, 3)


PIXEL_RGBA8 = 0   # PTO_PIXEL_RGBA8 (OutputToFile)
PIXEL_XRGB8 = 1   # PTO_PIXEL_XRGB8 (OutputToScreen)


def tonemap(rgb: np.ndarray, fmt: int = PIXEL_RGBA8) -> np.ndarray:
    """Output stage of v4 (oracle/pt_oracle_output.c) on an interleaved H x W x 3 accumulator."""
    a = np.ascontiguousarray(rgb, dtype=np.float32)
    h, w = a.shape[0], a.shape[1]
    out = np.empty((h, w), np.uint32)
    load().pto_tonemap(a.ctypes.data, w, h, fmt, out.ctypes.data)
    return out


def tonemap_channel(v: float) -> int:
    return int(load().pto_tonemap_channel(float(v)))
