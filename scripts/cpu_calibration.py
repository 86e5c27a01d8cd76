"""CPU calibration (BASELINE.md "Calibration to the reference"): the CPU restatements that
bench.py's cpu_baseline times, against the reference's own scalar build, on the same core.

One thread each, 640x360, 4 bounces (the reference build's compiled-in c_numBounces):
  reference_scalar  DemofoxRenderScalar built unmodified from /root/reference (oracle/_ref/)
  oracle_scalar     oracle/pt_oracle.c (the scalar restatement, bit-identical to it)
  simd_port         oracle/pt_cpu_simd.c (AVX2 + FMA port of simt_pooled, 10x15 tiles)
Prints one JSON object; the per-core ratios restate bench.py's CPU numbers in reference units.
The reference's SIMD build needs MSVC/SVML stand-ins and is not built.
usage: cpu_calibration.py [SECONDS_PER_LEG]
"""
import ctypes
import json
import platform
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from oracle import pyoracle  # noqa: E402

W, H, B = 640, 360, 4
SECONDS = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0


def timed(fn, first_frame_fn):
    t0 = time.perf_counter()
    first_frame_fn()
    t1 = time.perf_counter() - t0
    frames = int(max(1, min(512, round(SECONDS / max(t1, 1e-6)))))
    t0 = time.perf_counter()
    fn(frames)
    dt = time.perf_counter() - t0
    return {"frames": frames, "seconds": dt, "primary_samples_per_s": W * H * frames / dt}


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


out = {"workload": f"{W}x{H}, {B} bounces, 1 thread", "cpu_model": cpu_model()}
if pyoracle.REF_LIB.exists():
    L = ctypes.CDLL(str(pyoracle.REF_LIB))
    L.ref_render_scalar.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    rbuf = np.zeros((H, W, 3), np.float32)
    out["reference_scalar"] = timed(lambda n: L.ref_render_scalar(rbuf.ctypes.data, W, H, n),
                                    lambda: L.ref_render_scalar(rbuf.ctypes.data, W, H, 1))
obuf = pyoracle.render(W, H, frame_first=1, nframes=1, num_bounces=B, nthreads=1)
out["oracle_scalar"] = timed(lambda n: pyoracle.render(W, H, frame_first=2, nframes=n, num_bounces=B, nthreads=1, buf=obuf),
                             lambda: pyoracle.render(W, H, frame_first=1, nframes=1, num_bounces=B, nthreads=1))
if pyoracle.simd_supported():
    sbuf = pyoracle.render_simd_tiled(W, H, 10, 15, frame_first=1, nframes=1, num_bounces=B, nthreads=1)
    out["simd_port"] = timed(
        lambda n: pyoracle.render_simd_tiled(W, H, 10, 15, frame_first=2, nframes=n, num_bounces=B, nthreads=1, buf=sbuf),
        lambda: pyoracle.render_simd_tiled(W, H, 10, 15, frame_first=1, nframes=1, num_bounces=B, nthreads=1))
if "reference_scalar" in out:
    ref = out["reference_scalar"]["primary_samples_per_s"]
    out["per_core_ratio_vs_reference_scalar"] = {
        k: out[k]["primary_samples_per_s"] / ref for k in ("oracle_scalar", "simd_port") if k in out}
print(json.dumps(out))
