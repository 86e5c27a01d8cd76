"""PCIe-inclusive rate of the drop-in host-buffer path (dev tool).

DemofoxRenderScalar on a host numpy buffer, 1920x1080, 8 frames per call (samples_per_frame=8),
8 bounces: each call copies the 24.9 MB accumulator to HBM, runs the kernel and copies it back --
versus PT_FLAG_PIN_HOST (buffer page-locked, transfers overlapped with rendering in row bands)
and PT_FLAG_DEFER_READBACK (accumulator stays in HBM).
"""
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import cpuperformanceraytracer_amd as pt  # noqa: E402

W, H, S, B, K = 1920, 1080, 8, 8, 10
out = {}
for name, defer, pin in (("synchronous", False, False), ("pinned_pipelined", False, True),
                         ("deferred_readback", True, False)):
    pt.init(num_bounces=B, samples_per_frame=S, defer_readback=defer, pin_host=pin)
    buf = np.zeros((H, W, 3), np.float32)
    for _ in range(2):
        pt.DemofoxRenderScalar(buf, W, H, 3)
    t0 = time.perf_counter()
    for _ in range(K):
        pt.DemofoxRenderScalar(buf, W, H, 3)
    if defer:
        pt.readback(buf)
    dt = (time.perf_counter() - t0) / K
    out[name] = {"ms_per_call": dt * 1e3, "ray_samples_per_s": W * H * S * B / dt,
                 "primary_samples_per_s": W * H * S / dt}
print(json.dumps({"workload": f"{W}x{H}, {S} frames per call, {B} bounces, host buffer", **out}))
