"""Per-frame cadence of the shipping host (dev tool): DemofoxRenderOptV4 on host buffers, as
ApplicationState::Render calls it (Application.cpp:460-477): 1280x720 (global_preprocessor_flags.h
RENDER_BUFFER_PIXEL_*), one frame per call, 10 x 15 tiles, OUTPUT_TO_SCREEN into a u32 screen buffer.
Modes: synchronous (accumulator H2D + D2H every call), deferred readback (accumulator stays in HBM,
only the screen pixels come back), pinned (PT_FLAG_PIN_HOST)."""
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import cpuperformanceraytracer_amd as pt  # noqa: E402
from cpuperformanceraytracer_amd.config import synthetic_env  # noqa: E402

W, H, K = (int(sys.argv[1]), int(sys.argv[2]), 30) if len(sys.argv) > 2 else (1280, 720, 30)
env = synthetic_env()
tex = pt.texture(env, env.shape[1], env.shape[0], 3)
out = {}
for name, defer, pin in (("synchronous", False, False), ("deferred_readback", True, False),
                         ("pinned", False, True), ("pinned_deferred", True, True)):
    pt.init(defer_readback=defer, pin_host=pin)
    pt.v4_config()
    pt.InitializeGlobalRenderResources()
    buf = np.zeros(W * H * 3, np.float32)
    screen = np.zeros(W * H, np.uint32)
    for _ in range(3):
        pt.DemofoxRenderOptV4(buf, W, H, 10, 15, W // 10, H // 15, 3, tex, screen)
    t0 = time.perf_counter()
    for _ in range(K):
        pt.DemofoxRenderOptV4(buf, W, H, 10, 15, W // 10, H // 15, 3, tex, screen)
    dt = (time.perf_counter() - t0) / K
    out[name] = {"ms_per_frame": dt * 1e3, "fps": 1.0 / dt, "ray_samples_per_s": W * H * 8 / dt}
print(json.dumps({"workload": f"{W}x{H}, 1 frame per DemofoxRenderOptV4 call, 8 bounces, screen pixels", **out}))
