"""Per-frame cadence of the work-queue host path (dev tool): every frame, all NTX x NTY tiles of a
host buffer go through MakeWorkQueue / AddWorkQueueEntry / CompleteAllWork (work_queue.cpp:37-108,
the v4 host's RenderTile entries, v4 :1696-1721), 10 x 15 tiles as Application.cpp uses.
Modes: synchronous (accumulator H2D + D2H every call) and pinned (PT_FLAG_PIN_HOST: band pipeline).
usage: host_queue_perf.py [W H]"""
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import cpuperformanceraytracer_amd as pt  # noqa: E402
from cpuperformanceraytracer_amd import _native as N  # noqa: E402
from cpuperformanceraytracer_amd.config import synthetic_env  # noqa: E402

W, H = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (1920, 1080)
K = 30
env = synthetic_env()
out = {}
for renderer in ("diffuse", "v4"):
    for name, pin in (("synchronous", False), ("pinned", True)):
        if renderer == "v4":
            pt.init(pin_host=pin)
            pt.v4_config(env_mode=N.PT_V4_ENV_EQUIRECT)
            q = pt.MakeWorkQueue(N.PT_RENDERER_V4)
            begin = pt.v4_begin_frame
        else:
            pt.init(num_bounces=8, pin_host=pin)
            q = pt.MakeWorkQueue()
            begin = pt.BeginFrame
        pt.set_env_map(env)
        buf = np.zeros(W * H * 3, np.float32)
        bi = pt.RenderBufferInfo(buf, W, H, 3)
        tiles = pt.make_tiles(W, H, 10, 15)

        add_s = [0.0]

        def frame():
            begin()
            t = time.perf_counter()
            for tile in tiles:
                pt.AddWorkQueueEntry(q, bi, tile)
            add_s[0] += time.perf_counter() - t
            pt.CompleteAllWork(q)

        for _ in range(3):
            frame()
        add_s[0] = 0.0
        t0 = time.perf_counter()
        for _ in range(K):
            frame()
        dt = (time.perf_counter() - t0) / K
        out[f"{renderer}_{name}"] = {"ms_per_frame": dt * 1e3, "ray_samples_per_s": W * H * 8 / dt,
                                     "python_add_entries_ms": add_s[0] / K * 1e3}
        # the frame call of the same renderer on the same buffer, for comparison
        if renderer == "v4":
            tex = pt.texture(env, env.shape[1], env.shape[0], 3)
            call = lambda: pt.DemofoxRenderOptV4(buf, W, H, 10, 15, W // 10, H // 15, 3, tex, None)  # noqa: E731
        else:
            call = lambda: pt.DemofoxRenderSimdTiled(buf, W, H, 10, 15, W // 10, H // 15, 3)  # noqa: E731
        for _ in range(3):
            call()
        t0 = time.perf_counter()
        for _ in range(K):
            call()
        dt = (time.perf_counter() - t0) / K
        out[f"{renderer}_{name}"]["frame_call_ms"] = dt * 1e3
        if pin:
            pt.unpin_host(buf)
print(json.dumps({"workload": f"{W}x{H}, 1 frame per CompleteAllWork of 10x15 RenderTile entries, 8 bounces", **out}))
