"""Does recording a timing event pair around every launch (bench.py's per-step kernel timing) add to
the wall time per step?  Dev tool: K back-to-back launches of the headline workload, timed by two
bracketing events, with and without per-launch event pairs, interleaved over several rounds."""
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402
from cpuperformanceraytracer_amd.device import render_device  # noqa: E402

W, H, S, B = 1920, 1080, 8, 8
K = int(os.environ.get("PT_EO_K", "100"))
buf = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
stream = torch.cuda.current_stream()
frame = 1
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.15:   # clock ramp
    render_device(buf, W, H, frame_first=frame, nframes=S, num_bounces=B, stream=stream)
    frame += S
    torch.cuda.synchronize()
res = {"per_step_events": [], "bracket_only": []}
for rnd in range(6):
    for mode in ("per_step_events", "bracket_only"):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record(stream)
        for k in range(K):
            if mode == "per_step_events":
                ev[k][0].record(stream)
            render_device(buf, W, H, frame_first=frame, nframes=S, num_bounces=B, stream=stream)
            if mode == "per_step_events":
                ev[k][1].record(stream)
            frame += S
        b.record(stream)
        torch.cuda.synchronize()
        total = a.elapsed_time(b) / K
        kern = sum(x.elapsed_time(y) for x, y in ev) / K if mode == "per_step_events" else None
        res[mode].append({"ms_per_step": total, "kernel_ms": kern})
print(json.dumps({"K": K, **{m: {"ms_per_step": [round(r["ms_per_step"], 5) for r in v],
                                 "kernel_ms": [round(r["kernel_ms"], 5) for r in v if r["kernel_ms"]]}
                             for m, v in res.items()}}))
