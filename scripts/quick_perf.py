"""Quick device timing of the headline workload (1920x1080, 8 spp, 8 bounces); dev tool."""
import sys, time, json
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch
from cpuperformanceraytracer_amd.device import render_device, count_device
W, H, S, B = 1920, 1080, 8, 8
if len(sys.argv) > 1:
    W, H, S, B = map(int, sys.argv[1:5])
ENV = len(sys.argv) > 5 and sys.argv[5] == "env"
if ENV:
    from cpuperformanceraytracer_amd.config import synthetic_env
    from cpuperformanceraytracer_amd.device import set_env_map
    set_env_map(synthetic_env(), 0, B)
buf = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
count_device(buf, W, H, frame_first=1, nframes=S, num_bounces=B, use_env=ENV)   # warm
import os
_t0 = time.perf_counter()   # device warm-up (clock ramp), as bench.py --device-warmup-ms
while time.perf_counter() - _t0 < float(os.environ.get("PT_QP_WARM_S", "0.08")):
    render_device(buf, W, H, frame_first=1, nframes=S, num_bounces=B, use_env=ENV)
    torch.cuda.synchronize()
c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
c0.record()
cnt = count_device(buf, W, H, frame_first=1, nframes=S, num_bounces=B, use_env=ENV)
c1.record()
torch.cuda.synchronize()
count_ms = c0.elapsed_time(c1)
for i in range(3):
    render_device(buf, W, H, frame_first=1 + S * (i + 1), nframes=S, num_bounces=B, use_env=ENV)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
K = int(os.environ.get("PT_QP_K", "10"))
e0.record()
for i in range(K):
    render_device(buf, W, H, frame_first=1 + S * (i + 4), nframes=S, num_bounces=B, use_env=ENV)
e1.record(); torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / K
print(json.dumps({"lib": __import__("os").environ.get("PT_MI355_LIB", "default"),
                  "ct": __import__("os").environ.get("PT_MI355_NO_CT") != "1", "env": ENV, "W": W, "H": H, "spp": S, "B": B, "ms_per_launch": ms,
                  "primary_samples_per_s": W * H * S / ms * 1e3, "ray_samples_per_s": W * H * S * B / ms * 1e3,
                  "segments_per_sample": cnt["segments"] / cnt["samples"],
                  "ref_segments_per_sample": (cnt["segments"] - cnt["primary"]) / cnt["samples"] + 1,
                  "simd_eff": cnt["segments"] / max(1, cnt["lane_slots"]), "counts": cnt, "count_launch_ms": count_ms}))
