"""Quick device timing + work counts of the v4 renderer (1920x1080, 8 spp, equirect env, the
reference's default flags, as bench.py's v4_1080p); dev tool.  Prints one JSON line."""
import json, os, sys, time
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch
from cpuperformanceraytracer_amd.config import synthetic_env
from cpuperformanceraytracer_amd.device import count_v4_device, render_v4_device, set_env_map
from cpuperformanceraytracer_amd.renderer import v4_config
W, H, S, B = 1920, 1080, 8, 8
if len(sys.argv) > 4:
    W, H, S, B = map(int, sys.argv[1:5])
set_env_map(synthetic_env(), 0, B)
v4_config(num_bounces=B, random_jitter=os.environ.get("PT_QP_RJ", "1") == "1")
buf = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
kw = dict(frame_first=1, nframes=S, num_bounces=B, use_env=True)
cnt = count_v4_device(buf, W, H, **kw)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.1:
    render_v4_device(buf, W, H, **kw)
    torch.cuda.synchronize()
K = int(os.environ.get("PT_QP_K", "40"))
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for i in range(K):
    render_v4_device(buf, W, H, frame_first=1 + S * i, nframes=S, num_bounces=B, use_env=True)
e1.record()
torch.cuda.synchronize()
print(json.dumps({"ct": os.environ.get("PT_MI355_NO_CT") != "1", "W": W, "H": H, "spp": S, "ms_per_launch": e0.elapsed_time(e1) / K,
                  "lane_eff": cnt["segments"] / max(1, cnt["lane_slots"]), "counts": cnt}))
