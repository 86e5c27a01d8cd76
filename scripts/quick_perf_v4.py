"""Quick device timing of the v4 workload (1920x1080, 8 spp, 8 bounces, equirect 2k env); dev tool.
usage: quick_perf_v4.py [W H S B] [none|equirect|cubemap]"""
import json, os, sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch
from cpuperformanceraytracer_amd import _native as N
from cpuperformanceraytracer_amd.config import synthetic_env
from cpuperformanceraytracer_amd.device import count_v4_device, ensure_backend, render_v4_device, set_env_map
from cpuperformanceraytracer_amd.renderer import v4_config
W, H, S, B = 1920, 1080, 8, 8
if len(sys.argv) > 4:
    W, H, S, B = map(int, sys.argv[1:5])
mode = sys.argv[5] if len(sys.argv) > 5 else "equirect"
ensure_backend(0)
env_mode = {"none": N.PT_V4_ENV_NONE, "equirect": N.PT_V4_ENV_EQUIRECT, "cubemap": N.PT_V4_ENV_CUBEMAP}[mode]
v4_config(env_mode=env_mode, num_bounces=B)
use_env = env_mode != N.PT_V4_ENV_NONE
if use_env:
    env = synthetic_env() if env_mode == N.PT_V4_ENV_EQUIRECT else synthetic_env(6 * 512, 512)
    set_env_map(env, 0, B)
buf = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
cnt = count_v4_device(buf, W, H, frame_first=1, nframes=S, num_bounces=B, use_env=use_env)
import time
_t0 = time.perf_counter()   # device warm-up (clock ramp), as bench.py --device-warmup-ms
while time.perf_counter() - _t0 < float(os.environ.get("PT_QP_WARM_S", "0.08")):
    for i in range(3):
        render_v4_device(buf, W, H, frame_first=1 + S * (i + 1), nframes=S, num_bounces=B, use_env=use_env)
    torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
K = int(os.environ.get("PT_QP_K", "10"))
e0.record()
for i in range(K):
    render_v4_device(buf, W, H, frame_first=1 + S * (i + 4), nframes=S, num_bounces=B, use_env=use_env)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / K
print(json.dumps({"lib": os.environ.get("PT_MI355_LIB", "default"), "mode": mode, "W": W, "H": H, "spp": S, "B": B,
                  "ms_per_launch": ms, "ray_samples_per_s": W * H * S * B / ms * 1e3,
                  "segments_per_sample": cnt["segments"] / cnt["samples"],
                  "simd_eff": cnt["segments"] / cnt["lane_slots"]}))
