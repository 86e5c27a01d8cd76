"""Per-launch kernel time over the first 400 launches of a process (dev tool): shows the device clock ramp
that bench.py's --device-warmup-ms covers."""
import sys, json
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch
from cpuperformanceraytracer_amd.device import ensure_backend, render_device
ensure_backend(0, 8)
W, H = 1920, 1080
buf = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(400)]
f = 1
for k in range(400):
    ev[k][0].record()
    render_device(buf, W, H, frame_first=f, nframes=8, num_bounces=8)
    ev[k][1].record()
    f += 8
torch.cuda.synchronize()
ms = [a.elapsed_time(b) for a, b in ev]
for i in range(0, 400, 20):
    seg = ms[i:i + 20]
    print(f"steps {i:3d}-{i+19:3d}: mean {sum(seg)/len(seg):.4f} min {min(seg):.4f} max {max(seg):.4f}")
