"""Dev tool (round 5): full-image comparison of the presenting continuous-tiles kernel's accumulator
with the plain kernel's (3 x 8-frame JobLauncher launches, 1920x1080, 8 bounces).  Prints one JSON line."""
import json
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import cpuperformanceraytracer_amd as pt  # noqa: E402
from cpuperformanceraytracer_amd.device import JobLauncher  # noqa: E402

W, H, B, S = 1920, 1080, 8, 8
L = int(os.environ.get("PT_DBG_LAUNCHES", "3"))
out = {}
for mode in ("plain", "present"):
    pt.init(num_bounces=8)
    buf = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda:0")
    kw = {}
    if mode == "present":
        kw = dict(pixels=torch.zeros(H * W, dtype=torch.int32, device="cuda:0"), pixel_format=0)
    launch = JobLauncher(buf, W, H, nframes=S, num_bounces=B, **kw)
    for k in range(L):
        launch(1 + k * S)
    torch.cuda.synchronize()
    out[mode] = buf.cpu().numpy().reshape(H, W, 3)
bad = np.argwhere((out["plain"].view(np.uint32) != out["present"].view(np.uint32)).any(axis=2))
print(json.dumps({"env": {k: v for k, v in os.environ.items() if k.startswith("PT_MI355")}, "bad_px": int(len(bad)),
                  "first": [[int(y), int(x)] for y, x in bad[:30]],
                  "plain_vs_present": [[out["plain"][y, x].tolist(), out["present"][y, x].tolist()] for y, x in bad[:3]]}),
      flush=True)
