"""Dev tool (round 5): where do late-split launches differ from the oracle?  Plain and presenting
JobLauncher series of 3 x 8-frame launches at 1920x1080 (8 bounces); rows 0::54 against the oracle.
Run with PT_MI355_LATE_SPLIT set; prints one JSON line per series."""
import json
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tests"))
import torch  # noqa: E402

import cpuperformanceraytracer_amd as pt  # noqa: E402
from cpuperformanceraytracer_amd.device import JobLauncher  # noqa: E402
from oracle import pyoracle  # noqa: E402

W, H, B, S = 1920, 1080, 8, 8
L = int(os.environ.get("PT_DBG_LAUNCHES", "3"))
ref = pyoracle.render(W, H, nframes=L * S, num_bounces=B, row_start=0, row_stride=54, nrows=20)
for mode in ("plain", "present", "plain", "present"):
    pt.init(num_bounces=8)
    buf = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda:0")
    kw = {}
    if mode == "present":
        kw = dict(pixels=torch.zeros(H * W, dtype=torch.int32, device="cuda:0"), pixel_format=0)
    launch = JobLauncher(buf, W, H, nframes=S, num_bounces=B, **kw)
    for k in range(L):
        launch(1 + k * S)
    torch.cuda.synchronize()
    acc = buf.cpu().numpy().reshape(H, W, 3)[0::54]
    bad = np.argwhere((acc.view(np.uint32) != ref.view(np.uint32)).any(axis=2))
    ys = sorted(set(int(r) * 54 for r, _ in bad))
    xs = [int(x) for _, x in bad[:20]]
    # a missing / doubled half: compare against the oracle of fewer / more frames
    print(json.dumps({"mode": mode, "late_split": os.environ.get("PT_MI355_LATE_SPLIT"), "bad_px": int(len(bad)),
                      "rows": ys[:20], "rows_mod8": sorted(set(y % 8 for y in ys)), "xs": xs,
                      "tiles": sorted(set((y // 8, x // 8) for y, x in ((int(r) * 54, int(x)) for r, x in bad)))[:20]}),
          flush=True)
