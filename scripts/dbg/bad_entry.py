"""Debug: the PT_MI355_TEST_BAD_ENTRY hook, launch by launch."""
import os, sys
sys.path.insert(0, os.getcwd())
import torch
import cpuperformanceraytracer_amd as pt
from cpuperformanceraytracer_amd import _native as N
from cpuperformanceraytracer_amd.device import JobLauncher
imgs = {}
for hook in ("-1", "7", "0"):
    os.environ["PT_MI355_TEST_BAD_ENTRY"] = hook
    pt.init(num_bounces=8)
    W, H, S = 640, 360, 8
    buf = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda:0")
    L = JobLauncher(buf, W, H, nframes=S, num_bounces=8, stream=torch.cuda.current_stream())
    for k in range(4):
        L(1 + k * S)
        torch.cuda.synchronize()
        rc = N.load().pt_check_device_errors()
        print("hook", hook, "launch", k, "rc", rc, N.load().pt_last_error().decode() if rc else "", flush=True)
    imgs[hook] = buf.cpu()
    pt.shutdown()
for h in ("7", "0"):
    d = (imgs[h] != imgs["-1"]).reshape(-1, 3).any(1)
    print("hook", h, "pixels differing from no hook:", int(d.sum()))
