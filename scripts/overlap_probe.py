"""Upper bound of overlapping consecutive launches (dev probe).

Serial: K launches of the c2 job on one stream (the bench's loop).  Two: the same K launches
alternating over two streams and two independent buffers (no dependency between them), so a launch's
blocks fill the CUs its predecessor's finished waves free.  Needs PT_MI355_CT_AREAS2=1 (a slot area
per stream) and a fixed launch variant (PT_MI355_CT_WAVES, PT_MI355_BACK).  Prints ms per launch.
"""
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from cpuperformanceraytracer_amd.device import JobLauncher  # noqa: E402

W, H, S, B = 1920, 1080, 8, 8
if len(sys.argv) > 1:
    W, H, S, B = map(int, sys.argv[1:5])
K = int(os.environ.get("PT_OP_K", "200"))
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
bufs = [torch.zeros(W * H * 3, dtype=torch.float32, device="cuda") for _ in range(2)]
la = JobLauncher(bufs[0], W, H, nframes=S, num_bounces=B, stream=sa)
lb = JobLauncher(bufs[1], W, H, nframes=S, num_bounces=B, stream=sb)
ls = JobLauncher(bufs[0], W, H, nframes=S, num_bounces=B, stream=sa)
frame = [1, 1]


def serial(k):
    for _ in range(k):
        ls(frame[0])
        frame[0] += S


def two(k):
    for i in range(k):
        if i & 1:
            lb(frame[1])
            frame[1] += S
        else:
            la(frame[0])
            frame[0] += S


def timed(fn, k):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn(k)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / k


t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.3:   # clocks, schedules
    serial(20)
    two(20)
    torch.cuda.synchronize()
res = {"W": W, "H": H, "spp": S, "K": K, "serial": [], "two": []}
for _ in range(3):
    res["serial"].append(round(timed(serial, K), 5))
    res["two"].append(round(timed(two, K), 5))
res["gain"] = round(1 - min(res["two"]) / min(res["serial"]), 4)
print(json.dumps(res), flush=True)
