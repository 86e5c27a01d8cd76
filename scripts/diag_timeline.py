"""Per-wave / per-tile timeline of one launch (dev tool; diagnostic build).

Build the diagnostic library here:  bash scripts/build_variant.sh diag -DPT_DIAG=1  and run on the GPU box:
    PT_MI355_LIB=build/libpt_diag.so python scripts/diag_timeline.py [W H S B]
Prints the launch span, wave start/end skew, the idle lane-time at the end of the launch and what
the last tiles in flight were (pt_capi.cpp diag_dump layout: 4 u64 per wave + 32 tiles x 3 u64).
"""
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from cpuperformanceraytracer_amd.device import render_device  # noqa: E402

W, H, S, B = 1920, 1080, 8, 8
if len(sys.argv) > 4:
    W, H, S, B = map(int, sys.argv[1:5])
out = Path(os.environ.get("PT_DIAG_FILE", "gpurun_out/diag_timeline.bin"))
out.parent.mkdir(parents=True, exist_ok=True)
buf = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
t0 = time.perf_counter()
f = 1
while time.perf_counter() - t0 < 0.15:   # clock ramp + schedules built (async launches, no dump)
    for _ in range(20):
        render_device(buf, W, H, frame_first=f, nframes=S, num_bounces=B)
        f += S
    torch.cuda.synchronize()
for _ in range(20):                      # keep the clocks up right before the recorded launch
    render_device(buf, W, H, frame_first=f, nframes=S, num_bounces=B)
    f += S
os.environ["PT_DIAG_OUT"] = str(out)
for _ in range(int(os.environ.get("PT_DIAG_REPEAT", "1"))):   # the last one is analysed
    render_device(buf, W, H, frame_first=f, nframes=S, num_bounces=B)
    f += S
torch.cuda.synchronize()
del os.environ["PT_DIAG_OUT"]

raw = np.fromfile(out, np.uint64)
waves = raw[:4 * 65536].reshape(65536, 4)
tl = raw[4 * 65536:].reshape(65536, 32, 3)
alive = waves[:, 0] != 0
nw = int(alive.sum())
wv = waves[alive].astype(np.int64)
birth, death, ntiles, niter = wv[:, 0], wv[:, 1], wv[:, 2], wv[:, 3]
r0 = birth.min()
span = (death.max() - r0) * 0.01   # 100 MHz realtime ticks -> us
b_us = (birth - r0) * 0.01
d_us = (death - r0) * 0.01
idle_end = (span - d_us).sum() / (nw * span)
idle_start = b_us.sum() / (nw * span)
res = {"W": W, "H": H, "spp": S, "bounces": B, "waves": nw, "span_us": span,
       "birth_us_pct": np.percentile(b_us, [0, 50, 90, 99, 100]).round(1).tolist(),
       "death_us_pct": np.percentile(d_us, [0, 1, 10, 50, 90, 99, 100]).round(1).tolist(),
       "idle_frac_end": round(float(idle_end), 4), "idle_frac_start": round(float(idle_start), 4),
       "tiles_per_wave_pct": np.percentile(ntiles, [0, 50, 100]).tolist()}
# tile records of the waves (first 32 tiles of each)
t = tl[alive][:, :, :].astype(np.int64)
nt = np.minimum(ntiles, 32)
rows = []
for i in range(nw):
    for k in range(int(nt[i])):
        s_, e_, idw = t[i, k]
        rows.append(((s_ - r0) * 0.01, (e_ - r0) * 0.01, idw >> 32, idw & 0xffffffff))
a = np.array(rows)
np.savez_compressed(str(out.with_suffix(".npz")), tiles=a, birth=b_us, death=d_us,
                    wave=np.repeat(np.arange(nw), nt))
dur = a[:, 1] - a[:, 0]
res["tile_us_pct"] = np.percentile(dur, [50, 90, 99, 100]).round(1).tolist()
res["tile_work_pct"] = np.percentile(a[:, 3], [50, 90, 99, 100]).tolist()
res["us_per_work_iter"] = round(float(dur.sum() / a[:, 3].sum()), 3)
# tiles without pool iterations (work 1: every camera ray missed -- sky tiles and all-miss tiles):
# their share of the recorded wave-time and their duration (latency-bound: load, lerps, store)
sky = a[:, 3] == 1
res["work1_tiles"] = int(sky.sum())
res["work1_wave_time_frac"] = round(float(dur[sky].sum() / (nw * span)), 4)
res["work1_tile_us_pct"] = np.percentile(dur[sky], [10, 50, 90]).round(2).tolist() if sky.any() else []
res["recorded_tiles_frac"] = round(float(len(a) / max(1, ntiles.sum())), 4)
late = a[:, 1] > 0.9 * span
res["tiles_ending_last10pct"] = int(late.sum())
res["late_tile_start_us_pct"] = np.percentile(a[late, 0], [0, 50, 100]).round(1).tolist() if late.any() else []
res["late_tile_work_pct"] = np.percentile(a[late, 3], [0, 50, 100]).tolist() if late.any() else []
# time at which the queue ran dry: the last tile start
res["last_tile_start_us"] = round(float(a[:, 0].max()), 1)
# busy-wave count over time (20 bins)
edges = np.linspace(0, span, 21)
busy = [int(((b_us <= e) & (d_us > e)).sum()) for e in edges[1:-1]]
res["busy_waves_at_5pct_steps"] = busy
print(json.dumps(res))
