"""Dev tool: v4 kernel vs oracle on a small image, per bounce count (first mismatching pixel)."""
import os
import sys

sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
import numpy as np  # noqa: E402
import torch  # noqa: E402

from conftest import mismatch_report  # noqa: E402
from oracle import pyoracle as po  # noqa: E402
import cpuperformanceraytracer_amd as pt  # noqa: E402
from cpuperformanceraytracer_amd import _native as N  # noqa: E402
from cpuperformanceraytracer_amd.device import ensure_backend, render_v4_device  # noqa: E402

ensure_backend(0)
w, h = 160, 96
for B in (0, 1, 8):
    pt.v4_config(env_mode=N.PT_V4_ENV_NONE, num_bounces=B)
    buf = torch.zeros(w * h * 3, dtype=torch.float32, device='cuda')
    render_v4_device(buf, w, h, frame_first=1, nframes=1, num_bounces=B)
    got = buf.cpu().numpy().reshape(h, w, 3)
    ref = po.render4(w, h, nframes=1, env=None, num_bounces=B)
    print(os.environ.get('PT_MI355_LIB', 'default'), 'B', B, mismatch_report(got, ref))
    bad = np.nonzero((got.view('u4') != ref.view('u4')).any(2))
    if len(bad[0]):
        y, x = bad[0][0], bad[1][0]
        print('  pixel', y, x, got[y, x], ref[y, x])
