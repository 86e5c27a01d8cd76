"""The CPU baseline's AVX2 port of demofox_path_tracing_simt_pooled.cpp (oracle/pt_cpu_simd.c).

Not a parity checker: the reference's SIMD files draw their random numbers differently from the
scalar path (one state per lane, vector sin/cos), so images agree only statistically.  These checks
make sure bench.py times a renderer of the same scene that converges to the same image.
"""
from __future__ import annotations

import numpy as np
import pytest

from layouts import tiled_to_interleaved
from oracle import pyoracle as po

pytestmark = pytest.mark.skipif(not po.simd_supported(), reason="needs AVX2 + FMA")


def test_simd_port_converges_to_the_scalar_image():
    w, h, frames = 160, 120, 96
    b = po.render_simd_tiled(w, h, 5, 15, nframes=frames, num_bounces=8)
    img = tiled_to_interleaved(b, w, h, w // 5, h // 15)
    ref = po.render(w, h, nframes=frames, num_bounces=8)
    assert np.all(np.isfinite(img))
    m, mr = img.mean(axis=(0, 1)), ref.mean(axis=(0, 1))
    assert np.allclose(m, mr, rtol=0.02), (m, mr)
    # the open front is exactly the ambient in both (no randomness on a first-segment miss); the
    # SIMD camera uses FMA dot products (mathlib.h:145), so a few edge pixels may flip
    sky = ref.reshape(-1, 3)[:, 0] == ref.reshape(-1, 3)[0, 0]
    same = (img.reshape(-1, 3)[sky] == ref.reshape(-1, 3)[sky]).all(axis=1)
    assert sky.sum() > 1000 and same.mean() > 0.99, same.mean()


def test_simd_port_threads_and_frames():
    w, h = 64, 32
    a = po.render_simd_tiled(w, h, 2, 2, nframes=3, num_bounces=4, nthreads=1)
    b = po.render_simd_tiled(w, h, 2, 2, nframes=3, num_bounces=4, nthreads=4)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    c = po.render_simd_tiled(w, h, 2, 2, nframes=1, num_bounces=4)
    c = po.render_simd_tiled(w, h, 2, 2, frame_first=2, nframes=2, num_bounces=4, buf=c)
    assert np.array_equal(a.view(np.uint32), c.view(np.uint32))
    with pytest.raises(ValueError):
        po.render_simd_tiled(60, 32, 2, 2)   # tile width not a multiple of 8
