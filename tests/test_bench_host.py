"""Host logic of bench.py (no GPU): the global image of an N-rank weak-scaling run keeps the
1920x1080 view (aspect ratio) and gives every rank ~1920x1080 pixels of interleaved rows."""
from __future__ import annotations

import sys
from pathlib import Path

import pytest

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from cpuperformanceraytracer_amd.shard import rows_of  # noqa: E402


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8, 16])
def test_weak_image_keeps_view_and_per_rank_pixels(world):
    W, H = 1920, 1080
    Wg, Hg = bench.weak_image(W, H, world)
    assert Wg % 8 == 0
    assert abs((Wg / Hg) / (W / H) - 1.0) < 2e-3          # same aspect -> same camera view
    assert abs(Wg * Hg / (world * W * H) - 1.0) < 1e-2     # N x the pixels
    counts = [rows_of(r, world, Hg)[2] * Wg for r in range(world)]
    assert sum(counts) == Wg * Hg
    assert max(counts) - min(counts) <= Wg                 # balanced to one row
    if world == 1:
        assert (Wg, Hg) == (W, H)
    if world == 4:
        assert (Wg, Hg) == (3840, 2160)
