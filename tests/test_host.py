"""Host-side logic that needs no GPU: settings validation, tile lists, buffer layouts, argument
checks of the Python mirror of the reference interface."""
from __future__ import annotations

import numpy as np
import pytest

import cpuperformanceraytracer_amd as pt
from cpuperformanceraytracer_amd import config
from layouts import (interleaved_to_planar8, interleaved_to_tiled, planar8_to_interleaved,
                     tiled_to_interleaved)


def test_check_valid_settings_mirrors_application_cpp():
    # the reference's own defaults: 1280x720 in 10 x 15 tiles (global_preprocessor_flags.h:39-40,85-86)
    assert config.check_valid_settings(1280, 720) == []
    assert config.check_valid_settings(1920, 1080, 10, 15) == []      # 192 x 72 tiles
    assert any("tile width" in e for e in config.check_valid_settings(1000, 720, 10, 15))   # 100 % 8
    assert any("rows" in e for e in config.check_valid_settings(1280, 721, 10, 15))
    assert any("columns" in e for e in config.check_valid_settings(1288, 720, 12, 15))
    assert any("image width" in e for e in config.check_valid_settings(1284, 720, 3, 15))


def test_make_tiles_matches_simd_tiled_loop():
    tiles = pt.make_tiles(1280, 720, 10, 15)
    assert len(tiles) == 150
    # simd_tiled.cpp:549-571: TileX outer, TileY inner
    assert (tiles[0].TileX, tiles[0].TileY, tiles[1].TileX, tiles[1].TileY) == (0, 0, 0, 1)
    t = tiles[-1]
    assert (t.TileMinX, t.TileMaxX, t.TileMinY, t.TileMaxY) == (1152, 1279, 672, 719)
    cover = np.zeros((720, 1280), np.int32)
    for t in tiles:
        cover[t.TileMinY:t.TileMaxY + 1, t.TileMinX:t.TileMaxX + 1] += 1
    assert (cover == 1).all()


def test_planar8_layout_roundtrip_and_index_formula():
    w, h = 32, 3
    img = np.random.default_rng(0).random((h, w, 3), dtype=np.float32)
    p = interleaved_to_planar8(img)
    assert np.array_equal(planar8_to_interleaved(p, w, h), img)
    # simd.cpp:496-511: pixel (X,Y) channel c at (Y*W + (X & ~7))*3 + c*8 + (X & 7)
    for (x, y, c) in [(0, 0, 0), (9, 1, 2), (31, 2, 1)]:
        assert p[(y * w + (x & ~7)) * 3 + c * 8 + (x & 7)] == img[y, x, c]


def test_tiled_layout_roundtrip_and_index_formula():
    w, h, tw, th = 64, 12, 16, 4
    img = np.random.default_rng(1).random((h, w, 3), dtype=np.float32)
    t = interleaved_to_tiled(img, tw, th)
    assert np.array_equal(tiled_to_interleaved(t, w, h, tw, th), img)
    # simd_tiled.cpp:499-531
    for (x, y, c) in [(0, 0, 0), (17, 5, 2), (63, 11, 1), (40, 7, 0)]:
        tx, ty = x // tw, y // th
        lx, ly = x - tx * tw, y - ty * th
        idx = ty * th * w * 3 + tx * tw * th * 3 + (ly * tw + (lx & ~7)) * 3 + c * 8 + (lx & 7)
        assert t[idx] == img[y, x, c]


def test_buffer_validation_happens_before_any_device_call():
    from cpuperformanceraytracer_amd._native import PtError
    with pytest.raises(PtError):
        pt.DemofoxRenderScalar(np.zeros(12, np.float64), 2, 2, 3)
    with pytest.raises(PtError):
        pt.DemofoxRenderScalar(np.zeros(11, np.float32), 2, 2, 3)            # too small
    with pytest.raises(PtError):
        pt.DemofoxRenderScalar(np.zeros((3, 4, 3), np.float32)[:, ::2], 2, 3, 3)  # not contiguous


def test_workloads_match_baseline_configs():
    import json
    from pathlib import Path
    cfgs = json.loads((Path(__file__).resolve().parents[1] / "BASELINE.json").read_text())["configs"]
    c2 = config.CONFIGS["c2_1080p"]
    assert "1920×1080, 8 spp, 8 bounces" in cfgs[1]
    assert (c2.width, c2.height, c2.spp, c2.num_bounces) == (1920, 1080, 8, 8)
    assert c2.ray_samples == 1920 * 1080 * 8 * 8
    c3 = config.CONFIGS["c3_4k"]
    assert "3840×2160, 64 spp, 8 bounces" in cfgs[2]
    assert (c3.width, c3.height, c3.spp) == (3840, 2160, 64)
