"""GPU parity at the full sizes of BASELINE.json configs[2] (4K, 64 spp) and configs[4] (8K, 256 spp
on 8 GPUs -- here one rank's shard), where a whole-frame oracle run would take minutes.

Checked through properties that hold for the reference's algorithm at any size, plus bit-exact
sampled rows against the oracle:
  * sampled rows == oracle rows (the oracle renders just those rows: row_start / row_stride);
  * launch splitting: 64 frames in one launch == 4 launches of 16 (frames are sequential in the
    reference -- DemofoxRenderScalar's `iFrame += 1` per call, scalar.cpp:798-812);
  * determinism: the same launch twice gives the same bits;
  * row shards (the multi-GPU decomposition) reassemble to the full image, bit for bit.
"""
from __future__ import annotations

import numpy as np
import pytest

from conftest import bits_equal, mismatch_report
from oracle import pyoracle

pytestmark = pytest.mark.gpu


def _render(W, H, frame_first, nframes, B, buf=None, **rows):
    import torch
    from cpuperformanceraytracer_amd.device import render_device
    nrows = rows.get("nrows", H)
    if buf is None:
        buf = torch.zeros(nrows * W * 3, dtype=torch.float32, device="cuda:0")
    render_device(buf, W, H, frame_first=frame_first, nframes=nframes, num_bounces=B, **rows)
    return buf


def test_config3_4k_64spp():
    import torch
    W, H, S, B = 3840, 2160, 64, 8
    full = _render(W, H, 1, S, B)
    split = torch.zeros_like(full)
    for k in range(4):
        _render(W, H, 1 + 16 * k, 16, B, buf=split)
    again = _render(W, H, 1, S, B)
    torch.cuda.synchronize()
    a, b, c = (t.cpu().numpy().reshape(H, W, 3) for t in (full, split, again))
    assert bits_equal(a, b), "launch splitting changed the result: " + mismatch_report(a, b)
    assert bits_equal(a, c), "non-deterministic: " + mismatch_report(a, c)
    assert np.isfinite(a).all()
    rows = list(range(7, H, 135))                                      # 16 rows, 3.9 M samples
    ref = pyoracle.render(W, H, nframes=S, num_bounces=B, row_start=7, row_stride=135, nrows=len(rows))
    assert bits_equal(a[rows], ref), mismatch_report(a[rows], ref)
    # row shards of the multi-GPU decomposition (4 ranks, interleaved rows) reassemble exactly
    from cpuperformanceraytracer_amd.shard import max_rows, rows_of
    world = 4
    shard = torch.zeros(max_rows(world, H) * W * 3, dtype=torch.float32, device="cuda:0")
    for r in range(world):
        rs, st, n = rows_of(r, world, H)
        shard.zero_()
        _render(W, H, 1, S, B, buf=shard, row_start=rs, row_stride=st, nrows=n)
        torch.cuda.synchronize()
        got = shard[: n * W * 3].cpu().numpy().reshape(n, W, 3)
        assert bits_equal(got, a[rs::st][:n]), (r, mismatch_report(got, a[rs::st][:n]))


def test_config5_rank_shard_8k_256spp():
    """configs[4]: 7680x4320, 256 spp, 8 bounces over 8 GPUs -- rank 5's shard (540 interleaved
    rows, 1.06 G samples, the per-GPU work of the scaling run), sampled rows vs the oracle."""
    import torch
    from cpuperformanceraytracer_amd.shard import max_rows, rows_of
    W, H, S, B, world, rank = 7680, 4320, 256, 8, 8, 5
    rs, st, n = rows_of(rank, world, H)
    assert n == 540
    buf = torch.zeros(max_rows(world, H) * W * 3, dtype=torch.float32, device="cuda:0")
    _render(W, H, 1, S, B, buf=buf, row_start=rs, row_stride=st, nrows=n)
    torch.cuda.synchronize()
    img = buf[: n * W * 3].cpu().numpy().reshape(n, W, 3)
    assert np.isfinite(img).all()
    local = [3, 271, 539]                                             # shard rows -> global rs + k*st
    for k in local:
        ref = pyoracle.render(W, H, nframes=S, num_bounces=B, row_start=rs + k * st, row_stride=1, nrows=1)
        assert bits_equal(img[k:k + 1], ref), (k, mismatch_report(img[k:k + 1], ref))


def test_scheduled_launches_match_oracle():
    """The tile schedule (longest tiles first, built from the previous launches' costs and rebuilt
    every 64 launches) changes only the order tiles are processed in: 66 progressive 1-frame
    launches of one geometry -- unscheduled, scheduled, rebuilt -- equal the oracle bit for bit."""
    import torch
    W, H, B, K = 1280, 720, 8, 66
    buf = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda:0")
    for k in range(K):
        _render(W, H, 1 + k, 1, B, buf=buf)
    torch.cuda.synchronize()
    got = buf.cpu().numpy().reshape(H, W, 3)
    ref = pyoracle.render(W, H, nframes=K, num_bounces=B)
    assert bits_equal(got, ref), mismatch_report(got, ref)


@pytest.mark.parametrize("pool,env,frames", [("ct", False, 2), ("ct", False, 12), ("body", False, 2),
                                             ("body", False, 12), ("ring", False, 48), ("body", True, 3),
                                             ("ct", True, 3), ("ct", True, 12)])
def test_split_schedules_match_oracle(monkeypatch, pool, env, frames):
    """Split tiles (pt_tile_queue.h: a scheduled launch queues a tile that costs more than 1/split
    of a wave's share of the launch as its two halves, rows 0-3 and 4-7, taken by any two waves)
    change only which wave traces which pixels.  PT_MI355_SPLIT=100000 (read by pt_init) splits
    every tile of cost >= 2 from the second launch on; three launches of one geometry -- whole,
    split, split -- equal the oracle bit for bit on the continuous-tiles pool (ct), the chunked
    pool (body: PT_MI355_NO_CT=1), the ring pool (>= 48 frames) and the env kernels (ct, body)."""
    import torch
    import cpuperformanceraytracer_amd as pt
    from cpuperformanceraytracer_amd.device import render_device, set_env_map
    monkeypatch.setenv("PT_MI355_SPLIT", "100000")
    if pool != "ct":
        monkeypatch.setenv("PT_MI355_NO_CT", "1")
    W, H, B, K = 256, 128, 8, 3              # 512 tiles: scheduled
    pt.init(num_bounces=B)
    envmap = None
    if env:
        rng = np.random.default_rng(5)
        envmap = (rng.random((16, 32, 3), dtype=np.float32) * 4.0 + 0.01).astype(np.float32)
        set_env_map(envmap, 0, B)
    buf = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda:0")
    for k in range(K):
        render_device(buf, W, H, frame_first=1 + k * frames, nframes=frames, num_bounces=B, use_env=env)
    torch.cuda.synchronize()
    got = buf.cpu().numpy().reshape(H, W, 3)
    ref = pyoracle.render(W, H, nframes=K * frames, num_bounces=B, env=envmap)
    assert bits_equal(got, ref), mismatch_report(got, ref)
    pt.shutdown()


@pytest.mark.parametrize("waves", ["5", "6", "0"])
def test_ct_occupancy_variants_match_oracle(monkeypatch, waves):
    """The diffuse continuous-tiles kernel at 5 and 6 waves per SIMD (PT_MI355_CT_WAVES, read by
    pt_init) runs the same per-pixel code, and "0" -- the per-geometry timing, which times the arms
    (5 / 6 waves, and 6 waves at 45 % back claims for launches that take them) on a geometry's first
    12-18 scheduled launches in palindromic order, then keeps the fastest -- changes the grid between
    the launches of one accumulation: 12 launches of 2 frames of one scheduled geometry equal the
    oracle bit for bit in every mode (tests/test_gpu_regime.py: the same at bench sizes, including
    launches after the pick)."""
    import torch
    import cpuperformanceraytracer_amd as pt
    from cpuperformanceraytracer_amd.device import render_device
    monkeypatch.setenv("PT_MI355_CT_WAVES", waves)
    W, H, B, K, frames = 256, 128, 8, 12, 2   # 512 tiles: scheduled
    pt.init(num_bounces=B)
    buf = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda:0")
    for k in range(K):
        render_device(buf, W, H, frame_first=1 + k * frames, nframes=frames, num_bounces=B)
    torch.cuda.synchronize()
    got = buf.cpu().numpy().reshape(H, W, 3)
    ref = pyoracle.render(W, H, nframes=K * frames, num_bounces=B)
    assert bits_equal(got, ref), mismatch_report(got, ref)
    pt.shutdown()
