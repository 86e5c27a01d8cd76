"""Chained launches (pt_render_device_chain) against the oracle.

A chained launch may run overlapped with the previous chained launch of its geometry (pt_capi.cpp
launch_chain: two streams, a stream gate on the predecessor's started blocks, per half-tile epochs that
a launch waits for before it touches a tile's pixels -- render_body_ct).  The result must be the
reference's frame loop bit for bit: every pixel's frames folded in order by the progressive lerp of
demofox_path_tracing_scalar.cpp:812 (DemofoxRenderScalar :785-820).  These tests drive chained series
(the bench's regime, other geometries and frame counts, the env kernel, a row shard, forced waits,
chained launches mixed with plain and counted ones) and compare with oracle/pt_oracle.c; each also
checks that launches did continue the overlap (pt_chain_counts), so the overlapped path is the one
tested.
"""
from __future__ import annotations

import numpy as np
import pytest

from conftest import bits_equal, mismatch_report
from oracle import pyoracle

pytestmark = pytest.mark.gpu


@pytest.fixture
def fresh(monkeypatch):
    """A fresh library state initialised under the test's environment."""
    import cpuperformanceraytracer_amd as pt

    def init(B, **envs):
        for k, v in envs.items():
            monkeypatch.setenv(k, v)
        pt.init(num_bounces=B)
    yield init
    pt.shutdown()
    for k in ("PT_MI355_CT_WAVES", "PT_MI355_BACK", "PT_MI355_TEST_CHAIN_DELAY", "PT_MI355_V4_CT",
              "PT_MI355_TEST_CHAIN_POLLS"):
        monkeypatch.delenv(k, raising=False)


def _series(W, H, B, S, launches, *, row_start=0, row_stride=1, nrows=None, env=False, plain_at=(), count_at=(),
            sync_at=(), v4=False):
    """`launches` launches of S frames (frames 1 .. launches*S) into a zeroed buffer on the current
    stream: chained (JobLauncher(chain=True), as bench.py), except a plain pt_render_device launch at
    the indices in plain_at; a counted launch on a scratch buffer after the indices in count_at and a
    device synchronisation after those in sync_at.  Returns (image, frames, chain counts)."""
    import torch
    from cpuperformanceraytracer_amd.device import (JobLauncher, chain_counts, check_device_errors, count_device,
                                                    count_v4_device)
    nrows = H if nrows is None else nrows
    stream = torch.cuda.current_stream()
    buf = torch.zeros(nrows * W * 3, dtype=torch.float32, device="cuda:0")
    scratch = torch.zeros_like(buf)
    kw = dict(nframes=S, num_bounces=B, row_start=row_start, row_stride=row_stride, nrows=nrows, use_env=env,
              stream=stream)
    chained, plain = JobLauncher(buf, W, H, chain=True, v4=v4, **kw), JobLauncher(buf, W, H, v4=v4, **kw)
    cfn = count_v4_device if v4 else count_device
    c0 = chain_counts()
    frame = 1
    for k in range(launches):
        (plain if k in plain_at else chained)(frame)
        if k in count_at:
            cfn(scratch, W, H, frame_first=frame, **{a: kw[a] for a in kw if a != "nframes"}, nframes=S)
        if k in sync_at:
            torch.cuda.synchronize()
        frame += S
    torch.cuda.synchronize()
    check_device_errors()
    c1 = chain_counts()
    counts = {k: c1[k] - c0[k] for k in c1}
    return buf.cpu().numpy().reshape(nrows, W, 3), frame - 1, counts


def _check_rows(img, W, H, frames, B, local_rows, *, row_start=0, row_stride=1, env=None):
    for k in local_rows:
        y = row_start + k * row_stride
        ref = pyoracle.render(W, H, nframes=frames, num_bounces=B, row_start=y, row_stride=1, nrows=1, env=env)
        assert bits_equal(img[k:k + 1], ref), (k, y, mismatch_report(img[k:k + 1], ref))


def test_c2_chained_regime_matches_oracle(fresh):
    """configs[1] as bench.py now times it: 1920x1080, 8 spp per launch, 8 bounces, 70 chained
    launches with the default switches (the first scheduled launches time the launch variant and
    restart the chain; counted launches at 5 and 40 end it; the schedule rebuild at 64 restarts it),
    a synchronisation after launch 25 (the timed arms' pick is then taken, as after bench.py's device
    warm-up): 40 rows spread over the image equal the oracle after 560 frames, and most launches
    overlapped."""
    W, H, B, S = 1920, 1080, 8, 8
    fresh(B)   # (conftest: a schedule rebuild every 64 launches, so one inside the 70)
    img, frames, counts = _series(W, H, B, S, 70, count_at=(5, 40), sync_at=(25,))
    assert counts["continued"] >= 30, counts
    _check_rows(img, W, H, frames, B, range(13, H, 27))


def test_c2_chained_whole_image_matches_oracle(fresh):
    """configs[1] chained at 6 waves per SIMD (the timing's pick for it), 24 launches -- all but the
    first two continue the overlap, claiming their dynamic units cheapest-first (pt_capi.cpp
    kChainBack): the whole image after 192 frames equals the oracle bit for bit (a stale accumulator
    read would show as scattered pixels)."""
    W, H, B, S = 1920, 1080, 8, 8
    fresh(B, PT_MI355_CT_WAVES="6")
    img, frames, counts = _series(W, H, B, S, 24)
    assert counts["continued"] >= 21, counts
    ref = pyoracle.render(W, H, nframes=frames, num_bounces=B)
    assert bits_equal(img, ref), mismatch_report(img, ref)


@pytest.mark.parametrize("case", [
    # W, H, spp, launches, rows (None: the whole image), waves
    (1000, 600, 8, 14, None, "6"),        # odd size: partial tiles, split tiles (one-chunk launches)
    (640, 360, 1, 24, None, "5"),         # 1 spp launches at 5 waves per SIMD
    (1920, 1080, 16, 8, range(5, 1080, 97), "6"),   # two-chunk launches (no split, no back claims)
])
def test_chained_geometries_match_oracle(fresh, case):
    """Chained series at a fixed launch variant (PT_MI355_CT_WAVES), so every launch after the
    schedule's build continues the chain: images equal the oracle."""
    W, H, S, n, rows, waves = case
    B = 8
    fresh(B, PT_MI355_CT_WAVES=waves)
    img, frames, counts = _series(W, H, B, S, n)
    assert counts["continued"] >= n - 3, counts
    if rows is None:
        ref = pyoracle.render(W, H, nframes=frames, num_bounces=B)
        assert bits_equal(img, ref), mismatch_report(img, ref)
    else:
        _check_rows(img, W, H, frames, B, rows)


def test_chained_rank_shard_matches_oracle(fresh):
    """The 2-rank weak-scaling shard (2712 x 1526, rows 1::2: bench.py --gpus 2's rank 1), 12 chained
    launches at the timed default after a synchronisation: sampled rows equal the oracle."""
    W, H, B, S = 2712, 1526, 8, 8
    fresh(B, PT_MI355_CT_WAVES="6", PT_MI355_BACK="45")
    img, frames, counts = _series(W, H, B, S, 12, row_start=1, row_stride=2, nrows=763)
    assert counts["continued"] >= 9, counts
    _check_rows(img, W, H, frames, B, [0, 190, 381, 500, 762], row_start=1, row_stride=2)


def test_chained_launches_that_wait_match_oracle(fresh):
    """Forced waits: every chained launch's waves sleep ~300 us before publishing a tile
    (PT_MI355_TEST_CHAIN_DELAY), so the next launch reaches tiles whose previous frames are not yet
    stored and waits on their epochs.  The whole image equals the oracle."""
    W, H, B, S = 640, 360, 8, 8
    fresh(B, PT_MI355_CT_WAVES="6", PT_MI355_TEST_CHAIN_DELAY="300")
    img, frames, counts = _series(W, H, B, S, 10)
    assert counts["continued"] >= 7, counts
    ref = pyoracle.render(W, H, nframes=frames, num_bounces=B)
    assert bits_equal(img, ref), mismatch_report(img, ref)


def test_chain_wait_error_stops_chaining(fresh):
    """A chained launch whose wait for its predecessor's tile runs out -- forced here: a 16-poll bound
    (PT_MI355_TEST_CHAIN_POLLS) against ~2 ms publication delays -- is reported as guard 13
    (PT_EKERNEL), never a hang, and the device stops chaining ("Residency"): the next
    series of chained calls runs as plain launches (none continues) and equals the oracle."""
    from cpuperformanceraytracer_amd._native import PtError
    W, H, B, S = 320, 180, 8, 8
    fresh(B, PT_MI355_CT_WAVES="6", PT_MI355_TEST_CHAIN_DELAY="2000", PT_MI355_TEST_CHAIN_POLLS="16")
    with pytest.raises(PtError, match="guard 13"):
        _series(W, H, B, S, 6)
    img, frames, counts = _series(W, H, B, S, 6)
    assert counts["continued"] == 0 and counts["restarts"] == 0, counts
    ref = pyoracle.render(W, H, nframes=frames, num_bounces=B)
    assert bits_equal(img, ref), mismatch_report(img, ref)


def test_chain_mixed_with_plain_and_counted_launches(fresh):
    """Chained launches with a plain pt_render_device launch (4, 9) and counted launches on another
    buffer (6) between them: each ends the overlap, the next chained launch restarts it; the whole
    image equals the oracle."""
    W, H, B, S = 800, 480, 8, 8
    fresh(B, PT_MI355_CT_WAVES="6")
    img, frames, counts = _series(W, H, B, S, 16, plain_at=(4, 9), count_at=(6,))
    assert counts["continued"] >= 6 and counts["restarts"] >= 4, counts
    ref = pyoracle.render(W, H, nframes=frames, num_bounces=B)
    assert bits_equal(img, ref), mismatch_report(img, ref)


def test_c4_env_chained_matches_oracle(fresh):
    """configs[3] chained: 1920x1080, 16 spp per launch, the synthetic 2k env map, the env kernel at a
    fixed back-claim share (PT_MI355_BACK: no timed arms), 7 launches: the whole image after 112
    frames equals the oracle."""
    from cpuperformanceraytracer_amd.config import synthetic_env
    from cpuperformanceraytracer_amd.device import set_env_map
    W, H, B, S = 1920, 1080, 8, 16
    fresh(B, PT_MI355_BACK="20")
    env = synthetic_env()
    set_env_map(env, 0, B)
    img, frames, counts = _series(W, H, B, S, 7, env=True)
    assert counts["continued"] >= 4, counts
    ref = pyoracle.render(W, H, nframes=frames, num_bounces=B, env=env)
    assert bits_equal(img, ref), mismatch_report(img, ref)


def test_v4_chained_matches_oracle(fresh):
    """The v4 workload chained (pt_v4_render_device_chain): 1920x1080, 8 spp, 8 bounces, the default
    glass scene and the synthetic 2k equirect map, 12 launches with a counted launch at 4 (the
    continuous-tiles v4 kernel, its sky frames published at the claim): rows 5::90 after 96 frames
    equal the v4 oracle."""
    import cpuperformanceraytracer_amd as pt
    from cpuperformanceraytracer_amd.config import synthetic_env
    W, H, B, S = 1920, 1080, 8, 8
    fresh(B)
    env = synthetic_env()
    pt.v4_config(num_bounces=B)
    pt.set_env_map(env)
    img, frames, counts = _series(W, H, B, S, 12, env=True, v4=True, count_at=(4,))
    assert counts["continued"] >= 6, counts
    for k in range(5, H, 90):
        ref = pyoracle.render4(W, H, nframes=frames, num_bounces=B, row_start=k, row_stride=1, nrows=1, env=env)
        assert bits_equal(img[k:k + 1], ref), (k, mismatch_report(img[k:k + 1], ref))


def test_v4_chained_waits_match_oracle(fresh):
    """v4 chained with forced waits (PT_MI355_TEST_CHAIN_DELAY) and the continuous-tiles kernel forced
    (PT_MI355_V4_CT) at 640x360: the whole image equals the v4 oracle."""
    import cpuperformanceraytracer_amd as pt
    from cpuperformanceraytracer_amd.config import synthetic_env
    W, H, B, S = 640, 360, 8, 8
    fresh(B, PT_MI355_TEST_CHAIN_DELAY="300", PT_MI355_V4_CT="1")
    env = synthetic_env()
    pt.v4_config(num_bounces=B)
    pt.set_env_map(env)
    img, frames, counts = _series(W, H, B, S, 8, env=True, v4=True)
    assert counts["continued"] >= 5, counts
    ref = pyoracle.render4(W, H, nframes=frames, num_bounces=B, env=env)
    assert bits_equal(img, ref), mismatch_report(img, ref)
