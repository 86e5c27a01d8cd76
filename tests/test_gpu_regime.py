"""The bench's timed regime against the oracle.

bench.py times PREPARED-JOB launches (device.JobLauncher, bench.py render_fn): the 3rd and later
launches of one geometry, i.e. launches that run the rebuilt tile schedule, split tiles (one-chunk
launches), back claims on the last fifth of the grid and units of twice the adaptive cost
(pt_capi.cpp use_sched / launch).  Here the same launcher drives more than kSchedRebuild + 2 launches
of each workload with the default switches, with bench.py's work-count launches on a scratch buffer
of the same geometry interleaved, and the accumulated image (c2, c4: whole; c3, v4, shards: sampled
rows) is compared BIT FOR BIT with the oracle (oracle/pt_oracle.c, pinned to demofox_path_tracing_scalar.cpp:785-820 -- the frame
loop and the progressive lerp of :812).  So the oracle, not a library self-comparison, guards every
path the timed launches take.

Also here: changes of the continuous-tiles grid between the launches of one accumulation
(PT_MI355_CT_WAVES_SEQ, a forced 5/6-waves-per-SIMD sequence, and PT_MI355_CT_WAVES=0, the
per-geometry timing that alternates the two on a geometry's first scheduled launches) at the
2-rank weak-scaling shard geometry (2712 x 1526, rows 1::2) where the round-4 rehearsal reported a
mismatching row (its cause was the bench's per-rank warm-up count; the kernels are
grid-independent, which these tests pin).
"""
from __future__ import annotations

import numpy as np
import pytest

from conftest import bits_equal, mismatch_report
from oracle import pyoracle

pytestmark = pytest.mark.gpu

K_SCHED_REBUILD = 64   # PT_MI355_SCHED_REBUILD as tests/conftest.py sets it (pt_capi.cpp)


def _launch_series(W, H, B, S, launches, *, row_start=0, row_stride=1, nrows=None, env=False, count_at=(),
                   v4=False, sync_at=()):
    """`launches` JobLauncher launches of S frames (frames 1 .. launches*S) into a zeroed buffer, on
    the current stream, as bench.py's render_fn; at the launch indices in count_at also a counted
    launch on a scratch buffer of the same geometry (bench.py's count pass); after the launch indices
    in sync_at a device synchronisation (the timed arms' events are then complete, so the next
    launch takes the pick).  Returns the image."""
    import torch
    from cpuperformanceraytracer_amd.device import JobLauncher, check_device_errors, count_device, count_v4_device
    nrows = H if nrows is None else nrows
    stream = torch.cuda.current_stream()
    buf = torch.zeros(nrows * W * 3, dtype=torch.float32, device="cuda:0")
    scratch = torch.zeros_like(buf)
    launch = JobLauncher(buf, W, H, nframes=S, num_bounces=B, row_start=row_start, row_stride=row_stride,
                         nrows=nrows, use_env=env, stream=stream, v4=v4)
    cfn = count_v4_device if v4 else count_device
    frame = 1
    for k in range(launches):
        launch(frame)
        if k in count_at:
            cfn(scratch, W, H, frame_first=frame, nframes=S, num_bounces=B, row_start=row_start,
                row_stride=row_stride, nrows=nrows, use_env=env, stream=stream)
        if k in sync_at:
            torch.cuda.synchronize()
        frame += S
    torch.cuda.synchronize()
    check_device_errors()
    return buf.cpu().numpy().reshape(nrows, W, 3), frame - 1


def _check_rows(img, W, H, frames, B, local_rows, *, row_start=0, row_stride=1, env=None):
    for k in local_rows:
        y = row_start + k * row_stride
        ref = pyoracle.render(W, H, nframes=frames, num_bounces=B, row_start=y, row_stride=1, nrows=1, env=env)
        assert bits_equal(img[k:k + 1], ref), (k, y, mismatch_report(img[k:k + 1], ref))


@pytest.fixture
def fresh(monkeypatch):
    """A fresh library state (schedules, occupancy picks) initialised under the test's environment."""
    import cpuperformanceraytracer_amd as pt

    def init(B, **envs):
        for k, v in envs.items():
            monkeypatch.setenv(k, v)
        pt.init(num_bounces=B)
    yield init
    pt.shutdown()
    monkeypatch.delenv("PT_MI355_CT_WAVES", raising=False)
    monkeypatch.delenv("PT_MI355_CT_WAVES_SEQ", raising=False)


def test_c2_bench_regime_matches_oracle(fresh):
    """configs[1] as bench.py times it: 1920x1080, 8 spp per launch, 8 bounces, 70 prepared-job
    launches (unscheduled, scheduled -- the first 18 timing the launch variant's arms --, rebuilt at
    launch 65) with counted launches interleaved; the whole image after 560 frames equals the oracle
    bit for bit."""
    W, H, B, S = 1920, 1080, 8, 8
    fresh(B)
    img, frames = _launch_series(W, H, B, S, K_SCHED_REBUILD + 6, count_at=(5, 40))
    assert np.isfinite(img).all()
    ref = pyoracle.render(W, H, nframes=frames, num_bounces=B)   # (the whole image)
    assert bits_equal(img, ref), mismatch_report(img, ref)


def test_c2_occupancy_timing_matches_oracle(fresh):
    """PT_MI355_CT_WAVES=0 (the default): the geometry's first 18 scheduled uncounted launches time the
    three arms (5 waves / 6 waves per SIMD at the default 20 % back claims / 6 waves at 45 %) in the
    palindromic order ABCCBA, three rounds, between event pairs (pt_capi.cpp ct_occupancy); a counted
    launch in between is not timed; after a synchronisation the next launch takes the pick, and the
    launches after it run the picked arm -- the grid and the back-claim share change between the
    launches of one accumulation.  30 launches of configs[1]: rows equal the oracle, and the pick is
    one of the arms (pt_launch_variant)."""
    import torch
    from cpuperformanceraytracer_amd.device import launch_variant
    W, H, B, S = 1920, 1080, 8, 8
    fresh(B, PT_MI355_CT_WAVES="0")
    img, frames = _launch_series(W, H, B, S, 30, count_at=(7,), sync_at=(21,))
    _check_rows(img, W, H, frames, B, range(27, H, 108))
    buf = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda:0")
    v = launch_variant(buf, W, H, nframes=S, num_bounces=B)
    assert (v["waves_per_simd"], v["back_claim_pct"]) in ((5, 20), (6, 20), (6, 45)), v


@pytest.mark.parametrize("seq", ["5665", "56"])
def test_forced_grid_alternation_rank_shard(fresh, seq):
    """The 2-rank weak-scaling shard of the round-4 rehearsal -- image 2712 x 1526, rank 1's rows
    1::2 (763 rows; global row 763 is its local row 381) -- over 24 scheduled 8-frame launches whose
    continuous-tiles grid follows a forced 5/6-waves sequence (PT_MI355_CT_WAVES_SEQ), so every
    piece of cross-launch state (the tile-queue ring slot the previous launch zeroed, the static /
    dynamic unit split of group_waves(gridDim), the back-claim band, the per-wave slot area) is
    exercised under grid changes; sampled rows, among them global row 763, equal the oracle."""
    W, H, B, S = 2712, 1526, 8, 8
    fresh(B, PT_MI355_CT_WAVES_SEQ=seq)
    img, frames = _launch_series(W, H, B, S, 24, row_start=1, row_stride=2, nrows=763)
    _check_rows(img, W, H, frames, B, [0, 190, 381, 500, 762], row_start=1, row_stride=2)


def test_c4_env_bench_regime_matches_oracle(fresh):
    """configs[3] as bench.py times it: 1920x1080, 16 spp per launch, the synthetic 2k env map,
    6 prepared-job launches (the continuous-tiles env kernel with its timed back-claim shares); the
    whole image after 96 frames equals the oracle."""
    from cpuperformanceraytracer_amd.config import synthetic_env
    from cpuperformanceraytracer_amd.device import set_env_map
    W, H, B, S = 1920, 1080, 8, 16
    fresh(B)
    env = synthetic_env()
    set_env_map(env, 0, B)
    img, frames = _launch_series(W, H, B, S, 6, env=True, count_at=(3,))
    ref = pyoracle.render(W, H, nframes=frames, num_bounces=B, env=env)   # (the whole image)
    assert bits_equal(img, ref), mismatch_report(img, ref)


def test_c3_bench_regime_matches_oracle(fresh):
    """configs[2] as bench.py times it: 3840x2160, 64 spp per launch (multi-chunk: no split tiles,
    no back claims), 3 prepared-job launches (unscheduled, scheduled, scheduled); rows 31::108 after
    192 frames equal the oracle."""
    W, H, B, S = 3840, 2160, 8, 64
    fresh(B)
    img, frames = _launch_series(W, H, B, S, 3, count_at=(1,))
    _check_rows(img, W, H, frames, B, range(31, H, 108))


def test_v4_bench_regime_matches_oracle(fresh):
    """The v4 workload as bench.py times it: 1920x1080, 8 spp, 8 bounces, the default glass scene and
    the synthetic 2k equirect map, 10 prepared-job launches (scheduled from the 2nd on); rows 5::90
    after 80 frames equal the v4 oracle."""
    import cpuperformanceraytracer_amd as pt
    from cpuperformanceraytracer_amd.config import synthetic_env
    W, H, B, S = 1920, 1080, 8, 8
    fresh(B)
    env = synthetic_env()
    pt.v4_config(num_bounces=B)
    pt.set_env_map(env)
    img, frames = _launch_series(W, H, B, S, 10, env=True, v4=True, count_at=(4,))
    for k in range(5, H, 90):
        ref = pyoracle.render4(W, H, nframes=frames, num_bounces=B, row_start=k, row_stride=1, nrows=1, env=env)
        assert bits_equal(img[k:k + 1], ref), (k, mismatch_report(img[k:k + 1], ref))


def test_launch_variant_reports_the_pick(fresh):
    """pt_launch_variant: undecided before the geometry's timed launches, then the pick they made (5 or
    6 waves per SIMD; 20 or 45 % back claims for these one-chunk launches); with PT_MI355_CT_WAVES
    fixed, that occupancy and the default share at once.  bench.py reports it as launch_variant."""
    import torch
    from cpuperformanceraytracer_amd.device import launch_variant
    W, H, B, S = 1920, 1080, 8, 8
    buf = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda:0")
    fresh(B)
    assert launch_variant(buf, W, H, nframes=S, num_bounces=B)["waves_per_simd"] == 0
    _launch_series(W, H, B, S, 24)   # (ends synchronised: the timed launches' events are complete)
    # the pick is taken by the first launch that finds the timing events complete
    from cpuperformanceraytracer_amd.device import JobLauncher
    JobLauncher(buf, W, H, nframes=S, num_bounces=B, stream=torch.cuda.current_stream())(1)
    torch.cuda.synchronize()
    v = launch_variant(buf, W, H, nframes=S, num_bounces=B)
    assert (v["waves_per_simd"], v["back_claim_pct"]) in ((5, 20), (6, 20), (6, 45)), v
    fresh(B, PT_MI355_CT_WAVES="6")
    assert launch_variant(buf, W, H, nframes=S, num_bounces=B) == {"waves_per_simd": 6, "back_claim_pct": 20}
