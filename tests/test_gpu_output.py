"""GPU parity of the output stage: ACES + fast sRGB + 8-bit pack of the
accumulator (v4 :144-187, :1260-1331) against the CPU restatement (oracle/pt_oracle_output.c).

Bar: BIT-EXACT packed pixels.  Both sides use the correctly rounded 1/x for the reference's
_mm256_rcp_ps (CPU-model specific table, see the oracle header), fused fmadd/fmsub, IEEE sqrt,
MAXPS/MINPS NaN rules and round-to-nearest-even conversion.
"""
from __future__ import annotations

import numpy as np
import pytest

from conftest import bits_equal, mismatch_report
from layouts import interleaved_to_planar8, interleaved_to_tiled
from oracle import pyoracle

pytestmark = pytest.mark.gpu

import cpuperformanceraytracer_amd as pt  # noqa: E402
from cpuperformanceraytracer_amd import _native as N  # noqa: E402


def _accumulator(h, w, seed):
    rng = np.random.default_rng(seed)
    a = rng.lognormal(-1.0, 1.5, (h, w, 3)).astype(np.float32)
    flat = a.reshape(-1)
    special = np.array([0.0, -0.0, 1e-45, 1e-38, 0.0031308, 0.00313, 0.0032, 1.0, 16.0, 1e30, np.inf, -1.0,
                        np.nan, 3.4e38], np.float32)
    flat[: special.size] = special
    return a


@pytest.mark.parametrize("fmt", [N.PT_PIXEL_RGBA8, N.PT_PIXEL_XRGB8])
def test_tonemap_interleaved_vs_oracle(fmt):
    pt.init()
    a = _accumulator(135, 240, 1)
    got = pt.tonemap(a, 240, 135, fmt=fmt)
    ref = pyoracle.tonemap(a, fmt)
    assert np.array_equal(got, ref), f"{int((got != ref).sum())} pixels differ"


def test_tonemap_layouts_and_render():
    """A rendered image, in the three layouts of the frame calls."""
    pt.init(num_bounces=8, samples_per_frame=4)
    w, h = 320, 192
    img = np.zeros((h, w, 3), np.float32)
    pt.DemofoxRenderScalar(img, w, h, 3)
    ref = pyoracle.tonemap(img, pyoracle.PIXEL_RGBA8)
    assert np.array_equal(pt.tonemap(img, w, h), ref)
    assert np.array_equal(pt.tonemap(interleaved_to_planar8(img), w, h, layout=N.PT_LAYOUT_PLANAR8), ref)
    tiled = interleaved_to_tiled(img, 64, 48)
    assert np.array_equal(pt.tonemap(tiled, w, h, layout=N.PT_LAYOUT_TILED_PLANAR8, tile_width=64, tile_height=48), ref)
    screen = np.zeros((h, w), np.uint32)
    pt.CopyOutputToFile(tiled, w, h, 5, 4, 64, 48, 3, None, screen)
    assert np.array_equal(screen, ref)


def test_tonemap_of_deferred_accumulator():
    """PT_FLAG_DEFER_READBACK: the HBM accumulator is tonemapped without a readback."""
    pt.init(num_bounces=8, defer_readback=True)
    w, h = 256, 128
    buf = np.zeros((h, w, 3), np.float32)
    for _ in range(3):
        pt.DemofoxRenderScalar(buf, w, h, 3)
    got = pt.tonemap(buf, w, h)                         # buf itself is still zeros on the host
    ref = pyoracle.tonemap(pyoracle.render(w, h, nframes=3, num_bounces=8), pyoracle.PIXEL_RGBA8)
    assert np.array_equal(got, ref)


def test_tonemap_device_full_hd():
    import ctypes
    import torch
    pt.init()
    w, h = 1920, 1080
    a = _accumulator(h, w, 7)
    d_in = torch.from_numpy(a).to("cuda:0")
    d_out = torch.zeros(h * w, dtype=torch.int32, device="cuda:0")
    s = torch.cuda.current_stream()
    N.check(N.load().pt_tonemap_device(d_in.data_ptr(), w, h, N.PT_LAYOUT_INTERLEAVED, 0, 0, d_out.data_ptr(),
                                       N.PT_PIXEL_XRGB8, ctypes.c_void_p(s.cuda_stream)), "pt_tonemap_device")
    torch.cuda.synchronize()
    got = d_out.cpu().numpy().view(np.uint32).reshape(h, w)
    assert np.array_equal(got, pyoracle.tonemap(a, pyoracle.PIXEL_XRGB8))


def test_tonemap_errors():
    pt.init()
    a = np.zeros((8, 12, 3), np.float32)
    with pytest.raises(N.PtError):
        pt.tonemap(a, 12, 8, layout=N.PT_LAYOUT_PLANAR8)        # width not a multiple of 8
    with pytest.raises(N.PtError):
        pt.tonemap(a, 12, 8, fmt=7)
    with pytest.raises(N.PtError):
        pt.tonemap(np.zeros((8, 16, 3), np.float32), 16, 8, layout=N.PT_LAYOUT_TILED_PLANAR8, tile_width=12,
                   tile_height=8)


# ---- the output stage fused into the render (pt_render_device_present) ----
def _present_series(W, H, B, S, launches, fmt, *, use_env=False, pool_env=None, **rows):
    """`launches` fused launches of S frames (frames 1 .. launches*S); returns (accumulator, pixels)."""
    import torch
    from cpuperformanceraytracer_amd.device import JobLauncher
    nrows = rows.get("nrows", H)
    buf = torch.zeros(nrows * W * 3, dtype=torch.float32, device="cuda:0")
    pix = torch.zeros(nrows * W, dtype=torch.int32, device="cuda:0")
    launch = JobLauncher(buf, W, H, nframes=S, num_bounces=B, use_env=use_env, pixels=pix, pixel_format=fmt,
                         **rows)
    for k in range(launches):
        launch(1 + k * S)
    torch.cuda.synchronize()
    return buf.cpu().numpy().reshape(nrows, W, 3), pix.cpu().numpy().view(np.uint32).reshape(nrows, W)


@pytest.mark.parametrize("fmt", [N.PT_PIXEL_RGBA8, N.PT_PIXEL_XRGB8])
def test_fused_present_c2_matches_oracle(fmt):
    """configs[1] (1920x1080, 8 spp, 8 bounces) with the output stage fused into the continuous-tiles
    kernel: after 3 fused launches (the 2nd and 3rd scheduled, with split tiles) every pixel equals the
    standalone pass over the same accumulator, and the whole image equals the oracle (render, then
    OutputToFile / OutputToScreen of v4 :1260-1331) bit for bit."""
    import torch
    pt.init(num_bounces=8)
    W, H, B, S = 1920, 1080, 8, 8
    acc, pix = _present_series(W, H, B, S, 3, fmt)
    from cpuperformanceraytracer_amd.device import tonemap_device
    sep = torch.zeros(W * H, dtype=torch.int32, device="cuda:0")
    dbuf = torch.from_numpy(acc.reshape(-1).copy()).to("cuda:0")
    tonemap_device(dbuf, W, H, sep, pixel_format=fmt)
    torch.cuda.synchronize()
    assert np.array_equal(pix, sep.cpu().numpy().view(np.uint32).reshape(H, W))
    # the whole image (a presenting build once differed from the plain kernel in 341 of 2 M pixels
    # -- one frame of one path each -- which sampled rows can miss: profiles/r05/r05s_*)
    ref = pyoracle.render(W, H, nframes=3 * S, num_bounces=B)
    assert bits_equal(acc, ref), mismatch_report(acc, ref)
    assert np.array_equal(pix, pyoracle.tonemap(ref, fmt))


def test_fused_present_env_shard_and_fallback_pools(monkeypatch):
    """The env kernel (configs[3] miss term) and a row shard present in the fused kernel; with
    PT_MI355_NO_CT=1 (the per-tile / ring pools, which do not present) the standalone pass runs after
    the launch -- the same pixels either way, equal to the oracle's."""
    import torch
    from cpuperformanceraytracer_amd.device import set_env_map
    W, H, B = 256, 144, 8
    rng = np.random.default_rng(21)
    env = (rng.random((32, 64, 3), dtype=np.float32) * 3.0 + 0.01).astype(np.float32)
    rows = dict(row_start=1, row_stride=3, nrows=48)
    ref = pyoracle.render(W, H, nframes=2 * 16, num_bounces=B, env=env, **rows)
    for no_ct in ("0", "1"):
        monkeypatch.setenv("PT_MI355_NO_CT", no_ct)
        pt.init(num_bounces=B)
        set_env_map(env, 0, B)
        acc, pix = _present_series(W, H, B, 16, 2, N.PT_PIXEL_RGBA8, use_env=True, **rows)
        assert np.array_equal(acc.view(np.uint32), ref.view(np.uint32)), no_ct
        assert np.array_equal(pix, pyoracle.tonemap(ref, N.PT_PIXEL_RGBA8)), no_ct
        pt.shutdown()
    # 0 frames: nothing rendered, the accumulator is still converted
    monkeypatch.setenv("PT_MI355_NO_CT", "0")
    pt.init(num_bounces=B)
    from cpuperformanceraytracer_amd.device import render_device_present
    buf = torch.from_numpy(ref.reshape(-1).copy()).to("cuda:0")
    pix = torch.zeros(W * 48, dtype=torch.int32, device="cuda:0")
    render_device_present(buf, pix, W, H, frame_first=1, nframes=0, num_bounces=B, **rows)
    torch.cuda.synchronize()
    assert np.array_equal(pix.cpu().numpy().view(np.uint32).reshape(48, W), pyoracle.tonemap(ref, N.PT_PIXEL_RGBA8))
    pt.shutdown()


@pytest.mark.parametrize("waves", ["5", "6", "0"])
def test_fused_present_accumulator_equals_plain_every_occupancy(monkeypatch, waves):
    """The presenting continuous-tiles instances are separate template instances with their own
    register allocation: at each occupancy (5 / 6 waves per SIMD, and the timed variants) the whole
    accumulator of 4 presenting launches equals the plain kernel's bit for bit (1920x1080, 8 spp)."""
    import torch
    from cpuperformanceraytracer_amd.device import JobLauncher
    monkeypatch.setenv("PT_MI355_CT_WAVES", waves)
    W, H, B, S = 1920, 1080, 8, 8
    out = []
    try:
        for present in (False, True):
            pt.init(num_bounces=B)
            buf = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda:0")
            kw = dict(pixels=torch.zeros(H * W, dtype=torch.int32, device="cuda:0"), pixel_format=0) if present else {}
            launch = JobLauncher(buf, W, H, nframes=S, num_bounces=B, **kw)
            for k in range(4):
                launch(1 + k * S)
            torch.cuda.synchronize()
            out.append(buf.cpu().numpy().reshape(H, W, 3))
    finally:
        monkeypatch.delenv("PT_MI355_CT_WAVES")
        pt.init()
    assert bits_equal(out[1], out[0]), mismatch_report(out[1], out[0])


def test_fused_present_env_full_size_equals_plain():
    """configs[3] at full size (1920x1080, 16 spp, the synthetic 2k env map): the presenting env
    kernel's whole accumulator after 3 launches equals the plain env kernel's bit for bit, and its
    pixels equal the standalone conversion of that accumulator."""
    import torch
    from cpuperformanceraytracer_amd.config import synthetic_env
    from cpuperformanceraytracer_amd.device import JobLauncher, set_env_map, tonemap_device
    W, H, B, S = 1920, 1080, 8, 16
    out, pix = [], None
    for present in (False, True):
        pt.init(num_bounces=B)
        set_env_map(synthetic_env(), 0, B)
        buf = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda:0")
        p = torch.zeros(H * W, dtype=torch.int32, device="cuda:0")
        kw = dict(pixels=p, pixel_format=N.PT_PIXEL_XRGB8) if present else {}
        launch = JobLauncher(buf, W, H, nframes=S, num_bounces=B, use_env=True, **kw)
        for k in range(3):
            launch(1 + k * S)
        torch.cuda.synchronize()
        out.append(buf.cpu().numpy().reshape(H, W, 3))
        if present:
            sep = torch.zeros(H * W, dtype=torch.int32, device="cuda:0")
            tonemap_device(buf, W, H, sep, pixel_format=N.PT_PIXEL_XRGB8)
            torch.cuda.synchronize()
            assert np.array_equal(p.cpu().numpy(), sep.cpu().numpy())
    pt.init()
    assert bits_equal(out[1], out[0]), mismatch_report(out[1], out[0])
