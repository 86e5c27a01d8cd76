"""Several devices behind the C ABI (pt_config.device_count / PT_MI355_DEVICES): every host-buffer
entry point deals the frame's rows to the devices (row Y -> device Y mod N; each device mirrors its
own rows) -- the reference's fan-out of a frame's tiles over NUM_THREADS CPU threads
(simd_tiled.cpp:549-571, v4 :1696-1721), here over GPUs.  The test box has one GPU, so N logical
devices are mapped onto it (same ordinal; own streams, mirrors, queues, schedules): the sharding,
the pitched row transfers, the per-device output stage and the per-device mirrors are exercised
exactly as with N physical GPUs.

Bar: BIT-EXACT against the oracles (oracle/pt_oracle.c, oracle/pt_oracle_v4.c) for every layout,
the v4 path, RenderTile, work queues, deferred readback and the reference-shaped C++ host run
unchanged (examples/reference_host with PT_MI355_DEVICES).
"""
from __future__ import annotations

import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

from conftest import bits_equal, mismatch_report
from layouts import interleaved_to_planar8, interleaved_to_tiled, planar8_to_interleaved, tiled_to_interleaved
from oracle import pyoracle as po

pytestmark = pytest.mark.gpu

import cpuperformanceraytracer_amd as pt  # noqa: E402
from cpuperformanceraytracer_amd import _native as N  # noqa: E402

ROOT = Path(__file__).resolve().parents[1]


def _tex(h: int, w: int, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    return (rng.random((h, w, 3), dtype=np.float32) * 3.0 + 0.01).astype(np.float32)


@pytest.fixture(autouse=True)
def _reset():
    yield
    pt.shutdown()


@pytest.mark.parametrize("n", [2, 3, 5])
def test_scalar_and_simd_frames(n):
    w, h, b = 200, 122, 8     # 122 rows: uneven shards for 3 and 5 devices
    pt.init(num_bounces=b, devices=[0] * n)
    assert pt.initialized_devices() == [0] * n
    a = np.zeros((h, w, 3), np.float32)
    p8 = np.zeros(w * h * 3, np.float32)
    for _ in range(2):
        pt.DemofoxRenderScalar(a, w, h, 3)
    pt.set_frame(0)
    for _ in range(2):
        pt.DemofoxRenderSimd(p8, w, h, 3)
    ref = po.render(w, h, nframes=2, num_bounces=b)
    assert bits_equal(a, ref), mismatch_report(a, ref)
    got = planar8_to_interleaved(p8, w, h)
    assert bits_equal(got, ref), mismatch_report(got, ref)


@pytest.mark.parametrize("n,tiles", [(2, (10, 15)), (3, (10, 15)), (4, (4, 5)), (8, (5, 3))])
def test_simd_tiled_frames(n, tiles):
    ntx, nty = tiles
    w, h, b = 320, 240, 8
    tw, th = w // ntx, h // nty
    pt.init(num_bounces=b, samples_per_frame=2, devices=[0] * n)
    start = np.random.default_rng(5).random((h, w, 3), dtype=np.float32)
    buf = interleaved_to_tiled(start, tw, th)
    pt.DemofoxRenderSimdTiled(buf, w, h, ntx, nty, tw, th, 3)
    pt.DemofoxRenderSimdTiled(buf, w, h, ntx, nty, tw, th, 3)
    ref = po.render(w, h, nframes=4, num_bounces=b, buf=start.copy())
    got = tiled_to_interleaved(buf, w, h, tw, th)
    assert bits_equal(got, ref), mismatch_report(got, ref)


def test_simt_textured_frames():
    w, h, ntx, nty, b = 256, 120, 8, 6, 8
    tw, th = w // ntx, h // nty
    env = _tex(48, 96, seed=3)
    pt.init(num_bounces=b, devices=[0, 0, 0])
    buf = np.zeros(w * h * 3, np.float32)
    tex = pt.texture(env, 96, 48, 3)
    for _ in range(2):
        pt.DemofoxRenderSimtTextured(buf, w, h, ntx, nty, tw, th, 3, tex)
    ref = po.render(w, h, nframes=2, num_bounces=b, env=env)
    got = tiled_to_interleaved(buf, w, h, tw, th)
    assert bits_equal(got, ref), mismatch_report(got, ref)


def test_render_tile_fan_out():
    """Host-fanned RenderTile calls (the simt_pooled / v4 pattern): every device renders its rows of
    each tile; only the tile's rows move."""
    w, h, ntx, nty, b = 160, 96, 5, 4, 4
    tw, th = w // ntx, h // nty
    pt.init(num_bounces=b, devices=[0, 0, 0])
    start = np.random.default_rng(9).random((h, w, 3), dtype=np.float32)
    buf = interleaved_to_tiled(start, tw, th)
    bi = pt.RenderBufferInfo(buf, w, h, 3)
    tiles = pt.make_tiles(w, h, ntx, nty)
    pt.BeginFrame()
    for t in tiles[::2]:   # half the tiles: the others must stay untouched
        pt.RenderTile(bi, t)
    ref = po.render(w, h, nframes=1, num_bounces=b, buf=start.copy())
    got = tiled_to_interleaved(buf, w, h, tw, th)
    mask = np.zeros((h, w), bool)
    for t in tiles[::2]:
        mask[t.TileMinY:t.TileMaxY + 1, t.TileMinX:t.TileMaxX + 1] = True
    assert bits_equal(got[mask], ref[mask]), mismatch_report(got[mask], ref[mask])
    assert bits_equal(got[~mask], start[~mask])


@pytest.mark.parametrize("renderer", [N.PT_RENDERER_SIMD_TILED, N.PT_RENDERER_V4])
@pytest.mark.parametrize("full", [True, False])
def test_work_queue(renderer, full):
    w, h, ntx, nty = 320, 240, 10, 15
    tw, th = w // ntx, h // nty
    pt.init(num_bounces=8, devices=[0, 0, 0, 0])
    v4 = renderer == N.PT_RENDERER_V4
    if v4:
        pt.v4_config(env_mode=N.PT_V4_ENV_NONE)
    buf = np.zeros(w * h * 3, np.float32)
    bi = pt.RenderBufferInfo(buf, w, h, 3)
    tiles = pt.make_tiles(w, h, ntx, nty)
    chosen = tiles if full else tiles[::3]
    q = pt.MakeWorkQueue(renderer)
    for k in range(2):
        pt.v4_begin_frame() if v4 else pt.BeginFrame()
        for t in chosen:
            pt.AddWorkQueueEntry(q, bi, t)
        q.complete(wait=(k == 0))
    q.wait()
    q.close()
    ref = po.render4(w, h, nframes=2, env=None) if v4 else po.render(w, h, nframes=2, num_bounces=8)
    got = tiled_to_interleaved(buf, w, h, tw, th)
    mask = np.zeros((h, w), bool)
    for t in chosen:
        mask[t.TileMinY:t.TileMaxY + 1, t.TileMinX:t.TileMaxX + 1] = True
    assert bits_equal(got[mask], ref[mask]), mismatch_report(got[mask], ref[mask])
    assert not got[~mask].any()


@pytest.mark.parametrize("env_mode", [N.PT_V4_ENV_EQUIRECT, N.PT_V4_ENV_CUBEMAP])
def test_opt_v4_frames_screen_and_file(env_mode):
    w, h, ntx, nty = 320, 240, 10, 15
    tw, th = w // ntx, h // nty
    pt.init(devices=[0, 0, 0])
    pt.v4_config(env_mode=env_mode)
    pt.InitializeGlobalRenderResources()
    env = _tex(6 * 32, 32, seed=4) if env_mode == N.PT_V4_ENV_CUBEMAP else _tex(64, 128, seed=21)
    tex = pt.texture(env, env.shape[1], env.shape[0], 3)
    buf = np.zeros(w * h * 3, np.float32)
    screen = np.zeros(w * h, np.uint32)
    for _ in range(3):
        pt.DemofoxRenderOptV4(buf, w, h, ntx, nty, tw, th, 3, tex, screen)
    ref = po.render4(w, h, nframes=3, env=env, env_mode=env_mode)
    got = tiled_to_interleaved(buf, w, h, tw, th)
    assert bits_equal(got, ref), mismatch_report(got, ref)
    assert np.array_equal(screen.reshape(h, w), po.tonemap(ref, po.PIXEL_XRGB8))
    file_px = np.zeros(w * h, np.uint32)
    pt.CopyOutputToFile(buf, w, h, ntx, nty, tw, th, 3, tex, file_px)
    assert np.array_equal(file_px.reshape(h, w), po.tonemap(ref, po.PIXEL_RGBA8))


def _device_lists():
    """Logical shards of GPU 0, and -- where the box has several GPUs -- every physical GPU (ADVICE r3:
    hipSetDevice switching, per-device uploads and cross-device copies run only with distinct
    ordinals)."""
    import torch
    lists = [[0, 0, 0]]
    if torch.cuda.device_count() > 1:
        lists.append(list(range(min(torch.cuda.device_count(), 8))))
    return lists


@pytest.mark.parametrize("devices", _device_lists(), ids=lambda d: "x".join(map(str, d)))
@pytest.mark.parametrize("gather", [False, True], ids=["per_device", "gather_root"])
@pytest.mark.parametrize("layout", ["scalar", "tiled", "v4"])
def test_deferred_readback_and_tonemap(layout, gather, devices):
    """PT_FLAG_DEFER_READBACK: each device keeps its rows in HBM across calls; readback merges them,
    the output stage converts each device's rows in place -- or, PT_FLAG_GATHER_ROOT, every device
    stores its rows into the root's HBM (xGMI between GPUs) and the root converts / copies once."""
    w, h, ntx, nty = 240, 150, 6, 5
    tw, th = w // ntx, h // nty
    pt.init(num_bounces=8, defer_readback=True, devices=devices, gather_root=gather)
    buf = np.zeros(w * h * 3, np.float32)
    if layout == "v4":
        pt.v4_config(env_mode=N.PT_V4_ENV_NONE)
    for _ in range(3):
        if layout == "scalar":
            pt.DemofoxRenderScalar(buf, w, h, 3)
        elif layout == "tiled":
            pt.DemofoxRenderSimdTiled(buf, w, h, ntx, nty, tw, th, 3)
        else:
            pt.DemofoxRenderOptV4(buf, w, h, ntx, nty, tw, th, 3, None, None)
    assert not buf.any()   # nothing copied back yet
    ref = po.render4(w, h, nframes=3, env=None) if layout == "v4" else po.render(w, h, nframes=3, num_bounces=8)
    lay, tws, ths = (N.PT_LAYOUT_INTERLEAVED, 0, 0) if layout == "scalar" else (N.PT_LAYOUT_TILED_PLANAR8, tw, th)
    px = pt.tonemap(buf, w, h, lay, tws, ths)      # from the device-resident accumulator
    assert np.array_equal(px, po.tonemap(ref, po.PIXEL_RGBA8))
    if gather:   # the assembled accumulator in the root's HBM
        import ctypes
        dptr = pt.gather_root(buf)
        host = np.zeros(w * h * 3, np.float32)
        hip = ctypes.CDLL("libamdhip64.so.7")
        assert hip.hipMemcpy(ctypes.c_void_p(host.ctypes.data), ctypes.c_void_p(dptr), ctypes.c_size_t(host.nbytes),
                             2) == 0   # hipMemcpyDeviceToHost
        g = host.reshape(h, w, 3) if layout == "scalar" else tiled_to_interleaved(host, w, h, tw, th)
        assert bits_equal(g, ref), mismatch_report(g, ref)
        assert not buf.any()
    pt.readback(buf)
    got = buf.reshape(h, w, 3) if layout == "scalar" else tiled_to_interleaved(buf, w, h, tw, th)
    assert bits_equal(got, ref), mismatch_report(got, ref)


def test_device_jobs_use_the_buffers_device():
    """Device jobs run on the logical device holding their buffer (several devices initialised)."""
    import torch
    from cpuperformanceraytracer_amd.device import render_device
    pt.init(num_bounces=4, devices=[0, 0])
    w, h = 96, 64
    buf = torch.zeros(h * w * 3, dtype=torch.float32, device="cuda:0")
    render_device(buf, w, h, frame_first=1, nframes=3, num_bounces=4)
    torch.cuda.synchronize()
    ref = po.render(w, h, nframes=3, num_bounces=4)
    got = buf.cpu().numpy().reshape(h, w, 3)
    assert bits_equal(got, ref), mismatch_report(got, ref)


def test_caller_device_restored():
    import torch
    pt.init(devices=[0, 0])
    torch.cuda.set_device(0)
    a = np.zeros((32, 64, 3), np.float32)
    pt.DemofoxRenderScalar(a, 64, 32, 3)
    assert torch.cuda.current_device() == 0


def test_invalid_device_lists():
    with pytest.raises(N.PtError):
        pt.init(devices=[0, 99])
    with pytest.raises(N.PtError):
        pt.init(devices=[0] * (N.PT_MAX_DEVICES + 1))


@pytest.mark.parametrize("renderer", ["v4", "tiled", "scalar"])
def test_reference_host_unchanged_on_three_devices(tmp_path, renderer):
    """examples/reference_host (reference names only, never calls pt_init) with PT_MI355_DEVICES:
    the same bytes as on one device."""
    exe = ROOT / "examples" / "reference_host"
    if not exe.exists():
        from cpuperformanceraytracer_amd.build import build_examples
        build_examples()
    w, h, frames = 320, 240, 2
    outs = []
    for devs in (None, "0,0,0"):
        env = dict(os.environ)
        env.pop("PT_MI355_DEVICES", None)
        if devs:
            env["PT_MI355_DEVICES"] = devs
        out = tmp_path / f"{renderer}_{devs or 'one'}.f32"
        args = [str(exe), renderer, str(w), str(h), str(frames), str(out)]
        if renderer != "scalar":
            args.append(str(tmp_path / f"{renderer}_{devs or 'one'}.bmp"))
        r = subprocess.run(args, capture_output=True, text=True, timeout=120, env=env)
        assert r.returncode == 0, r.stderr
        outs.append(out.read_bytes())
        if renderer != "scalar":
            outs.append((tmp_path / f"{renderer}_{devs or 'one'}.bmp").read_bytes())
    half = len(outs) // 2
    assert outs[:half] == outs[half:]
