"""Every kernel instance the library can launch, reached through the C ABI and checked bit for bit
against the oracle.

The kernels are templates over layout (interleaved / planar8 / tiled-planar8), env miss term, counted
launches, launch shape (continuous-tiles pool at 5 or 6 waves per SIMD, per-tile pool: one chunk,
MULTI chunks, the RING pool), the fused output stage, and for v4 the env mode, scene (the default
InitializeScene geometry or an Add*ToScene one) and sampling / exp flags.  Each case below picks one
instance with the switches that select it (pt_kernel.hip launch_t / launch_ct / launch_pools,
pt_v4.hip launch_t) on a small image, renders through the public entry point that reaches it, and
compares with oracle/pt_oracle.c or oracle/pt_oracle_v4.c.  DESIGN.md §3d lists the instances;
scripts/gpu_coverage.sh runs this suite under rocprofv3 --kernel-trace and
tests/test_kernel_coverage.py checks that the launched set covers every instance in the library.

Which entry points reach what: counted launches are device jobs (row layouts); the tiled layout is
the drop-in's host calls (DemofoxRenderSimdTiled / RenderTile: samples_per_frame frames per call;
DemofoxRenderSimtTextured for the env term; DemofoxRenderOptV4: one frame per call, so v4's tiled
layout has only per-tile, uncounted instances); the per-tile diffuse pools run with
PT_MI355_NO_CT=1 (the continuous-tiles slots unused) and the v4 continuous-tiles kernel for
launches of >= 8 frames with PT_MI355_V4_CT=1 (below its occupancy threshold otherwise)."""
from __future__ import annotations

import numpy as np
import pytest

from conftest import bits_equal, mismatch_report
from layouts import planar8_to_interleaved, tiled_to_interleaved
from oracle import pyoracle as po

pytestmark = pytest.mark.gpu

import cpuperformanceraytracer_amd as pt  # noqa: E402
from cpuperformanceraytracer_amd import _native as N  # noqa: E402

W, H = 64, 40            # 8 x 5 tiles
NTX, NTY = 2, 2          # tiled layout: 32 x 20 tiles
TW, TH = W // NTX, H // NTY
B = 8


def _tex(h, w, seed):
    rng = np.random.default_rng(seed)
    return (rng.random((h, w, 3), dtype=np.float32) * 3.0 + 0.01).astype(np.float32)


ENV2 = _tex(32, 64, 5)            # diffuse config-4 map / v4 equirect
CUBE = _tex(6 * 16, 16, 6)         # v4 cubemap: six 16 x 16 faces


@pytest.fixture
def lib(monkeypatch):
    """Library state initialised under the case's switches (read by pt_init), released after."""
    def init(env_vars=None, **kw):
        for k in ("PT_MI355_NO_CT", "PT_MI355_CT_WAVES", "PT_MI355_V4_CT"):
            monkeypatch.delenv(k, raising=False)
        for k, v in (env_vars or {}).items():
            monkeypatch.setenv(k, v)
        pt.init(num_bounces=B, **kw)
    yield init
    pt.shutdown()


def _check(got, ref):
    assert bits_equal(got, ref), mismatch_report(got, ref)


# ---- diffuse renderer (pt_kernel.hip) ---------------------------------------------------------------
# modes: "ct5" / "ct6" the continuous-tiles kernel at 5 / 6 waves per SIMD (the env kernel has one
# occupancy), "tile" the per-tile pool (one chunk), "multi" its chunked MULTI form, "ring" the ring pool
MODES = {"ct5": ({"PT_MI355_CT_WAVES": "5"}, 3), "ct6": ({"PT_MI355_CT_WAVES": "6"}, 3),
         "tile": ({"PT_MI355_NO_CT": "1"}, 3), "multi": ({"PT_MI355_NO_CT": "1"}, 12),
         "ring": ({"PT_MI355_NO_CT": "1"}, 50)}


def _device_diffuse(layout, frames, env, how):
    import torch
    from cpuperformanceraytracer_amd.device import count_device, render_device, render_device_present, set_env_map
    if env:
        set_env_map(ENV2, 0, B)
    buf = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda:0")
    kw = dict(frame_first=1, nframes=frames, num_bounces=B, layout=layout, use_env=env)
    pix = None
    if how == "count":
        c = count_device(buf, W, H, **kw)
        assert c["samples"] == W * H * frames
    elif how == "present":
        pix = torch.zeros(H * W, dtype=torch.int32, device="cuda:0")
        render_device_present(buf, pix, W, H, **kw)
    else:
        render_device(buf, W, H, **kw)
    torch.cuda.synchronize()
    a = buf.cpu().numpy()
    img = a.reshape(H, W, 3) if layout == N.PT_LAYOUT_INTERLEAVED else planar8_to_interleaved(a, W, H)
    return img, (None if pix is None else pix.cpu().numpy().view(np.uint32).reshape(H, W))


DIFFUSE_ROW_CASES = (
    [(L, False, m, how) for L in (0, 1) for m in ("ct5", "ct6") for how in ("render", "count", "present")]
    + [(L, False, m, how) for L in (0, 1) for m in ("tile", "multi", "ring") for how in ("render", "count")]
    + [(L, True, "ct6", how) for L in (0, 1) for how in ("render", "count", "present")]
    + [(L, True, m, how) for L in (0, 1) for m in ("tile", "multi") for how in ("render", "count")])


@pytest.mark.parametrize("layout,env,mode,how", DIFFUSE_ROW_CASES)
def test_diffuse_row_layout_instance(lib, layout, env, mode, how):
    envs, frames = MODES[mode]
    lib(envs)
    img, pix = _device_diffuse(layout, frames, env, how)
    ref = po.render(W, H, nframes=frames, num_bounces=B, env=ENV2 if env else None)
    _check(img, ref)
    if pix is not None:   # the fused output stage = the standalone one on the same accumulator
        assert np.array_equal(pix, po.tonemap(ref))


@pytest.mark.parametrize("env,mode", [(False, m) for m in MODES] + [(True, m) for m in ("ct6", "tile", "multi")])
def test_diffuse_tiled_instance(lib, env, mode):
    """The tiled layout through the drop-in's frame calls, samples_per_frame frames per call."""
    envs, frames = MODES[mode]
    lib(envs, samples_per_frame=frames)
    buf = np.zeros(W * H * 3, np.float32)
    if env:
        pt.DemofoxRenderSimtTextured(buf, W, H, NTX, NTY, TW, TH, 3, pt.texture(ENV2, ENV2.shape[1], ENV2.shape[0], 3))
    else:
        pt.DemofoxRenderSimdTiled(buf, W, H, NTX, NTY, TW, TH, 3)
    ref = po.render(W, H, nframes=frames, num_bounces=B, env=ENV2 if env else None)
    _check(tiled_to_interleaved(buf, W, H, TW, TH), ref)


@pytest.mark.parametrize("layout", [0, 1, 2])
@pytest.mark.parametrize("fast_aces,fast_gamma", [(True, True), (True, False), (False, True), (False, False)])
def test_tonemap_instance(lib, layout, fast_aces, fast_gamma):
    """pt_tonemap_kernel<layout, fast ACES, fast gamma> (USE_FAST_APPROXIMATE_ACES_TONEMAP / _GAMMA,
    global_preprocessor_flags.h:62-63) on a synthetic accumulator in each layout."""
    from layouts import interleaved_to_planar8, interleaved_to_tiled
    lib()
    pt.v4_config(fast_aces=fast_aces, fast_gamma=fast_gamma)
    rgb = (np.random.default_rng(layout).random((H, W, 3), dtype=np.float32) * 4.0).astype(np.float32)
    acc = {0: rgb.reshape(-1), 1: interleaved_to_planar8(rgb), 2: interleaved_to_tiled(rgb, TW, TH)}[layout]
    got = pt.tonemap(acc, W, H, layout, TW if layout == 2 else 0, TH if layout == 2 else 0)
    assert np.array_equal(got, po.tonemap(rgb, fast_aces=fast_aces, fast_gamma=fast_gamma))


# ---- v4 renderer (pt_v4.hip) --------------------------------------------------------------------------
V4_ENVS = {"none": (N.PT_V4_ENV_NONE, po.ENV_NONE, None), "equirect": (N.PT_V4_ENV_EQUIRECT, po.ENV_EQUIRECT, ENV2),
           "cubemap": (N.PT_V4_ENV_CUBEMAP, po.ENV_CUBEMAP, CUBE)}
# variant -> (scene, random_jitter, rejection, fast_exp); "dfl" = the reference's default flags
V4_VARIANTS = {"dfl": ("default", True, True, True), "fast": ("default", False, True, True),
               "exact": ("default", True, True, False), "custom_fast": ("custom", True, False, True),
               "custom_exact": ("custom", True, True, False)}


def _custom_scene():
    from test_gpu_v4 import _random_scene
    s, quads, spheres, mats = _random_scene(3)
    pt.ClearScene()
    for m in mats:
        pt.AddMaterialToScene(m["albedo"], m["emissive"], m["spec_chance"], m["spec_rough"], m["spec_color"],
                              m["ior"], m["refr_chance"], m["refr_rough"], m["refr_color"])
    for q in quads:
        pt.AddQuadObjectToScene(q)
    for q in spheres:
        pt.AddSphereObjectToScene(q)
    return s


def _v4_setup(env, variant):
    mode, _, tex = V4_ENVS[env]
    scene, jit, rej, fexp = V4_VARIANTS[variant]
    pt.v4_config(env_mode=mode, random_jitter=jit, rejection=rej, num_bounces=B, fast_exp=fexp)
    if tex is not None:
        pt.set_env_map(tex)
    s = _custom_scene() if scene == "custom" else None
    return s, jit, rej, fexp


def _v4_ref(env, frames, s, jit, rej, fexp):
    _, omode, tex = V4_ENVS[env]
    return po.render4(W, H, nframes=frames, env=tex, env_mode=omode, random_jitter=jit, rejection=rej, scene=s,
                      fast_exp=fexp)


V4_ROW_CASES = ([(e, L, ct, v, False) for e in V4_ENVS for L in (0, 1) for ct in (False, True) for v in V4_VARIANTS]
                + [(e, L, ct, v, True) for e in V4_ENVS for L in (0, 1) for ct in (False, True)
                   for v in ("dfl", "custom_fast")])


@pytest.mark.parametrize("env,layout,ct,variant,count", V4_ROW_CASES)
def test_v4_row_layout_instance(lib, env, layout, ct, variant, count):
    """Device jobs: per-tile pool (3 frames) or continuous-tiles pool (8 frames, PT_MI355_V4_CT=1),
    counted launches on the default scene (the DEF counting instance) and on a custom one."""
    import torch
    from cpuperformanceraytracer_amd.device import count_v4_device, render_v4_device
    lib({"PT_MI355_V4_CT": "1"} if ct else None)
    try:
        s, jit, rej, fexp = _v4_setup(env, variant)
        frames = 8 if ct else 3
        buf = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda:0")
        kw = dict(frame_first=1, nframes=frames, num_bounces=B, layout=layout, use_env=env != "none")
        if count:
            c = count_v4_device(buf, W, H, **kw)
            assert c["samples"] == W * H * frames
        else:
            render_v4_device(buf, W, H, **kw)
        torch.cuda.synchronize()
        a = buf.cpu().numpy()
        img = a.reshape(H, W, 3) if layout == 0 else planar8_to_interleaved(a, W, H)
        _check(img, _v4_ref(env, frames, s, jit, rej, fexp))
    finally:
        pt.InitializeScene()


@pytest.mark.parametrize("env", list(V4_ENVS))
@pytest.mark.parametrize("variant", list(V4_VARIANTS) + ["present"])
def test_v4_tiled_instance(lib, env, variant):
    """DemofoxRenderOptV4 (the tiled layout, one frame per call: the per-tile pool), two calls; with
    ScreenBufferData on the default flags and scene, the presenting instance (RenderTile +
    OutputToScreen in one pass, v4 :1562-1564)."""
    lib()
    present = variant == "present"
    try:
        s, jit, rej, fexp = _v4_setup(env, "dfl" if present else variant)
        _, _, tex = V4_ENVS[env]
        t = None if tex is None else pt.texture(tex, tex.shape[1], tex.shape[0], 3)
        buf = np.zeros(W * H * 3, np.float32)
        screen = np.zeros(W * H, np.uint32) if present else None
        for _ in range(2):
            pt.DemofoxRenderOptV4(buf, W, H, NTX, NTY, TW, TH, 3, t, screen)
        ref = _v4_ref(env, 2, s, jit, rej, fexp)
        _check(tiled_to_interleaved(buf, W, H, TW, TH), ref)
        if present:
            assert np.array_equal(screen.reshape(H, W), po.tonemap(ref, po.PIXEL_XRGB8))
    finally:
        pt.InitializeScene()
