"""The non-default branches of the reference's global_preprocessor_flags.h (:60-64) on the GPU:

  ACCUMULATE_FRAMES 0                  RenderTile stores each frame's colour (v4 :1199-1250)
  USE_FAST_APPROXIMATE_EXP 0           Beer absorption by exp_ps (v4 :785-787, :973-975)
  USE_FAST_APPROXIMATE_ACES_TONEMAP 0  ACESFilm with unfused ops and '/' (v4 :172-174)
  USE_FAST_APPROXIMATE_GAMMA 0         LinearToSRGB by pow_ps (v4 :184-185)

and the bridge that applies a host's macros (include/pt_flags.h), through examples/reference_host
built with -D overrides.  Bar: BIT-EXACT against the oracles (oracle/pt_oracle_v4.c,
oracle/pt_oracle_output.c), which substitute the host libm's expf / powf for SVML's exp_ps / pow_ps
(as for its atan2 / asin / sincos); the GPU's glibc restatements (csrc/pt_libmf.h) are checked
against that libm on every relevant input by tests/test_libmf.py.
"""
from __future__ import annotations

import os
import shutil
import subprocess
from pathlib import Path

import numpy as np
import pytest

from conftest import bits_equal, mismatch_report
from layouts import tiled_to_interleaved
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


def _device_v4(w, h, frames, env, *, frame_first=1, start=None, **cfg):
    import torch
    from cpuperformanceraytracer_amd.device import ensure_backend, render_v4_device
    ensure_backend(0)
    pt.v4_config(env_mode=N.PT_V4_ENV_EQUIRECT if env is not None else N.PT_V4_ENV_NONE, **cfg)
    if env is not None:
        pt.set_env_map(env)
    init = np.zeros((h, w, 3), np.float32) if start is None else start
    buf = torch.from_numpy(init.reshape(-1).copy()).to("cuda:0")
    render_v4_device(buf, w, h, frame_first=frame_first, nframes=frames, num_bounces=8, use_env=env is not None)
    torch.cuda.synchronize()
    return buf.cpu().numpy().reshape(h, w, 3)


@pytest.mark.parametrize("fast_exp", [True, False])
@pytest.mark.parametrize("accumulate", [True, False])
def test_v4_accumulate_and_exp(accumulate, fast_exp):
    """The default glass-sphere scene: paths inside the spheres take the Beer term; frames 7..11 on a
    random non-zero start (accumulate 0 overwrites it with the last frame)."""
    w, h, frames = 192, 120, 5
    env = _tex(64, 128, seed=2)
    start = np.random.default_rng(7).random((h, w, 3), dtype=np.float32)
    got = _device_v4(w, h, frames, env, frame_first=7, start=start, accumulate_frames=accumulate, fast_exp=fast_exp)
    ref = po.render4(w, h, frame_first=7, nframes=frames, env=env, buf=start.copy(), accumulate=accumulate,
                     fast_exp=fast_exp)
    assert bits_equal(got, ref), mismatch_report(got, ref)


def test_v4_exact_exp_changes_the_image():
    """exp_ps vs approx_exp_ps differ on the paths through the glass (the switch is live)."""
    w, h = 160, 96
    env = _tex(64, 128, seed=2)
    a = po.render4(w, h, nframes=2, env=env)
    b = po.render4(w, h, nframes=2, env=env, fast_exp=False)
    assert not bits_equal(a, b)
    got = _device_v4(w, h, 2, env, fast_exp=False)
    assert bits_equal(got, b), mismatch_report(got, b)


def _special_values() -> np.ndarray:
    rng = np.random.default_rng(11)
    v = [0.0, -0.0, 1e-45, 1e-38, 0.0031308, 0.00313079, 0.0031309, 0.001, 0.5, 1.0, 1.0000001, 4.0, 16.0,
         1e30, 3.4028235e38, np.inf, -np.inf, np.nan, -1.0, -1e-3]
    r = np.concatenate([np.array(v, np.float32), rng.random(20000, dtype=np.float32) * 2.0,
                        np.exp(rng.normal(-2.0, 2.5, 20000)).astype(np.float32),
                        rng.random(4000, dtype=np.float32) * 0.01])
    n = (len(r) + 2) // 3 * 3
    return np.resize(r, n).reshape(-1, 1, 3).astype(np.float32)


@pytest.mark.parametrize("fast_aces", [True, False])
@pytest.mark.parametrize("fast_gamma", [True, False])
def test_tonemap_flag_branches(fast_aces, fast_gamma):
    """The output stage (pt_tonemap) under each ACES / gamma branch on values across the whole
    tonemap curve (0, denormals, the sRGB threshold, the saturation knee, inf, NaN, negatives)."""
    pt.init()
    pt.v4_config(fast_aces=fast_aces, fast_gamma=fast_gamma)
    rgb = _special_values()
    h, w = rgb.shape[0], 1
    for fmt in (N.PT_PIXEL_RGBA8, N.PT_PIXEL_XRGB8):
        got = pt.tonemap(rgb.reshape(-1), w, h, fmt=fmt)
        ref = po.tonemap(rgb, fmt, fast_aces=fast_aces, fast_gamma=fast_gamma)
        assert np.array_equal(got, ref), (fmt, int((got != ref).sum()))
    if not fast_gamma:   # the gamma branch changes some 8-bit pixels (the ACES one differs below 1 LSB here)
        assert not np.array_equal(po.tonemap(rgb, 0), po.tonemap(rgb, 0, fast_aces=fast_aces, fast_gamma=fast_gamma))


def test_drop_in_v4_with_all_exact_branches():
    """DemofoxRenderOptV4 + OutputToScreen + CopyOutputToFile with every exact branch selected."""
    w, h, ntx, nty = 320, 240, 10, 15
    tw, th = w // ntx, h // nty
    pt.init()
    pt.v4_config(accumulate_frames=False, fast_aces=False, fast_gamma=False, fast_exp=False)
    pt.InitializeGlobalRenderResources()
    env = _tex(64, 128, seed=21)
    tex = pt.texture(env, 128, 64, 3)
    buf = np.zeros(w * h * 3, np.float32)
    screen = np.zeros(w * h, np.uint32)
    for _ in range(3):
        pt.DemofoxRenderOptV4(buf, w, h, ntx, nty, tw, th, 3, tex, screen)
    ref = po.render4(w, h, frame_first=3, nframes=1, env=env, accumulate=False, fast_exp=False)
    got = tiled_to_interleaved(buf, w, h, tw, th)
    assert bits_equal(got, ref), mismatch_report(got, ref)
    assert np.array_equal(screen.reshape(h, w), po.tonemap(ref, po.PIXEL_XRGB8, fast_aces=False, fast_gamma=False))
    file_px = np.zeros(w * h, np.uint32)
    pt.CopyOutputToFile(buf, w, h, ntx, nty, tw, th, 3, tex, file_px)
    assert np.array_equal(file_px.reshape(h, w), po.tonemap(ref, po.PIXEL_RGBA8, fast_aces=False, fast_gamma=False))
    cfg = pt.v4_get_config()
    assert (cfg["accumulate_frames"], cfg["fast_aces"], cfg["fast_gamma"], cfg["fast_exp"]) == (0, 0, 0, 0)


def _host_texture(w=128, h=64):
    i = np.arange(w * h * 3, dtype=np.uint64)
    t = ((i * 2654435761) % (1 << 32)).astype(np.uint32).astype(np.float32) * np.float32(4.0 / 4294967296.0)
    return (t + np.float32(0.01)).astype(np.float32).reshape(h, w, 3)


@pytest.mark.parametrize("defines,kw", [
    (["ACCUMULATE_FRAMES=0", "USE_FAST_APPROXIMATE_EXP=0", "USE_FAST_APPROXIMATE_GAMMA=0",
      "USE_FAST_APPROXIMATE_ACES_TONEMAP=0"],
     dict(accumulate=False, fast_exp=False, fast_aces=False, fast_gamma=False)),
    (["USE_ENV_MAP=0", "USE_UNIT_VECTOR_REJECTION_SAMPLING=0", "PT_DEVICES=\"0,0\""],
     dict(env=False, rejection=False)),
])
def test_reference_host_with_flag_overrides(tmp_path, defines, kw):
    """examples/reference_host built with -D overrides of the reference's macros: the bridge
    (include/pt_flags.h) applies them; output = the oracle under the same switches."""
    cxx = shutil.which("g++")
    if not cxx:
        pytest.skip("g++ not available")
    exe = tmp_path / "reference_host_flags"
    pkg = ROOT / "cpuperformanceraytracer_amd"
    subprocess.run([cxx, "-std=c++17", "-O2", f"-I{ROOT / 'include'}", *[f"-D{d}" for d in defines],
                    str(ROOT / "examples" / "reference_host.cpp"), f"-L{pkg}", "-lpt_mi355", f"-Wl,-rpath,{pkg}",
                    "-o", str(exe)], check=True)
    w, h, frames = 320, 240, 3
    out, bmp = tmp_path / "v4.f32", tmp_path / "v4.bmp"
    env = dict(os.environ)
    env.pop("PT_MI355_DEVICES", None)
    r = subprocess.run([str(exe), "v4", str(w), str(h), str(frames), str(out), str(bmp)], capture_output=True,
                       text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr
    got = tiled_to_interleaved(np.fromfile(out, np.float32), w, h, w // 10, h // 15)
    accumulate = kw.get("accumulate", True)
    tex = _host_texture() if kw.get("env", True) else None
    ref = po.render4(w, h, frame_first=1 if accumulate else frames, nframes=frames if accumulate else 1, env=tex,
                     accumulate=accumulate, fast_exp=kw.get("fast_exp", True), rejection=kw.get("rejection", True))
    assert bits_equal(got, ref), mismatch_report(got, ref)
    px = po.tonemap(ref, po.PIXEL_RGBA8, fast_aces=kw.get("fast_aces", True), fast_gamma=kw.get("fast_gamma", True))
    rows = np.frombuffer(bmp.read_bytes()[54:], np.uint8).reshape(h, w, 3)[::-1, :, ::-1]   # bottom-up, BGR
    assert np.array_equal(rows, px.view(np.uint8).reshape(h, w, 4)[..., :3])


@pytest.mark.parametrize("fast_exp", [True, False])
@pytest.mark.parametrize("accumulate", [True, False])
def test_v4_ct_accumulate_and_exp(monkeypatch, accumulate, fast_exp):
    """As above through the continuous-tiles v4 kernel (PT_MI355_V4_CT=1: every launch of >= 8
    frames): 9 frames from 7."""
    monkeypatch.setenv("PT_MI355_V4_CT", "1")
    pt.init()
    w, h, frames = 136, 88, 9
    env = _tex(64, 128, seed=3)
    start = np.random.default_rng(8).random((h, w, 3), dtype=np.float32)
    got = _device_v4(w, h, frames, env, frame_first=7, start=start, accumulate_frames=accumulate, fast_exp=fast_exp)
    ref = po.render4(w, h, frame_first=7, nframes=frames, env=env, buf=start.copy(), accumulate=accumulate,
                     fast_exp=fast_exp)
    assert bits_equal(got, ref), mismatch_report(got, ref)
