"""Device-resident rendering on torch tensors (HBM in, HBM out; the bench and multi-GPU path).

PyTorch is plumbing here: it owns the device allocation and the stream; the work is the HIP
kernel in libpt_mi355.so, reached through pt_render_device / pt_count_device.
"""
from __future__ import annotations

import ctypes

from . import _native as N


def ensure_backend(device_index: int, num_bounces: int = 4) -> None:
    """Initialise libpt_mi355 on `device_index` (the torch device of this rank) if it is not
    initialised yet.  The library state (env map, schedules, pinned buffer, frame counters) is per
    process; a device job runs on the logical device holding its buffer, and a job on a device the
    library was not initialised with raises PtError(PT_ESTATE) instead of silently re-initialising
    (renderer.init(devices=[...]) drives several GPUs from one process; bench.py and shard.py run one
    process per GPU).  The caller's current HIP device is restored after an initialisation."""
    from . import renderer
    cur = renderer.initialized_devices()
    if device_index in cur:
        return
    if cur:
        raise N.PtError(N.PT_ESTATE, "ensure_backend",
                        f"libpt_mi355 is initialised on devices {cur}; a job on device {device_index} needs "
                        "renderer.init(devices=[...]) naming it, or its own process")
    import torch
    prev = torch.cuda.current_device()
    try:
        renderer.init(num_bounces=num_bounces, device=device_index)
    finally:
        torch.cuda.set_device(prev)


def set_env_map(env, device_index: int = 0, num_bounces: int = 4) -> None:
    """Copy an env map (H x W x 3 f32, row 0 = bottom, as LoadTexture returns it) into HBM for
    device jobs with use_env=True; None releases it."""
    ensure_backend(device_index, num_bounces)
    from .renderer import set_env_map as _set
    _set(env)


def _job(buf, width: int, height: int, row_start: int, row_stride: int, nrows: int, frame_first: int,
         nframes: int, num_bounces: int, layout: int, use_env: bool = False) -> N.PtDeviceJob:
    import torch
    if not isinstance(buf, torch.Tensor) or buf.device.type != "cuda":
        raise N.PtError(N.PT_EINVAL, "render_device", "buf must be a device (cuda/hip) tensor")
    if buf.dtype != torch.float32 or not buf.is_contiguous():
        raise N.PtError(N.PT_EINVAL, "render_device", "buf must be contiguous float32")
    if buf.numel() < nrows * width * 3:
        raise N.PtError(N.PT_EINVAL, "render_device", f"buf holds {buf.numel()} < {nrows}x{width}x3 floats")
    ensure_backend(buf.device.index if buf.device.index is not None else torch.cuda.current_device(), num_bounces)
    return N.PtDeviceJob(buf.data_ptr(), width, height, row_start, row_stride, nrows, layout, frame_first,
                         nframes, num_bounces, 1 if use_env else 0)


def _stream(stream):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def render_device(buf, width: int, height: int, *, frame_first: int, nframes: int, num_bounces: int,
                  row_start: int = 0, row_stride: int = 1, nrows: int | None = None,
                  layout: int = N.PT_LAYOUT_INTERLEAVED, use_env: bool = False, stream=None,
                  chain: bool = False) -> None:
    """Accumulate frames [frame_first, frame_first+nframes) of global rows row_start + k*row_stride
    (k < nrows) into `buf` (nrows x width x 3 f32, in HBM).  Asynchronous on `stream`.
    use_env: miss radiance from the env map of set_env_map (config 4) instead of the ambient.
    chain: pt_render_device_chain -- this launch may overlap the previous chained launch of the same
    geometry on `stream` (same result; nothing enqueued on `stream` since that call may be needed)."""
    nrows = height if nrows is None else nrows
    job = _job(buf, width, height, row_start, row_stride, nrows, frame_first, nframes, num_bounces, layout, use_env)
    fn = "pt_render_device_chain" if chain else "pt_render_device"
    N.check(getattr(N.load(), fn)(ctypes.byref(job), _stream(stream)), fn)


def chain_counts() -> dict:
    """pt_chain_counts: chained launches since init that restarted / continued the overlap."""
    r, c = ctypes.c_uint64(0), ctypes.c_uint64(0)
    N.check(N.load().pt_chain_counts(ctypes.byref(r), ctypes.byref(c)), "pt_chain_counts")
    return {"restarts": int(r.value), "continued": int(c.value)}


def render_device_present(buf, pixels, width: int, height: int, *, frame_first: int, nframes: int,
                          num_bounces: int, row_start: int = 0, row_stride: int = 1, nrows: int | None = None,
                          layout: int = N.PT_LAYOUT_INTERLEAVED, use_env: bool = False,
                          pixel_format: int = N.PT_PIXEL_RGBA8, stream=None) -> None:
    """render_device with the output stage fused into the render (pt_render_device_present): also
    writes the job's rows as packed 8-bit pixels (nrows x width int32/uint32 device tensor `pixels`,
    PT_PIXEL_RGBA8 = OutputToFile, PT_PIXEL_XRGB8 = OutputToScreen) -- equal to render_device followed
    by the standalone output stage on those rows.  Asynchronous on `stream`."""
    nrows = height if nrows is None else nrows
    job = _job(buf, width, height, row_start, row_stride, nrows, frame_first, nframes, num_bounces, layout, use_env)
    _check_pixels(pixels, width * nrows, buf)
    N.check(N.load().pt_render_device_present(ctypes.byref(job), pixels.data_ptr(), pixel_format, _stream(stream)),
            "pt_render_device_present")


def launch_variant(buf, width: int, height: int, *, nframes: int, num_bounces: int, row_start: int = 0,
                   row_stride: int = 1, nrows: int | None = None, layout: int = N.PT_LAYOUT_INTERLEAVED,
                   use_env: bool = False) -> dict:
    """The continuous-tiles launch variant of this job's geometry (pt_launch_variant): waves per SIMD
    (0: not decided yet) and the back-claim share in percent."""
    nrows = height if nrows is None else nrows
    job = _job(buf, width, height, row_start, row_stride, nrows, 1, nframes, num_bounces, layout, use_env)
    w, b = ctypes.c_int32(0), ctypes.c_int32(0)
    N.check(N.load().pt_launch_variant(ctypes.byref(job), ctypes.byref(w), ctypes.byref(b)), "pt_launch_variant")
    return {"waves_per_simd": int(w.value), "back_claim_pct": int(b.value)}


def tonemap_device(buf, width: int, nrows: int, pixels, *, layout: int = N.PT_LAYOUT_INTERLEAVED,
                   pixel_format: int = N.PT_PIXEL_RGBA8, stream=None) -> None:
    """The standalone output stage (pt_tonemap_device) on an HBM accumulator of nrows x width pixels
    into `pixels` (nrows x width 32-bit words).  Asynchronous on `stream`."""
    _check_pixels(pixels, width * nrows, buf)
    N.check(N.load().pt_tonemap_device(buf.data_ptr(), width, nrows, layout, 0, 0, pixels.data_ptr(), pixel_format,
                                       _stream(stream)), "pt_tonemap_device")


def _check_pixels(pixels, n: int, buf) -> None:
    import torch
    if not isinstance(pixels, torch.Tensor) or pixels.device != buf.device:
        raise N.PtError(N.PT_EINVAL, "render_device_present", "pixels must be a tensor on the buffer's device")
    if pixels.element_size() != 4 or not pixels.is_contiguous() or pixels.numel() < n:
        raise N.PtError(N.PT_EINVAL, "render_device_present", f"pixels must hold >= {n} contiguous 32-bit words")


def count_device(buf, width: int, height: int, *, frame_first: int, nframes: int, num_bounces: int,
                 row_start: int = 0, row_stride: int = 1, nrows: int | None = None,
                 layout: int = N.PT_LAYOUT_INTERLEAVED, use_env: bool = False, stream=None) -> dict:
    """Like render_device (it does render into buf) but also counts the work: traced segments,
    issued lane-slots, samples, escaped paths.  Synchronous."""
    nrows = height if nrows is None else nrows
    job = _job(buf, width, height, row_start, row_stride, nrows, frame_first, nframes, num_bounces, layout, use_env)
    out = N.PtWorkCounts()
    N.check(N.load().pt_count_device(ctypes.byref(job), _stream(stream), ctypes.byref(out)), "pt_count_device")
    return {"segments": out.segments, "lane_slots": out.lane_slots, "samples": out.samples, "escaped": out.escaped,
            "primary": out.primary, "quad_fallbacks": out.quad_fallbacks, "sky_skipped": out.sky_skipped}


class JobLauncher:
    """A prepared device job: the argument checks and the ctypes job are built once, and each call
    enqueues one render (pt_render_device, or pt_v4_render_device with v4=True) changing only
    frame_first -- a launch then costs the host a few microseconds instead of the tens a full
    render_device call spends in Python (the bench's timed loop; bench.py)."""

    def __init__(self, buf, width: int, height: int, *, nframes: int, num_bounces: int, row_start: int = 0,
                 row_stride: int = 1, nrows: int | None = None, layout: int = N.PT_LAYOUT_INTERLEAVED,
                 use_env: bool = False, stream=None, v4: bool = False, pixels=None,
                 pixel_format: int = N.PT_PIXEL_RGBA8, chain: bool = False):
        nrows = height if nrows is None else nrows
        self._buf = buf   # (kept alive with the job that points at it)
        self.job = _job(buf, width, height, row_start, row_stride, nrows, 1, nframes, num_bounces, layout, use_env)
        L = N.load()
        self._ref = ctypes.byref(self.job)
        self._stream = _stream(stream)
        if pixels is not None:   # the fused output stage (pt_render_device_present)
            if v4:
                raise N.PtError(N.PT_EINVAL, "JobLauncher", "pixels: diffuse renderer only")
            _check_pixels(pixels, width * nrows, buf)
            self._pixels = pixels
            fn, args = L.pt_render_device_present, (self._ref, pixels.data_ptr(), pixel_format, self._stream)
            self._what = "pt_render_device_present"
        else:
            # chain: pt_render_device_chain / pt_v4_render_device_chain, consecutive launches overlap
            self._what = ("pt_v4_render_device" if v4 else "pt_render_device") + ("_chain" if chain else "")
            fn = getattr(L, self._what)
            args = (self._ref, self._stream)
        self._fn, self._args = fn, args

    def __call__(self, frame_first: int) -> None:
        if frame_first < 1:
            raise N.PtError(N.PT_EINVAL, self._what, "frame_first must be >= 1")
        self.job.frame_first = frame_first
        rc = self._fn(*self._args)
        if rc != N.PT_OK:
            N.check(rc, self._what)


def check_device_errors() -> None:
    """Raise PtError(PT_EKERNEL) if a device-resident launch since the last check abandoned a tile
    (pt_check_device_errors).  Call after synchronising the streams the jobs ran on."""
    N.check(N.load().pt_check_device_errors(), "pt_check_device_errors")


def render_v4_device(buf, width: int, height: int, *, frame_first: int, nframes: int, num_bounces: int = 8,
                     row_start: int = 0, row_stride: int = 1, nrows: int | None = None,
                     layout: int = N.PT_LAYOUT_INTERLEAVED, use_env: bool = False, stream=None) -> None:
    """The v4 renderer on an HBM-resident accumulator (see render_device); use_env selects the env
    mode of renderer.v4_config with the map of set_env_map.  Asynchronous on `stream`."""
    nrows = height if nrows is None else nrows
    job = _job(buf, width, height, row_start, row_stride, nrows, frame_first, nframes, num_bounces, layout, use_env)
    N.check(N.load().pt_v4_render_device(ctypes.byref(job), _stream(stream)), "pt_v4_render_device")


def count_v4_device(buf, width: int, height: int, *, frame_first: int, nframes: int, num_bounces: int = 8,
                    row_start: int = 0, row_stride: int = 1, nrows: int | None = None,
                    layout: int = N.PT_LAYOUT_INTERLEAVED, use_env: bool = False, stream=None) -> dict:
    """render_v4_device + work counters (segments, lane_slots, samples, escaped).  Synchronous."""
    nrows = height if nrows is None else nrows
    job = _job(buf, width, height, row_start, row_stride, nrows, frame_first, nframes, num_bounces, layout, use_env)
    out = N.PtWorkCounts()
    N.check(N.load().pt_v4_count_device(ctypes.byref(job), _stream(stream), ctypes.byref(out)), "pt_v4_count_device")
    return {"segments": out.segments, "lane_slots": out.lane_slots, "samples": out.samples, "escaped": out.escaped,
            "sphere_fallbacks": out.sphere_fallbacks, "sky_skipped": out.sky_skipped}
