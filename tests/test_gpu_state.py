"""GPU tests of the boundary's buffer and stream state (round-1 review findings):

* PT_FLAG_DEFER_READBACK with two alternating host buffers: the device mirror holds one buffer at a
  time, and handing it to the other buffer first writes the old accumulation back (nothing lost);
* PT_FLAG_PIN_HOST with the render target freed and reallocated between calls (numpy reuses the
  address): the page-lock is released by the buffer's finalizer, every call still equals the oracle;
* a deferred buffer freed or released (pt_release_buffer, ReinitializeRenderTileData) is never
  written back; the same address with another size is a new buffer;
* device jobs alternating between two HIP streams for more launches than the tile-queue ring has
  slots: a slot reused across streams waits for its previous launch (event-ordered);
* a device job on a device other than the initialised one is an error, not a silent re-init;
* a caller's stream destroyed between launches; the ring pool's guard reported as PT_EKERNEL.
All results bit-exact against the CPU oracle (oracle/pt_oracle.c).
"""
from __future__ import annotations

import gc

import numpy as np
import pytest

from conftest import bits_equal, mismatch_report
from layouts import tiled_to_interleaved
from oracle import pyoracle

pytestmark = pytest.mark.gpu

import cpuperformanceraytracer_amd as pt  # noqa: E402
from cpuperformanceraytracer_amd import _native as N  # noqa: E402


def test_deferred_alternating_buffers():
    w, h, b = 200, 120, 8
    pt.init(num_bounces=b, defer_readback=True)
    a = np.zeros((h, w, 3), np.float32)
    c = np.zeros((h, w, 3), np.float32)
    ra = np.zeros_like(a)
    rc = np.zeros_like(c)
    rc_prev = None
    for k in range(3):   # frames 1, 3, 5 -> a; 2, 4, 6 -> c (one global iFrame)
        pt.DemofoxRenderScalar(a, w, h, 3)
        pyoracle.render(w, h, frame_first=2 * k + 1, nframes=1, num_bounces=b, buf=ra)
        pt.DemofoxRenderScalar(c, w, h, 3)
        rc_prev = rc.copy()
        pyoracle.render(w, h, frame_first=2 * k + 2, nframes=1, num_bounces=b, buf=rc)
    # `a` was written back when `c` took the mirror; `c` holds what was written back when `a` took
    # it for frame 5 (frames 2, 4); its frame 6 is still device-resident
    assert bits_equal(a, ra), mismatch_report(a, ra)
    assert bits_equal(c, rc_prev), mismatch_report(c, rc_prev)
    with pytest.raises(N.PtError):
        pt.readback(a)   # no longer the deferred buffer
    pt.readback(c)
    assert bits_equal(c, rc), mismatch_report(c, rc)
    pt.shutdown()


def test_deferred_work_queue_two_buffers():
    """One work queue holding every tile of two buffers (the mirror switches inside run_queue)."""
    w, h, tw, th = 160, 96, 32, 24
    pt.init(num_bounces=4, defer_readback=True)
    bufs = [np.zeros(w * h * 3, np.float32), np.zeros(w * h * 3, np.float32)]
    q = pt.MakeWorkQueue(N.PT_RENDERER_SIMD_TILED)
    pt.BeginFrame()
    for buf in bufs:
        info = pt.RenderBufferInfo(buf, w, h, 3)
        for t in pt.make_tiles(w, h, w // tw, h // th):
            pt.AddWorkQueueEntry(q, info, t)
    pt.CompleteAllWork(q)
    q.close()
    ref = pyoracle.render(w, h, nframes=1, num_bounces=4)
    assert bits_equal(tiled_to_interleaved(bufs[0], w, h, tw, th), ref)   # written back at the switch
    pt.readback(bufs[1])
    assert bits_equal(tiled_to_interleaved(bufs[1], w, h, tw, th), ref)
    pt.shutdown()


def test_pinned_buffer_reallocated_between_calls():
    w, h, b = 640, 384, 8
    pt.init(num_bounces=b, pin_host=True)
    addrs = set()
    for k in range(4):
        a = np.zeros((h, w, 3), np.float32)   # a fresh zeroed render target (Resize)
        addrs.add(a.ctypes.data)
        pt.DemofoxRenderScalar(a, w, h, 3)    # frame k + 1 blended into zeros
        ref = pyoracle.render(w, h, frame_first=k + 1, nframes=1, num_bounces=b)
        assert bits_equal(a, ref), (k, mismatch_report(a, ref))
        del a
        gc.collect()
    # explicit unpin before a free (the C++ host's Resize calls ReinitializeRenderTileData)
    a = np.zeros((h, w, 3), np.float32)
    pt.DemofoxRenderScalar(a, w, h, 3)
    pt.unpin_host(a)
    pt.ReinitializeRenderTileData()
    pt.unpin_host(None)
    pt.DemofoxRenderScalar(a, w, h, 3)        # re-pinned on use
    ref = pyoracle.render(w, h, frame_first=5, nframes=2, num_bounces=b)
    assert bits_equal(a, ref), mismatch_report(a, ref)
    pt.shutdown()


def test_deferred_buffer_freed_then_new_size():
    """A deferred buffer is freed (its finalizer releases it: no write-back into freed memory), then
    a buffer of another size is rendered (round-2 advisor finding)."""
    pt.init(num_bounces=4, defer_readback=True)
    a = np.zeros((60, 80, 3), np.float32)
    pt.DemofoxRenderScalar(a, 80, 60, 3)
    pt.DemofoxRenderScalar(a, 80, 60, 3)
    del a
    gc.collect()
    b = np.zeros((96, 128, 3), np.float32)
    pt.DemofoxRenderScalar(b, 128, 96, 3)   # frame 3
    pt.readback(b)
    ref = pyoracle.render(128, 96, frame_first=3, nframes=1, num_bounces=4)
    assert bits_equal(b, ref), mismatch_report(b, ref)
    pt.shutdown()


def test_release_buffer_drops_without_write_back():
    """pt_release_buffer (called directly, as a C host would before free): the released buffer is
    never written to again; the same pointer with another size is treated as a new buffer; the
    host's Resize hook (ReinitializeRenderTileData) releases too."""
    L = N.load()
    pt.init(num_bounces=4, defer_readback=True)
    a = np.zeros((60, 80, 3), np.float32)
    pt.DemofoxRenderScalar(a, 80, 60, 3)
    assert not a.any()                          # deferred: nothing copied back yet
    assert L.pt_release_buffer(a.ctypes.data) == 0
    b = np.zeros((40, 64, 3), np.float32)
    pt.DemofoxRenderScalar(b, 64, 40, 3)        # would have written `a` back before taking the mirror
    assert not a.any()
    with pytest.raises(N.PtError):
        pt.readback(a)
    # the same address, another size (a reallocation in place): dropped, staged from the host
    big = np.zeros((60, 80, 3), np.float32)
    pt.DemofoxRenderScalar(big, 80, 60, 3)      # frame 3 into big's mirror
    pt.DemofoxRenderScalar(big, 64, 40, 3)      # same pointer, 64x40: not written back, re-staged
    pt.readback(big)
    ref = pyoracle.render(64, 40, frame_first=4, nframes=1, num_bounces=4)
    assert bits_equal(big.reshape(-1)[:64 * 40 * 3].reshape(40, 64, 3), ref)
    assert not big.reshape(-1)[64 * 40 * 3:].any()
    pt.ReinitializeRenderTileData()
    with pytest.raises(N.PtError):
        pt.readback(big)
    pt.shutdown()


torch = pytest.importorskip("torch")


def test_queue_ring_reuse_across_streams():
    """600 launches alternating between two streams (> the 256-slot tile-queue ring)."""
    from cpuperformanceraytracer_amd.device import render_device
    pt.shutdown()
    w, h, b, n = 96, 64, 4, 300
    bufs = [torch.zeros(h * w * 3, dtype=torch.float32, device="cuda") for _ in range(2)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    torch.cuda.synchronize()
    for f in range(n):
        for s, buf in zip(streams, bufs):
            render_device(buf, w, h, frame_first=f + 1, nframes=1, num_bounces=b, stream=s)
    torch.cuda.synchronize()
    ref = pyoracle.render(w, h, nframes=n, num_bounces=b)
    for buf in bufs:
        got = buf.cpu().numpy().reshape(h, w, 3)
        assert bits_equal(got, ref), mismatch_report(got, ref)


def test_job_on_other_device_is_an_error():
    from cpuperformanceraytracer_amd.device import ensure_backend
    pt.shutdown()
    ensure_backend(0)
    assert pt.initialized_device() == 0
    ensure_backend(0)   # no re-init: the frame counter survives
    pt.set_frame(7)
    ensure_backend(0)
    assert pt.get_frame() == 7
    with pytest.raises(N.PtError):
        ensure_backend(1)
    assert pt.initialized_device() == 0 and pt.get_frame() == 7
    pt.shutdown()
    assert pt.initialized_device() is None


class _RawStream:
    """A HIP stream the test creates and destroys itself (torch pools its streams: never destroyed)."""
    def __init__(self, handle: int):
        self.cuda_stream = handle


def test_destroyed_stream_between_launches():
    """A caller's stream destroyed between device launches on different streams: the
    library never enqueues work on a previous launch's stream, so the next launch on a new stream
    neither fails nor waits on a dead handle.  256x256 = 1024 tiles: the scheduled path with
    tile-queue ring slots skipped on every change of stream."""
    import ctypes
    from cpuperformanceraytracer_amd.device import check_device_errors, render_device
    pt.shutdown()
    hip = ctypes.CDLL("libamdhip64.so.7")   # the HIP runtime torch loaded (same soname)
    w, h, b, n = 256, 256, 4, 6
    buf = torch.zeros(h * w * 3, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    for f in range(n):
        st = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(st)) == 0
        render_device(buf, w, h, frame_first=f + 1, nframes=1, num_bounces=b, stream=_RawStream(st.value))
        assert hip.hipStreamSynchronize(st) == 0
        assert hip.hipStreamDestroy(st) == 0
    torch.cuda.synchronize()
    check_device_errors()
    ref = pyoracle.render(w, h, nframes=n, num_bounces=b)
    got = buf.cpu().numpy().reshape(h, w, 3)
    assert bits_equal(got, ref), mismatch_report(got, ref)
    pt.shutdown()


@pytest.mark.parametrize("pool", ["ct", "ring"])
def test_pool_guard_fires_loudly(monkeypatch, pool):
    """The pools' iteration guards (pt_kernel.hip: the ring pool's per-tile bound, the continuous-
    tiles pool's stall bound) end a wave only on a scheduling fault; when one fires, no call returns
    success: the host-buffer call that waited for the launch raises PtError(PT_EKERNEL) naming the
    tile, and device jobs report it through pt_check_device_errors.  PT_MI355_RING_GUARD_CAP (read
    by pt_init) lowers the guards so that they fire on a correct launch; errors are reported once,
    then the library works normally.  ring: PT_MI355_NO_CT=1 selects the ring pool (>= 48 frames)."""
    from cpuperformanceraytracer_amd.device import check_device_errors, render_device
    w, h, f = 64, 64, 49                      # >= 48 frames: one launch
    if pool == "ring":
        monkeypatch.setenv("PT_MI355_NO_CT", "1")
    monkeypatch.setenv("PT_MI355_RING_GUARD_CAP", "2")   # ct: 7 chunks per tile; ring: per-tile iterations
    pt.init(num_bounces=8, samples_per_frame=f)
    buf = np.zeros((h, w, 3), np.float32)
    with pytest.raises(N.PtError) as ei:
        pt.DemofoxRenderScalar(buf, w, h, 3)
    assert ei.value.code == N.PT_EKERNEL and "tile" in str(ei.value), str(ei.value)
    dev = torch.zeros(h * w * 3, dtype=torch.float32, device="cuda")
    render_device(dev, w, h, frame_first=1, nframes=f, num_bounces=8)   # returns when launched
    torch.cuda.synchronize()
    with pytest.raises(N.PtError) as ei:
        check_device_errors()
    assert ei.value.code == N.PT_EKERNEL
    check_device_errors()                     # reported once
    monkeypatch.delenv("PT_MI355_RING_GUARD_CAP")
    pt.init(num_bounces=8, samples_per_frame=f)
    buf[:] = 0
    pt.DemofoxRenderScalar(buf, w, h, 3)       # the normal guard never fires
    ref = pyoracle.render(w, h, nframes=f, num_bounces=8)
    assert bits_equal(buf, ref), mismatch_report(buf, ref)
    pt.shutdown()
