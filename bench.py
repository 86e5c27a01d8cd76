#!/usr/bin/env python3
"""Benchmark of the MI355X path-tracing hot path (BASELINE.json metric and configs).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME]   (N > 1: starts N ranks itself)
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
         --master-port P bench.py --gpus N --steps K --warmup W [--workload NAME]

Default workload (configs[1], c2_1080p): 1920x1080, 8 spp, 8 bounces, the demofox quad+sphere
scene, diffuse+emissive.  One STEP = one launch that accumulates 8 more frames (8 spp) into the
HBM-resident f32 accumulator of every pixel -- bit-identical to 8 calls of the reference's
DemofoxRenderScalar.  Frames advance step to step like the reference's progressive render.

Scaling modes (the workload's `scaling`, config.py):
  weak    (c2..c4, v4; the default run) N > 1: the image grows to ~N x 1920x1080 pixels at the same
          aspect ratio (the same view: sqrt(N) x 1920 by sqrt(N) x 1080, e.g. 3840x2160 for N = 4)
          and every rank renders its interleaved 1/N of the rows, ~1920x1080 pixels (shard.py);
          after the K steps the sub-images are gathered to rank 0 over RCCL (inside the timed
          region, also reported as gather_ms).
  strong  (c5_8k, configs[4]) the image is FIXED at 7680x4320, 256 spp, 8 bounces: a step renders
          the whole image once (256 frames) -- rank r the rows r::N -- and gathers it to rank 0
          over RCCL (the job's only exchange), so every step ends with the complete image on
          rank 0.  Per-step render and gather times are reported (render_ms_per_step, gather_ms).

PT_BENCH_REHEARSE=1 runs the N-rank code on ONE GPU (every rank on cuda:0, gloo, gathers through
host memory): correctness of the multi-rank path, not scaling numbers; --verify-rows (default 2
when rehearsing) then checks sampled rows of rank 0's gathered image against a single-rank render
of the same rows and frames, bit for bit.

Printed (rank 0, one JSON line): the BASELINE metric (ray-samples/s = pixels x spp x bounces / s),
ms per step, a roofline object for the render kernel (algorithmic FP32 FLOP/s against the 157.3
TFLOP/s FP32 vector peak; HBM traffic from the committed rocprofv3 PMC pass), and the CPU baseline
(the oracle's C restatement of the reference scalar path on this host's cores, bounded sample).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "ray-samples/sec (pixels×spp×bounces) at 1920×1080; ms/frame"


def metric_label(W: int, H: int) -> str:
    """BASELINE.json's metric string for the headline 1920x1080 workloads; other images (c3's 4K, the
    configs[4] leg's 7680x4320) name their own size in the same form."""
    return METRIC if (W, H) == (1920, 1080) else METRIC.replace("1920×1080", f"{W}×{H}")


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # c2: 100 steps of 0.3 ms (the launch latency before the first step and the final
    # synchronisation stay out of the per-step time); c5_8k: 5 steps of ~150 ms (one GPU)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c2_1080p")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-chain", action="store_true",
                    help="plain pt_render_device / pt_v4_render_device steps, one after the other, instead of chained "
                         "launches (pt_render_device_chain) that overlap consecutive steps")
    ap.add_argument("--no-configs4", action="store_true",
                    help="default workload: skip the configs[4] strong-scaling leg (c5_8k, a few steps)")
    ap.add_argument("--device-warmup-ms", type=float, default=60.0,
                    help="untimed GPU work before the warmup steps (clock ramp; 0 = none)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="wall time of the CPU baseline sample (whole frames of the workload)")
    ap.add_argument("--verify-rows", type=int, default=None,
                    help="rank 0: compare this many sampled rows of the gathered image with a single-rank "
                         "render of the same rows (default 2 with PT_BENCH_REHEARSE=1, else 0)")
    a = ap.parse_args(argv)
    return a


def default_steps(wl) -> int:
    return 5 if wl.scaling == "strong" else 100


def host_cpu_share() -> dict:
    """The CPUs this process may use on the host: the affinity mask and, where the cgroup sets one,
    the CPU quota (cpu.max: quota/period).  On the GPU box the affinity mask shows the whole machine
    while the cgroup quota is the box's share."""
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    quota = None
    for p in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(p).read().split()[:2]
            if q != "max":
                quota = float(q) / float(per)
        except (OSError, ValueError):
            pass
    if quota is None:
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    usable = affinity if quota is None else max(1, min(affinity, int(math.floor(quota + 1e-6))))
    # the GPU box declares its CPU share in OMP_NUM_THREADS (16 per GPU; the affinity mask there
    # lists the whole machine): honour it as the cap when it is set
    omp = os.environ.get("OMP_NUM_THREADS")
    try:
        if omp is not None and int(omp) > 0:
            usable = min(usable, int(omp))
    except ValueError:
        pass
    return {"affinity_cpus": affinity, "cgroup_cpu_quota": quota, "omp_num_threads": omp, "threads": usable,
            "rule": "threads = min(affinity mask, cgroup CPU quota, OMP_NUM_THREADS) -- the CPUs this job may use"}


def cpu_baseline(wl, seconds: float, env=None) -> dict:
    """The oracle (C restatement of demofox_path_tracing_scalar.cpp, bit-identical to the
    reference's own scalar build) timed on this host's cores -- every CPU the cgroup quota and the
    affinity mask grant this process -- on a bounded sample of the same workload: full-size frames,
    as many as fit in about `seconds` of wall time.  Beside it the reference's CPU SIMD path (an
    AVX2 port of simt_pooled, `simd_port`; the value reported is the faster of the two CPU paths,
    which is the scalar restatement: the SIMD file traces every bounce of every lane under masks).
    The reference's own compiled scalar code is never shipped to the GPU box; its
    per-core rate relative to the restatement is the build-container calibration
    (profiles/cpu_calibration.json), quoted as `reference_scalar_calibration`."""
    from oracle import pyoracle
    share = host_cpu_share()
    cores = share["threads"]
    if wl.renderer == "v4":
        return cpu_baseline_v4(wl, seconds, env, cores, share)
    kw = dict(num_bounces=wl.num_bounces, nthreads=cores, env=env)
    t0 = time.perf_counter()
    pyoracle.render(wl.width, wl.height, frame_first=1, nframes=1, **kw)      # calibration frame
    t1 = time.perf_counter() - t0
    frames = int(max(1, min(1024, round(seconds / max(t1, 1e-6)))))
    t0 = time.perf_counter()
    pyoracle.render(wl.width, wl.height, frame_first=2, nframes=frames, **kw)
    dt = time.perf_counter() - t0
    samples = wl.width * wl.height * frames
    out = {"value": samples * wl.num_bounces / dt, "unit": "ray-samples/s", "cores": cores, "kind": "port",
           "sample": f"{wl.width}x{wl.height}, {frames} frames (spp), {wl.num_bounces} bounces, "
                     f"oracle/pt_oracle.c (gcc -O2, {cores} threads, row-cyclic){', env map' if env is not None else ''}; "
                     f"{dt:.2f} s wall",
           "primary_samples_per_s": samples / dt, "host_cpu_share": share, "cpu_model": _cpu_model()}
    if env is None:
        out["simd_port"] = cpu_simd_port(wl, seconds / 2, cores)
    cal = ROOT / "profiles" / "cpu_calibration.json"
    if cal.exists():
        out["reference_scalar_calibration"] = {"file": "profiles/cpu_calibration.json",
                                               "note": "reference scalar build vs this restatement, one core, "
                                                       "measured in the build container (the reference's compiled "
                                                       "code does not travel to the GPU box)"}
    return out


def cpu_simd_port(wl, seconds: float, cores: int) -> dict:
    """The reference's CPU SIMD path (demofox_path_tracing_simt_pooled.cpp: 8 pixels per AVX2 register,
    per-lane RNG, all bounces under masks, a thread pool over tiles) as an AVX2 port
    (oracle/pt_cpu_simd.c; the MSVC/SVML original cannot be built here), same workload, NUM_TILES 10x15."""
    from oracle import pyoracle
    if not pyoracle.simd_supported():
        return {"skipped": "host CPU lacks AVX2/FMA"}
    kw = dict(num_bounces=wl.num_bounces, nthreads=cores)
    t0 = time.perf_counter()
    buf = pyoracle.render_simd_tiled(wl.width, wl.height, 10, 15, frame_first=1, nframes=1, **kw)
    t1 = time.perf_counter() - t0
    frames = int(max(1, min(1024, round(seconds / max(t1, 1e-6)))))
    t0 = time.perf_counter()
    pyoracle.render_simd_tiled(wl.width, wl.height, 10, 15, frame_first=2, nframes=frames, buf=buf, **kw)
    dt = time.perf_counter() - t0
    samples = wl.width * wl.height * frames
    return {"value": samples * wl.num_bounces / dt, "unit": "ray-samples/s", "cores": cores, "kind": "port",
            "sample": f"{wl.width}x{wl.height}, {frames} frames, {wl.num_bounces} bounces, AVX2+FMA port of "
                      f"demofox_path_tracing_simt_pooled.cpp (oracle/pt_cpu_simd.c, {cores} threads); {dt:.2f} s wall",
            "primary_samples_per_s": samples / dt}


def cpu_baseline_v4(wl, seconds: float, env, cores: int, share: dict) -> dict:
    """The v4 oracle (oracle/pt_oracle_v4.c, the restatement the kernel matches bit for bit) on
    this host's cores, whole frames of the workload for about `seconds`."""
    from oracle import pyoracle
    kw = dict(num_bounces=wl.num_bounces, nthreads=cores, env=env)
    t0 = time.perf_counter()
    pyoracle.render4(wl.width, wl.height, frame_first=1, nframes=1, **kw)
    t1 = time.perf_counter() - t0
    frames = int(max(1, min(1024, round(seconds / max(t1, 1e-6)))))
    t0 = time.perf_counter()
    pyoracle.render4(wl.width, wl.height, frame_first=2, nframes=frames, **kw)
    dt = time.perf_counter() - t0
    samples = wl.width * wl.height * frames
    return {"value": samples * wl.num_bounces / dt, "unit": "ray-samples/s", "cores": cores, "kind": "port",
            "sample": f"{wl.width}x{wl.height}, {frames} frames (spp), {wl.num_bounces} bounces, v4 default scene + "
                      f"env map, oracle/pt_oracle_v4.c (gcc -O2, {cores} threads, row-cyclic); {dt:.2f} s wall",
            "primary_samples_per_s": samples / dt, "host_cpu_share": share, "cpu_model": _cpu_model()}


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def load_pmc(workload: str) -> dict:
    """The committed rocprofv3 PMC summary of this workload's render kernel (profiles/pmc_summary.json
    for the headline c2, pmc_summary_<workload>.json else): HBM bytes per launch, VALU counts."""
    p = ROOT / "profiles" / ("pmc_summary.json" if workload == "c2_1080p" else f"pmc_summary_{workload}.json")
    if not p.exists():
        return {}
    return json.loads(p.read_text())


def weak_image(W: int, H: int, world: int) -> tuple[int, int]:
    """The global image of an N-rank weak-scaling run: W x H scaled by sqrt(N) in both directions
    (width a multiple of 8), so it shows the same view at N times the pixels and every rank's
    interleaved rows hold ~W x H pixels.  (Growing only the height would change the camera's aspect
    ratio and with it what the rows see -- mostly sky for a tall image.)"""
    if world == 1:
        return W, H
    s = math.sqrt(world)
    Wg = max(8, int(round(W * s / 8.0)) * 8)
    Hg = max(world, int(round(Wg * H / W)))
    return Wg, Hg


def job_image(wl, world: int) -> tuple[int, int]:
    """The global image of an N-rank run: fixed for strong scaling (configs[4]), grown for weak."""
    if wl.scaling == "strong":
        return wl.width, wl.height
    return weak_image(wl.width, wl.height, world)


def measure_output_stage(buf, W: int, H: int, stream) -> dict:
    """the output stage (ACES + sRGB + 8-bit pack, v4 :1260-1331) on this
    rank's accumulator -- an HBM-bound pass: 12 B read + 4 B written per pixel."""
    import ctypes
    import torch
    from cpuperformanceraytracer_amd import _native as N
    from cpuperformanceraytracer_amd import roofline as RL
    out = torch.empty(W * H, dtype=torch.int32, device=buf.device)
    L = N.load()
    args = (buf.data_ptr(), W, H, N.PT_LAYOUT_INTERLEAVED, 0, 0, out.data_ptr(), N.PT_PIXEL_RGBA8,
            ctypes.c_void_p(stream.cuda_stream))
    for _ in range(3):
        N.check(L.pt_tonemap_device(*args), "pt_tonemap_device")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    e0.record(stream)
    for _ in range(reps):
        L.pt_tonemap_device(*args)
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    nbytes = 16 * W * H
    return {"kernel": "pt_tonemap_kernel<INTERLEAVED>", "pixels": W * H, "ms": ms,
            "bound": "hbm", "achieved_gbps": nbytes / (ms * 1e-3) / 1e9, "peak_gbps": RL.PEAK_HBM_GBPS,
            "frac": nbytes / (ms * 1e-3) / 1e9 / RL.PEAK_HBM_GBPS, "bytes": nbytes}


def measure_fused_output(make_launcher, W: int, nrows: int, S: int, stream, frame0: int, reps: int = 20,
                         rounds: int = 3) -> dict:
    """The output stage fused into the render (pt_render_device_present: each pixel's 8-bit value
    written by the continuous-tiles kernel at its last fold) -- its cost is the difference between
    launches that present and launches that do not, interleaved (`rounds` x `reps` launches each) on
    a scratch accumulator of the step's geometry.  make_launcher(buf, pixels) -> launch(frame)."""
    import torch
    buf = torch.zeros(nrows * W * 3, dtype=torch.float32, device=stream.device)
    pix = torch.zeros(nrows * W, dtype=torch.int32, device=stream.device)
    plain, fused = make_launcher(buf, None), make_launcher(buf, pix)
    t = {"plain": 0.0, "fused": 0.0}
    frame = frame0
    for _ in range(2):   # (the scratch geometry's schedule: built from the 2nd launch on)
        plain(frame)
        frame += S
    for _ in range(rounds):
        for name, fn in (("plain", plain), ("fused", fused)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(reps):
                fn(frame)
                frame += S
            e1.record(stream)
            torch.cuda.synchronize()
            t[name] += e0.elapsed_time(e1)
    n = rounds * reps
    plain_ms, fused_ms = t["plain"] / n, t["fused"] / n
    return {"launch_ms": plain_ms, "presenting_launch_ms": fused_ms, "extra_ms": fused_ms - plain_ms,
            "pixels": W * nrows, "launches": n,
            "note": "pt_render_device_present vs pt_render_device, interleaved launches of the step's geometry; "
                    "extra_ms = the fused output stage's cost per presented frame (the standalone pass: ms above)"}


class DeviceOps:
    """Timing / synchronisation of the GPU run: HIP events on the render stream (torch.cuda)."""

    def __init__(self, dev, stream):
        self.dev, self.stream = dev, stream

    def event(self):
        import torch
        return torch.cuda.Event(enable_timing=True)

    def record(self, e):
        e.record(self.stream)

    def elapsed_ms(self, a, b) -> float:
        return a.elapsed_time(b)

    def sync(self):
        import torch
        torch.cuda.synchronize(self.dev)

    def zeros(self, n):
        import torch
        return torch.zeros(n, dtype=torch.float32, device=self.dev)


class HostOps:
    """The same interface on the host clock (tests of the N-rank path on CPU, gloo)."""

    def __init__(self):
        self.dev = "cpu"

    def event(self):
        return [0.0]

    def record(self, e):
        e[0] = time.perf_counter()

    def elapsed_ms(self, a, b) -> float:
        return (b[0] - a[0]) * 1e3

    def sync(self):
        pass

    def zeros(self, n):
        import torch
        return torch.zeros(n, dtype=torch.float32)


def reduce_values(vals, op, *, world: int, dev, rehearse: bool = False, force_collective: bool = False) -> list:
    """vals (numbers) reduced over the ranks with the ReduceOp `op`: an all-reduce of one f64 tensor, on
    the rank's device under RCCL (nccl), in host memory under gloo (CPU tests, PT_BENCH_REHEARSE).  One
    rank returns the values themselves, unless force_collective (the RCCL call an N-GPU run makes,
    executed on one GPU by tests/test_gpu_rccl.py).  Counts stay exact below 2^53."""
    import torch
    import torch.distributed as dist
    if world == 1 and not force_collective:
        return [float(v) for v in vals]
    t = torch.tensor([float(v) for v in vals], dtype=torch.float64)
    if not rehearse and str(dev) != "cpu" and dist.get_backend() == "nccl":
        t = t.to(dev)
    dist.all_reduce(t, op=op)
    return [float(v) for v in t.tolist()]


def run(args, wl, rank: int, world: int, ops, render_fn, count_fn, *, rehearse: bool = False,
        roofline: bool = True, chain_counts=None) -> dict | None:
    """The timed job of one rank (both scaling modes); returns rank 0's result dict (None elsewhere).

    render_fn(buf, Wg, Hg, frame_first, nframes, row_start, row_stride, nrows) renders asynchronously
    into buf; count_fn(...) the same, synchronously, returning the work counters.  Multi-rank runs
    need torch.distributed initialised (RCCL, or gloo when rehearsing / on CPU).
    chain_counts: () -> {"restarts", "continued"} (pt_chain_counts) when render_fn takes chain=True
    (pt_render_device_chain): the weak-scaling steps are then chained launches -- consecutive steps
    overlap on the GPU, each pixel's frames still folded in order -- and the line reports
    how many of the timed launches continued the overlap.  Strong-scaling steps (a gather of the image
    between them) are never chained."""
    import torch
    import torch.distributed as dist
    from cpuperformanceraytracer_amd import roofline as RL
    from cpuperformanceraytracer_amd.shard import gather_rows, max_rows, rows_of

    S, B = wl.spp, wl.num_bounces
    strong = wl.scaling == "strong"
    Wg, Hg = job_image(wl, world)
    row_start, row_stride, nrows = rows_of(rank, world, Hg)
    mr = max_rows(world, Hg)
    buf = ops.zeros(mr * Wg * 3)
    K = args.steps if args.steps is not None else default_steps(wl)
    verify_rows = args.verify_rows if args.verify_rows is not None else (2 if rehearse else 0)
    frame = 1

    chained = chain_counts is not None and not strong
    chain_kw = {"chain": True} if chained else {}

    def step(f):
        render_fn(buf, Wg, Hg, f, S, row_start, row_stride, nrows, **chain_kw)

    def gather():
        return gather_rows(buf.cpu() if rehearse else buf, Wg, Hg, rank, world)

    def all_ranks(vals, op):
        return reduce_values(vals, op, world=world, dev=ops.dev, rehearse=rehearse)

    # Device warm-up, untimed, before the W warmup steps: the MI355X reaches its steady clocks only
    # after ~25 ms of sustained load (per-launch time at 1080p, 8 spp: 0.46 ms over the first 20
    # launches, 0.379 over the next 20, 0.357 from the 60th on -- scripts/clock_ramp.py), and the
    # reference's progressive renderer runs continuously.  Reported as "device_warmup".
    # Every rank accumulates the same frames: the decision to run another warm-up batch is taken by
    # all ranks together (another batch while ANY rank is under the time budget).  Decided per rank,
    # two ranks whose clocks crossed the budget in different batches accumulated different frame
    # ranges -- the rows-763 mismatch of the round-4 two-process rehearsals.
    dw_ms, dw_steps = 0.0, 0
    batch = 1 if strong else 10
    while all_ranks([float(dw_ms < args.device_warmup_ms and dw_steps < 4000)], dist.ReduceOp.MAX)[0] > 0:
        e0, e1 = ops.event(), ops.event()
        ops.record(e0)
        for _ in range(batch):
            step(frame)
            frame += S
        ops.record(e1)
        ops.sync()
        dw_ms += ops.elapsed_ms(e0, e1)
        dw_steps += batch
    for _ in range(args.warmup):
        step(frame)
        frame += S
    ops.sync()
    if world > 1:
        dist.barrier()
    ops.sync()
    # Two events bracket the K launches on their stream: the average launch duration is their
    # interval / K (back to back, so it includes the inter-launch gaps: an upper bound of the kernel
    # time; it agrees with rocprofv3's kernel-trace average).  An event pair around EVERY launch
    # would add ~9 us per step to the timed region (scripts/event_overhead.py), so per-launch pairs
    # are recorded only in an untimed pass after it (kernel_ms_event_pairs).  Strong scaling: the
    # step's render and its gather are bracketed separately (render_ms, gather_ms per step).
    timed_first = frame
    full = None
    render_ms = gather_ms = 0.0
    cc0 = chain_counts() if chained else None
    t0 = time.perf_counter()
    if strong:
        for k in range(K):
            ea, eb, ec = ops.event(), ops.event(), ops.event()
            ops.record(ea)
            step(frame)
            frame += S
            ops.record(eb)
            if world > 1:
                full = gather()
            ops.record(ec)
            ops.sync()
            render_ms += ops.elapsed_ms(ea, eb)
            gather_ms += ops.elapsed_ms(eb, ec)
        launch_ms_avg = render_ms / K
    else:
        ev_a, ev_b = ops.event(), ops.event()
        ops.record(ev_a)
        for k in range(K):
            step(frame)
            frame += S
        ops.record(ev_b)
        if world > 1:
            g0, g1 = ops.event(), ops.event()
            ops.record(g0)
            full = gather()
            ops.record(g1)
    ops.sync()
    if world > 1:
        dist.barrier()
    ops.sync()
    elapsed = time.perf_counter() - t0
    timed_end = frame
    cc1 = chain_counts() if chained else None
    lo, hi = all_ranks([-timed_end, timed_end], dist.ReduceOp.MAX)
    if -lo != hi:   # (the invariant the gathered image and its check rely on)
        raise AssertionError(f"the ranks accumulated different frame ranges: ends {-lo:.0f} .. {hi:.0f}")
    if not strong:
        launch_ms_avg = ops.elapsed_ms(ev_a, ev_b) / K
        if world > 1:
            gather_ms = ops.elapsed_ms(g0, g1)
    if world > 1:
        elapsed, gather_ms, launch_ms_avg = all_ranks([elapsed, gather_ms, launch_ms_avg], dist.ReduceOp.MAX)
        if rank == 0:
            assert full is not None and tuple(full.shape) == (Hg, Wg, 3)

    verified = None
    if rank == 0 and verify_rows > 0 and full is not None:
        # the gathered rows against a single-rank render of the same rows and frames (frames
        # [1, timed_end) have been accumulated into a zeroed buffer when the gather ran)
        import numpy as np
        ys = sorted({int(v) for v in np.linspace(0, Hg - 1, verify_rows + 2)[1:-1]} | {Hg // 2})
        one = ops.zeros(Wg * 3)
        bad = []
        for y in ys:
            one.zero_()
            render_fn(one, Wg, Hg, 1, timed_end - 1, y, 1, 1)
            ops.sync()
            got = full[y].reshape(-1).cpu().numpy().view(np.uint32)
            if not np.array_equal(one.cpu().numpy().view(np.uint32), got):
                bad.append(y)
        verified = {"rows": ys, "frames": [1, timed_end - 1], "bit_exact": not bad, "mismatch_rows": bad}
        if bad:
            raise AssertionError(f"gathered rows {bad} differ from the single-rank render")

    # Untimed: per-launch event pairs (the event overhead lands inside each pair).
    pairs = [(ops.event(), ops.event()) for _ in range(min(K, 20))]
    for a, b in pairs:
        ops.record(a)
        step(frame)
        ops.record(b)
        frame += S
    ops.sync()
    pair_ms = [ops.elapsed_ms(a, b) for a, b in pairs]

    # Exact work of the timed launches (deterministic: same frames, counted on a scratch buffer).
    scratch = ops.zeros(mr * Wg * 3)
    segs = samples = slots = prim = escaped = sky = 0
    for k in range(K):
        c = count_fn(scratch, Wg, Hg, timed_first + k * S, S, row_start, row_stride, nrows)
        escaped += c["escaped"]
        segs += c["segments"]
        samples += c["samples"]
        slots += c["lane_slots"]
        prim += c.get("primary", c["samples"])
        sky += c.get("sky_skipped", 0)
    del scratch
    if world > 1:   # whole-job work: summed over ranks
        segs, samples, slots, prim, escaped, sky = (
            int(v) for v in all_ranks([segs, samples, slots, prim, escaped, sky], dist.ReduceOp.SUM))
    if rank != 0:
        return None

    v4 = wl.renderer == "v4"
    ms_step = elapsed * 1e3 / K
    total_ray_samples = Wg * Hg * S * B * K
    value = total_ray_samples / elapsed
    avg_kernel_s = launch_ms_avg / 1e3
    # per-launch figures of ONE rank's kernel (the roofline is per GPU): the whole-job counts / world
    per_rank = 1.0 / world
    if v4:   # every frame traces its own jittered camera ray
        flops_launch = RL.v4_launch_flops(segs, samples) / K * per_rank
        flops_launch_ref = flops_launch
        flop_model = (f"segments x V4_F_SEGMENT + samples x V4_F_SAMPLE; F = {RL.V4_F_SEGMENT}/{RL.V4_F_SAMPLE} "
                      "(roofline.py, counted by oracle/pt_oracle_v4.c)")
        # pt_v4.hip launch_t: the continuous-tiles kernel for launches of >= 4 8-frame chunks per
        # resident wave (6144 at its 6 waves per SIMD on MI355X), the per-tile pool kernel else (this
        # label mirrors that rule)
        tiles = ((Wg + 7) // 8) * (((Hg + world - 1) // world + 7) // 8)
        v4_ct = os.environ.get("PT_MI355_NO_CT") != "1" and S >= 8 and (
            os.environ.get("PT_MI355_V4_CT") == "1" or S * tiles >= 4 * 8 * 6144)
        kernel_name = "pt_v4_ct_kernel<EQUIRECT, INTERLEAVED>" if v4_ct else "pt_v4_kernel<EQUIRECT, INTERLEAVED>"
    else:
        env_esc = escaped if wl.env else 0
        flops_launch = RL.launch_flops_alg(segs, samples, env_esc) / K * per_rank
        flops_launch_ref = RL.launch_flops_ref(segs, prim, samples, env_esc) / K * per_rank
        flop_model = ("algorithmic (SURVEY.md §8d) = device-counted segments x F_SEGMENT + samples x F_SAMPLE"
                      + (" + escaped paths x F_ENV_ESCAPE" if wl.env else "") +
                      f"; F = {RL.F_SEGMENT}/{RL.F_SAMPLE}" + (f"/{RL.F_ENV_ESCAPE}" if wl.env else "") +
                      " (roofline.py; a pixel's camera ray is one segment)")
        # the continuous-tiles kernels (pt_kernel.hip render_body_ct) unless PT_MI355_NO_CT=1
        ct = os.environ.get("PT_MI355_NO_CT") != "1"
        kernel_name = (("pt_render_ct_env_kernel" if ct else "pt_render_env_kernel") if wl.env else
                       ("pt_render_ct_kernel" if ct else "pt_render_kernel")) + "<INTERLEAVED>"
    achieved_tf = flops_launch / avg_kernel_s / 1e12
    pmc = load_pmc(wl.name) if roofline else {}
    # config 4: one 12-byte texel gather per escaping path
    env_bytes = RL.BYTES_PER_ENV_GATHER * escaped / K * per_rank if wl.env else 0
    alg_bytes = RL.BYTES_PER_PIXEL_PER_LAUNCH * Wg * nrows + env_bytes
    valu = None
    if pmc.get("sq_insts_valu_per_launch"):
        valu = {"wave_insts_per_launch": pmc["sq_insts_valu_per_launch"],
                "per_simd_per_ns": pmc["sq_insts_valu_per_launch"] / (avg_kernel_s * 1e9 * 1024.0),
                "ceiling_2cycle_ops": 1.0,
                "source": pmc.get("source"),
                "note": "SQ_INSTS_VALU of the committed PMC pass over this run's kernel time and the 1024 SIMDs; "
                        "2-cycle f32 ops issue at ~1.0 per SIMD per ns, the 4-cycle class (compares, selects, "
                        "min/max, f64, conversions) at ~0.58 (DESIGN.md §3)"}
    launch_chain = {"enabled": False}
    if chained:
        launch_chain = {"enabled": True, "timed_restarts": cc1["restarts"] - cc0["restarts"],
                        "timed_continued": cc1["continued"] - cc0["continued"],
                        "note": "pt_render_device_chain: consecutive steps overlap on two streams (the next "
                                "launch's waves fill the CUs the finishing ones free); a launch touches a tile "
                                "only after the previous one stored it, so every pixel's frames fold in order "
                                "(DESIGN.md 3e).  kernel_ms_avg is then the per-step time of the overlapped "
                                "launches, not one launch's duration"}
    res = {
        "metric": metric_label(wl.width, wl.height),
        "value": value,
        "unit": "ray-samples/s",
        "n_gpus": world,
        "steps": K,
        "warmup": args.warmup,
        "device_warmup": {"steps": dw_steps, "ms": round(dw_ms, 3)},
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": wl.scaling,
        "vs_baseline": None,
        "dtype": "f32",
        "data": ("synthetic (the reference's v4 InitializeScene: 4 quads + 7 glass spheres; no dataset)" if v4 else
                 "synthetic (the reference's fixed demofox quad+sphere scene; no dataset)") + (
            "; env map: 2048x1024 log-normal f32, seed 0xC0FFEE, standing in for the missing chinese_garden_2k.hdr"
            if wl.env else ""),
        "config": {"workload": wl.name, "width": wl.width, "height": wl.height, "spp": S, "bounces": B,
                   "image": [Wg, Hg], "parallelism": f"rows interleaved x{world}" if world > 1 else "single GPU",
                   "step": (f"one pass of the fixed {Wg}x{Hg} image ({S} frames) on all ranks + RCCL gather to rank 0"
                            if strong else f"one launch accumulating {S} frames (spp) of every pixel in HBM")},
        "primary_samples_per_s": Wg * Hg * S * K / elapsed,
        "ms_per_frame_1spp": ms_step / S,
        "traced_segments_per_s": segs / (avg_kernel_s * K),
        "segments_per_sample": segs / samples,
        "ref_segments_per_sample": (segs if v4 else RL.ref_segments(segs, prim, samples)) / samples,
        "simd_lane_efficiency": segs / slots if slots else None,
        "sky_skipped_traces_per_launch": sky / K * per_rank,
        "launch_chain": launch_chain,
        "kernel_ms_avg": avg_kernel_s * 1e3,
        "kernel_ms_source": ("per step: HIP events around the render launch on its stream (max over ranks)" if strong
                             else "HIP events bracketing the K timed launches on their stream, interval / K"),
        "kernel_ms_event_pairs": {"launches": len(pair_ms), "avg": sum(pair_ms) / len(pair_ms), "min": min(pair_ms),
                                  "note": "untimed pass, an event pair around each launch"},
        "roofline": {
            "bound": "valu",
            "achieved": achieved_tf,
            "peak": RL.PEAK_FP32_TFLOPS,
            "unit": "TFLOP/s",
            "frac": achieved_tf / RL.PEAK_FP32_TFLOPS,
            "traffic": pmc.get("hbm_bytes_per_launch"),
            "kernel": kernel_name,
            "flops_per_launch": flops_launch,
            "flop_model": flop_model,
            "flops_per_launch_ref_equivalent": flops_launch_ref,
            "achieved_ref_equivalent": flops_launch_ref / avg_kernel_s / 1e12,
            "algorithmic_bytes_per_launch": alg_bytes,
            "hbm_achieved_gbps": alg_bytes / avg_kernel_s / 1e9,
            "hbm_peak_gbps": RL.PEAK_HBM_GBPS,
            "traffic_source": pmc.get("source"),
            "valu_issue": valu,
        },
    }
    if world > 1:
        res["gather_ms"] = gather_ms / K if strong else gather_ms
        res["gather_bytes"] = Wg * Hg * 12
        if strong:
            res["render_ms_per_step"] = launch_ms_avg
            res["gather_note"] = "per step: the RCCL gather of the sub-images to rank 0 + un-interleave (max over ranks)"
        if rehearse:
            res["rehearsal"] = "PT_BENCH_REHEARSE=1: all ranks on one GPU, gloo, host-memory gather (not scaling numbers)"
    if verified is not None:
        res["verified"] = verified
    res["_accumulator"] = buf   # (popped by main: the output stage runs on the rendered accumulator)
    return res


def strong_leg(wl4, rank: int, world: int, ops, render_fn, count_fn, *, rehearse: bool = False,
               steps: int = 3) -> dict | None:
    """BASELINE configs[4] beside the default line: the FIXED image of the strong-scaling workload
    (c5_8k: 7680x4320, 256 spp, 8 bounces), rows r::N per rank, each step one render + the RCCL
    gather of the sub-images to rank 0 (both timed, reported separately), a few steps -- so the
    driver's N = 1, 2, 4, 8 runs of the default line also trace configs[4]'s scaling curve.  The
    gathered image is checked against a single-rank render of two rows.  Rank 0 returns a summary."""
    a4 = parse(["--gpus", str(world), "--steps", str(steps), "--warmup", "1", "--device-warmup-ms", "0",
                "--verify-rows", "2" if world > 1 else "0"])
    r = run(a4, wl4, rank, world, ops, render_fn, count_fn, rehearse=rehearse, roofline=False)
    if r is None:
        return None
    r.pop("_accumulator", None)
    keep = ("metric", "value", "unit", "n_gpus", "steps", "ms_per_step", "scaling", "config", "kernel_ms_avg",
            "render_ms_per_step", "gather_ms", "gather_bytes", "verified", "primary_samples_per_s")
    out = {k: r[k] for k in keep if k in r}
    if world == 1:   # one GPU renders the whole image: the step is the render alone
        out["render_ms_per_step"] = r["kernel_ms_avg"]
        out["gather_ms"] = 0.0
    out["note"] = ("BASELINE configs[4] (the fixed 7680x4320 image, 256 spp, 8 bounces), strong scaling: every "
                   "step renders the whole image over the N ranks (rows r::N) and gathers it to rank 0 over "
                   "RCCL; value = ray-samples/s of the whole job, render and gather per step reported apart")
    return out


class Hooks:
    """What `drive` needs beyond bench.run's render/count functions: check_errors() raises on a device
    error the run left (PT_EKERNEL); launch_variant(buf, Wg, Hg, rs, st, nr) -> dict, the
    continuous-tiles variant the timed launches picked (None: not reported); output_stage(buf, res)
    -> dict, rank 0's output-stage measurement on its accumulator (None: skipped); cpu_baseline()
    -> dict (None: skipped)."""

    def __init__(self, check_errors=None, launch_variant=None, output_stage=None, cpu_baseline=None,
                 chain_counts=None):
        self.check_errors = check_errors or (lambda: None)
        self.chain_counts = chain_counts   # (bench.run: render_fn takes chain=True)
        self.launch_variant = launch_variant
        self.output_stage = output_stage
        self.cpu_baseline = cpu_baseline


def drive(args, wl, rank: int, world: int, ops, render_fn, count_fn, hooks: Hooks, *,
          rehearse: bool = False, leg_workload=None) -> dict | None:
    """Everything main() does after the device is set up, on every rank: the timed job (run), the
    reports that need only the rank's own state, the configs[4] strong leg of the default line (all
    ranks take part: it gathers), then rank 0's output stage and CPU baseline.  Returns rank 0's JSON
    object, None on the other ranks -- whose only duty after run() is to take part in the leg's
    collectives (a report that assumed a result dict there crashed ranks 1..N-1 before the leg and
    left rank 0 waiting in its all-reduce: ADVICE round 5).  leg_workload: the strong leg's workload
    (default configs[4], c5_8k; tests pass a tiny one)."""
    from cpuperformanceraytracer_amd.shard import rows_of
    from cpuperformanceraytracer_amd._native import PtError
    try:
        res = run(args, wl, rank, world, ops, render_fn, count_fn, rehearse=rehearse, chain_counts=hooks.chain_counts)
        hooks.check_errors()   # no launch of the run abandoned a tile (PT_EKERNEL otherwise)
    except PtError as e:
        # A chained launch whose wait for its predecessor's tile ran out (guard PT_G_CHAIN_WAIT: the
        # predecessor's waves stopped running -- DESIGN.md 3e, "Residency"): the run's accumulator is
        # invalid and the error stands for it; the line is measured again with plain launches (one
        # rank: N ranks would leave the others in the run's collectives), and says so.
        if hooks.chain_counts is None or world > 1 or "guard 13 (chained launch" not in str(e):
            raise
        print(f"bench: chained run failed ({e}); measuring again with plain launches", file=sys.stderr)
        res = run(args, wl, rank, world, ops, render_fn, count_fn, rehearse=rehearse, chain_counts=None)
        hooks.check_errors()
        if res is not None:
            res["launch_chain"] = {"enabled": False, "chained_run_failed": str(e)[:400]}
    acc = None
    if res is not None:
        acc = res.pop("_accumulator")
        if hooks.launch_variant is not None:   # the continuous-tiles launch variant (pt_launch_variant)
            Wg, Hg = job_image(wl, world)
            rs, st, nr = rows_of(rank, world, Hg)
            try:   # (a report: it never costs the line)
                res["launch_variant"] = hooks.launch_variant(acc, Wg, Hg, rs, st, nr)
            except Exception as e:   # noqa: BLE001
                res["launch_variant"] = {"error": str(e)}
    # configs[4] beside the default workload's line (its scaling curve from the driver's N-GPU runs)
    configs4 = None
    if args.workload == "c2_1080p" and not args.no_configs4:
        from cpuperformanceraytracer_amd.config import CONFIGS
        configs4 = strong_leg(leg_workload or CONFIGS["c5_8k"], rank, world, ops, render_fn, count_fn, rehearse=rehearse)
        hooks.check_errors()
    if rank != 0:
        return None
    if hooks.output_stage is not None:
        res["output_stage"] = hooks.output_stage(acc, res)
    if configs4 is not None:
        res["configs4"] = configs4
    if world == 1 and not args.no_cpu_baseline and hooks.cpu_baseline is not None:
        res["cpu_baseline"] = hooks.cpu_baseline()
    return res


def spawn_ranks(n: int, argv: list[str], script: str | None = None) -> int:
    """`--gpus N` without a launcher: start N rank processes of `script` (default: this file) with
    the environment torch.distributed.run gives each rank (RANK, LOCAL_RANK, WORLD_SIZE,
    LOCAL_WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT), rank r on GPU r.  Called before anything
    touches the GPU; the parent only waits (it is not replaced).  Rank 0 inherits stdout and prints the
    JSON line.  Returns 0, or the first failing rank's exit code after killing the others."""
    import signal
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    script = script or str(Path(__file__).resolve())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script, *argv], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0] if bad[0] > 0 else 128 - bad[0]   # (a signal: 128 + its number)
                break
            if all(c == 0 for c in codes):
                break
            time.sleep(0.1)
    finally:
        for p in procs:   # a failed rank leaves the others waiting in a collective: end them
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    return rc


def main() -> None:
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # the driver's own invocation (`python bench.py --gpus N`, no torch.distributed.run): one
        # process per GPU, started here before any GPU call
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    import torch
    import torch.distributed as dist

    from cpuperformanceraytracer_amd.config import CONFIGS, synthetic_env
    from cpuperformanceraytracer_amd.shard import rows_of
    from cpuperformanceraytracer_amd.device import (JobLauncher, chain_counts, check_device_errors, count_device,
                                                    count_v4_device, ensure_backend, launch_variant, set_env_map)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"--gpus {args.gpus} disagrees with WORLD_SIZE {world}")
    # PT_BENCH_REHEARSE=1: rehearsal of the N-rank path on one GPU -- every rank on cuda:0, gloo
    # instead of RCCL, the gather through host memory (correctness of the multi-rank code only;
    # the numbers are not scaling numbers)
    rehearse = world > 1 and os.environ.get("PT_BENCH_REHEARSE") == "1"
    if world > 1:
        if rehearse:
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local if world > 1 and not rehearse else 0)
    torch.cuda.set_device(dev)
    wl = CONFIGS[args.workload]
    B = wl.num_bounces
    ensure_backend(dev.index, B)
    env = synthetic_env() if wl.env else None
    if env is not None:
        set_env_map(env, dev.index, B)
    v4 = wl.renderer == "v4"
    if v4:
        from cpuperformanceraytracer_amd.renderer import v4_config
        v4_config(num_bounces=B)   # the reference's default flags (equirect, random jitter, rejection)
    cfn = count_v4_device if v4 else count_device
    stream = torch.cuda.current_stream(dev)

    # the step's launch through a prepared job (device.JobLauncher: only frame_first changes from
    # step to step), so the host enqueues a step in a few microseconds
    launchers = {}

    def render_fn(buf, Wg, Hg, f, n, rs, st, nr, chain=False):
        key = (buf.data_ptr(), Wg, Hg, n, rs, st, nr, chain)
        launch = launchers.get(key)
        if launch is None:
            launch = launchers[key] = JobLauncher(buf, Wg, Hg, nframes=n, num_bounces=B, row_start=rs, row_stride=st,
                                                  nrows=nr, use_env=wl.env, stream=stream, v4=v4, chain=chain)
        launch(f)

    def count_fn(buf, Wg, Hg, f, n, rs, st, nr):
        return cfn(buf, Wg, Hg, frame_first=f, nframes=n, num_bounces=B, row_start=rs, row_stride=st, nrows=nr,
                   use_env=wl.env, stream=stream)

    ops = DeviceOps(dev, stream)

    def output_stage(buf, res):
        # the presented frame: rank 0's rendered accumulator (its first W x H pixels when sharded)
        W, H = wl.width, wl.height
        acc = buf if buf.numel() >= W * H * 3 else torch.zeros(W * H * 3, dtype=torch.float32, device=dev)
        if acc is not buf:
            acc[:buf.numel()].copy_(buf)
        out = measure_output_stage(acc, W, H, stream)
        if not v4:
            Wg, Hg = job_image(wl, world)
            rs, st, nr = rows_of(rank, world, Hg)
            out["fused"] = measure_fused_output(
                lambda b, px: JobLauncher(b, Wg, Hg, nframes=wl.spp, num_bounces=B, row_start=rs, row_stride=st,
                                          nrows=nr, use_env=wl.env, stream=stream, pixels=px),
                Wg, nr, wl.spp, stream, frame0=1)
        return out

    hooks = Hooks(check_errors=check_device_errors,
                  launch_variant=None if v4 else (
                      lambda buf, Wg, Hg, rs, st, nr: launch_variant(buf, Wg, Hg, nframes=wl.spp, num_bounces=B,
                                                                     row_start=rs, row_stride=st, nrows=nr,
                                                                     use_env=wl.env)),
                  output_stage=output_stage,
                  cpu_baseline=lambda: cpu_baseline(wl, args.cpu_seconds, env),
                  # the steps are chained launches (pt_render_device_chain / pt_v4_render_device_chain) unless
                  # --no-chain
                  chain_counts=None if args.no_chain else chain_counts)
    res = drive(args, wl, rank, world, ops, render_fn, count_fn, hooks, rehearse=rehearse)
    if rank == 0:
        print(json.dumps(res))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
