#!/usr/bin/env python3
"""Benchmark of the MI355X path-tracing hot path (BASELINE.json metric and configs).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
         --master-port P bench.py --gpus N --steps K --warmup W

Workload (configs[1]): 1920x1080, 8 spp, 8 bounces, the demofox quad+sphere scene,
diffuse+emissive.  One STEP = one launch that accumulates 8 more frames (8 spp) into the
HBM-resident f32 accumulator of every pixel -- bit-identical to 8 calls of the reference's
DemofoxRenderScalar.  Frames advance step to step like the reference's progressive render.

N > 1 (weak scaling): the image grows to ~N x 1920x1080 pixels at the same aspect ratio (so the
same view: sqrt(N) x 1920 by sqrt(N) x 1080, e.g. 3840x2160 for N = 4) and every rank renders
its interleaved 1/N of the rows, ~1920x1080 pixels (shard.py); after the K steps the sub-images
are gathered to rank 0 over RCCL (the job's only exchange, inside the timed region, also reported
separately).

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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 100 steps of 0.3 ms: the launch latency before the first step and the final synchronisation
    # (~2 us per step at 20 steps) stay out of the per-step time
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c2_1080p")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--device-warmup-ms", type=float, default=60.0,
                    help="untimed GPU work before the warmup steps (clock ramp; 0 = none)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="wall time of the CPU baseline sample (whole frames of the workload)")
    return ap.parse_args()


def cpu_baseline(wl, seconds: float, env=None) -> dict:
    """The oracle (C restatement of demofox_path_tracing_scalar.cpp, bit-identical to it) timed on
    this host's cores on a bounded sample of the same workload -- full-size frames, as many as fit
    in about `seconds` of wall time; beside it the reference's CPU SIMD path (an AVX2 port of
    simt_pooled, `simd_port`; the value reported is the faster of the two CPU paths, which is the
    scalar restatement: the SIMD file traces every bounce of every lane under masks) and the
    reference's own scalar build (oracle/_ref, c_numBounces=4 compiled in) single-threaded."""
    from oracle import pyoracle
    try:
        ncpu = len(os.sched_getaffinity(0))
    except AttributeError:
        ncpu = os.cpu_count() or 1
    cores = max(1, min(16, ncpu))
    if wl.renderer == "v4":
        return cpu_baseline_v4(wl, seconds, env, cores, ncpu)
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
           "primary_samples_per_s": samples / dt, "host_cpus_visible": ncpu,
           "cpu_model": _cpu_model()}
    if env is None:
        out["simd_port"] = cpu_simd_port(wl, seconds / 2, cores)
    ref = ROOT / "oracle" / "_ref" / "libref_scalar.so"
    if ref.exists() and env is None:
        import ctypes
        import numpy as np
        L = ctypes.CDLL(str(ref))
        L.ref_render_scalar.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        w, h = 640, 360
        buf = np.zeros((h, w, 3), np.float32)
        t0 = time.perf_counter()
        L.ref_render_scalar(buf.ctypes.data, w, h, 1)
        t1 = time.perf_counter() - t0
        rf = int(max(1, min(256, round(seconds / 4 / max(t1, 1e-6)))))
        t0 = time.perf_counter()
        L.ref_render_scalar(buf.ctypes.data, w, h, rf)
        dt = time.perf_counter() - t0
        out["reference_scalar"] = {"primary_samples_per_s": w * h * rf / dt, "ray_samples_per_s": w * h * rf * 4 / dt,
                                   "cores": 1, "sample": f"{w}x{h}, {rf} frames, 4 bounces (compiled-in "
                                   f"c_numBounces), DemofoxRenderScalar built unmodified by oracle/build_ref.sh; "
                                   f"{dt:.2f} s wall"}
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


def cpu_baseline_v4(wl, seconds: float, env, cores: int, ncpu: int) -> dict:
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
            "primary_samples_per_s": samples / dt, "host_cpus_visible": ncpu, "cpu_model": _cpu_model()}


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def load_traffic(workload: str):
    """Per-launch HBM bytes of the render kernel from the committed rocprofv3 PMC summary of this
    workload (profiles/pmc_summary.json for the headline c2, pmc_summary_<workload>.json else)."""
    p = ROOT / "profiles" / ("pmc_summary.json" if workload == "c2_1080p" else f"pmc_summary_{workload}.json")
    if not p.exists():
        return None, None
    d = json.loads(p.read_text())
    return d.get("hbm_bytes_per_launch"), d.get("source")


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


def main() -> None:
    args = parse()
    import torch
    import torch.distributed as dist

    from cpuperformanceraytracer_amd import roofline as RL
    from cpuperformanceraytracer_amd.config import CONFIGS, synthetic_env
    from cpuperformanceraytracer_amd.device import (count_device, count_v4_device, ensure_backend, render_device,
                                                    render_v4_device, set_env_map)
    from cpuperformanceraytracer_amd.shard import gather_rows, max_rows, rows_of

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            sys.exit("run N>1 under torch.distributed.run (one process per GPU)")
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
    W, H, S, B = wl.width, wl.height, wl.spp, wl.num_bounces
    Wg, Hg = weak_image(W, H, world)                 # weak scaling: ~W*H pixels per rank, same view
    row_start, row_stride, nrows = rows_of(rank, world, Hg)
    mr = max_rows(world, Hg)
    ensure_backend(dev.index, B)
    env = synthetic_env() if wl.env else None
    if env is not None:
        set_env_map(env, dev.index, B)
    v4 = wl.renderer == "v4"
    if v4:
        from cpuperformanceraytracer_amd.renderer import v4_config
        v4_config(num_bounces=B)   # the reference's default flags (equirect, random jitter, rejection)
    render_fn, count_fn = (render_v4_device, count_v4_device) if v4 else (render_device, count_device)

    buf = torch.zeros(mr * Wg * 3, dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev)
    frame = 1

    def step(f):
        render_fn(buf, Wg, Hg, frame_first=f, nframes=S, num_bounces=B, row_start=row_start,
                  row_stride=row_stride, nrows=nrows, use_env=wl.env, stream=stream)

    # Device warm-up, untimed, before the W warmup steps: the MI355X reaches its steady clocks only
    # after ~25 ms of sustained load (per-launch time at 1080p, 8 spp: 0.46 ms over the first 20
    # launches, 0.379 over the next 20, 0.357 from the 60th on -- scripts/clock_ramp.py), and the
    # reference's progressive renderer runs continuously.  Reported as "device_warmup".
    dw_ms, dw_steps = 0.0, 0
    while dw_ms < args.device_warmup_ms and dw_steps < 4000:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(10):
            step(frame)
            frame += S
        e1.record(stream)
        e1.synchronize()
        dw_ms += e0.elapsed_time(e1)
        dw_steps += 10
    for _ in range(args.warmup):
        step(frame)
        frame += S
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    K = args.steps
    # Two HIP events bracket the K launches on their stream: the average launch duration is their
    # interval / K (back to back, so it includes the inter-launch gaps: an upper bound of the kernel
    # time; it agrees with rocprofv3's kernel-trace average).  An event pair around EVERY launch
    # would add ~9 us per step to the timed region (scripts/event_overhead.py), so per-launch pairs
    # are recorded only in an untimed pass after it (kernel_ms_event_pairs).
    ev_a, ev_b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    timed_first = frame
    t0 = time.perf_counter()
    ev_a.record(stream)
    for k in range(K):
        step(frame)
        frame += S
    ev_b.record(stream)
    gather_ms = 0.0
    if world > 1:
        g0 = torch.cuda.Event(enable_timing=True)
        g1 = torch.cuda.Event(enable_timing=True)
        g0.record(stream)
        full = gather_rows(buf.cpu() if rehearse else buf, Wg, Hg, rank, world)
        g1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    launch_ms_avg = ev_a.elapsed_time(ev_b) / K
    if world > 1:
        gather_ms = g0.elapsed_time(g1)
        t = torch.tensor([elapsed, gather_ms], dtype=torch.float64, device="cpu" if rehearse else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, gather_ms = float(t[0]), float(t[1])
        if rank == 0:
            assert full is not None and full.shape == (Hg, Wg, 3)

    # Untimed: per-launch event pairs (the event overhead lands inside each pair).
    pairs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(min(K, 20))]
    for a, b in pairs:
        a.record(stream)
        step(frame)
        b.record(stream)
        frame += S
    torch.cuda.synchronize(dev)
    pair_ms = [a.elapsed_time(b) for a, b in pairs]

    # Exact work of the timed launches (deterministic: same frames, counted on a scratch buffer).
    scratch = torch.zeros_like(buf)
    segs = samples = slots = prim = escaped = sky = 0
    for k in range(K):
        c = count_fn(scratch, Wg, Hg, frame_first=timed_first + k * S, nframes=S, num_bounces=B,
                     row_start=row_start, row_stride=row_stride, nrows=nrows, use_env=wl.env, stream=stream)
        escaped += c["escaped"]
        segs += c["segments"]
        samples += c["samples"]
        slots += c["lane_slots"]
        prim += c.get("primary", c["samples"])
        sky += c.get("sky_skipped", 0)
    del scratch

    output_stage = None
    if rank == 0:   # the presented 1080p frame of configs[1]: a W x H accumulator
        acc = buf if world == 1 else torch.zeros(W * H * 3, dtype=torch.float32, device=dev)
        if world > 1:
            n = min(acc.numel(), buf.numel())
            acc[:n].copy_(buf[:n])
        output_stage = measure_output_stage(acc, W, H, stream)

    if rank != 0:
        dist.destroy_process_group()
        return

    ms_step = elapsed * 1e3 / K
    total_ray_samples = Wg * Hg * S * B * K
    value = total_ray_samples / elapsed
    avg_kernel_s = launch_ms_avg / 1e3
    if v4:   # every frame traces its own jittered camera ray; all-sky iterations skip the trace
        flops_launch = RL.v4_launch_flops(segs, samples, sky) / K
        flops_launch_ref = RL.v4_launch_flops(segs, samples) / K
        flop_model = (f"segments x V4_F_SEGMENT - sky_skipped x V4_F_SKY_TRACE + samples x V4_F_SAMPLE; F = "
                      f"{RL.V4_F_SEGMENT}/{RL.V4_F_SKY_TRACE}/{RL.V4_F_SAMPLE} (roofline.py, counted by oracle/pt_oracle_v4.c)")
        kernel_name = "pt_v4_kernel<EQUIRECT, INTERLEAVED>"
    else:
        flops_launch = RL.launch_flops_exec(segs, prim, samples, sky) / K
        flops_launch_ref = RL.launch_flops_ref(segs, prim, samples) / K
        flop_model = ("executed = (segments_ref x F_SEGMENT + samples x F_SAMPLE) - (samples - pixels) x "
                      f"F_SHARED - sky_skipped x F_SKY_TRACE; F = {RL.F_SEGMENT}/{RL.F_SAMPLE}/{RL.F_SHARED}/"
                      f"{RL.F_SKY_TRACE} (roofline.py)")
        kernel_name = "pt_render_env_kernel<INTERLEAVED>" if wl.env else "pt_render_kernel<INTERLEAVED>"
    achieved_tf = flops_launch / avg_kernel_s / 1e12
    hbm_launch, traffic_src = load_traffic(wl.name)
    # config 4: one 12-byte texel gather per escaping path
    env_bytes = RL.BYTES_PER_ENV_GATHER * escaped / K if wl.env else 0
    res = {
        "metric": METRIC,
        "value": value,
        "unit": "ray-samples/s",
        "n_gpus": world,
        "steps": K,
        "warmup": args.warmup,
        "device_warmup": {"steps": dw_steps, "ms": round(dw_ms, 3)},
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": ("synthetic (the reference's v4 InitializeScene: 4 quads + 7 glass spheres; no dataset)" if v4 else
                 "synthetic (the reference's fixed demofox quad+sphere scene; no dataset)") + (
            "; env map: 2048x1024 log-normal f32, seed 0xC0FFEE, standing in for the missing chinese_garden_2k.hdr"
            if wl.env else ""),
        "config": {"workload": wl.name, "width": W, "height": H, "spp": S, "bounces": B,
                   "image": [Wg, Hg], "parallelism": f"rows interleaved x{world}" if world > 1 else "single GPU",
                   "step": f"one launch accumulating {S} frames (spp) of every pixel in HBM"},
        "primary_samples_per_s": Wg * Hg * S * K / elapsed,
        "ms_per_frame_1spp": ms_step / S,
        "traced_segments_per_s": segs * world / (avg_kernel_s * K),
        "segments_per_sample": segs / samples,
        "ref_segments_per_sample": (segs if v4 else RL.ref_segments(segs, prim, samples)) / samples,
        "simd_lane_efficiency": segs / slots if slots else None,
        "sky_skipped_traces_per_launch": sky / K,
        "kernel_ms_avg": avg_kernel_s * 1e3,
        "kernel_ms_source": "HIP events bracketing the K timed launches on their stream, interval / K",
        "kernel_ms_event_pairs": {"launches": len(pair_ms), "avg": sum(pair_ms) / len(pair_ms), "min": min(pair_ms),
                                  "note": "untimed pass, an event pair around each launch"},
        "roofline": {
            "bound": "valu",
            "achieved": achieved_tf,
            "peak": RL.PEAK_FP32_TFLOPS,
            "unit": "TFLOP/s",
            "frac": achieved_tf / RL.PEAK_FP32_TFLOPS,
            "traffic": hbm_launch,
            "kernel": kernel_name,
            "flops_per_launch": flops_launch,
            "flop_model": flop_model,
            "flops_per_launch_ref_equivalent": flops_launch_ref,
            "achieved_ref_equivalent": flops_launch_ref / avg_kernel_s / 1e12,
            "algorithmic_bytes_per_launch": RL.BYTES_PER_PIXEL_PER_LAUNCH * Wg * nrows + env_bytes,
            "hbm_achieved_gbps": (RL.BYTES_PER_PIXEL_PER_LAUNCH * Wg * nrows + env_bytes) / avg_kernel_s / 1e9,
            "hbm_peak_gbps": RL.PEAK_HBM_GBPS,
            "traffic_source": traffic_src,
        },
    }
    if world > 1:
        res["gather_ms"] = gather_ms
    res["output_stage"] = output_stage
    if world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(wl, args.cpu_seconds, env)
    print(json.dumps(res))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
