"""bench.py's N-rank code path on CPU (gloo, world size 2): bench.run with the host clock and the
oracle standing in for the GPU render, for both scaling modes -- the strong-scaling configs[4]
shape (a FIXED image, rows r::N per rank, a gather to rank 0 every step) at a tiny size, and the
weak-scaling default.  Rank 0's gathered image must equal the single-process oracle image bit for
bit, and the bench's own --verify-rows check must pass."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _SkewedOps:
    """bench.HostOps whose clock runs at a rank-dependent rate (rank 0: 5 ms per interval, rank 1:
    25 ms): left to decide alone, the ranks would run different numbers of device warm-up batches."""

    def __init__(self, rank):
        import bench
        self._h = bench.HostOps()
        self.dev = "cpu"
        self._ms = 5.0 if rank == 0 else 25.0

    def __getattr__(self, name):
        return getattr(self._h, name)

    def elapsed_ms(self, a, b):
        return self._ms


def _worker(rank, world, port, scaling, q, skew=False):
    import sys
    from pathlib import Path
    root = str(Path(__file__).resolve().parents[1])
    sys.path.insert(0, root)
    import torch.distributed as dist
    import bench
    from cpuperformanceraytracer_amd.config import Workload
    from oracle import pyoracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        wl = Workload("tiny", 64, 36, 3, 8, scaling=scaling)   # configs[4]'s shape, scaled down
        args = bench.parse(["--gpus", str(world), "--steps", "2", "--warmup", "1", "--device-warmup-ms",
                            "20" if skew else "0", "--verify-rows", "2"])

        def render_fn(buf, W, H, f, n, rs, st, nr):
            pyoracle.render(W, H, frame_first=f, nframes=n, num_bounces=wl.num_bounces, row_start=rs,
                            row_stride=st, nrows=nr, nthreads=2, buf=buf.numpy())

        def count_fn(buf, W, H, f, n, rs, st, nr):
            render_fn(buf, W, H, f, n, rs, st, nr)
            _, c = pyoracle.render_counted(W, H, frame_first=f, nframes=n, num_bounces=wl.num_bounces,
                                           row_start=rs, row_stride=st, nrows=nr)
            return {"segments": c["segments"], "samples": c["samples"], "escaped": c["escaped"],
                    "lane_slots": c["segments"], "primary": c["samples"]}

        ops = _SkewedOps(rank) if skew else bench.HostOps()
        res = bench.run(args, wl, rank, world, ops, render_fn, count_fn, roofline=False)
        if rank == 0:
            acc = res.pop("_accumulator")
            q.put((res, acc.numpy().copy()))
        else:
            assert res is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("scaling", ["strong", "weak"])
def test_bench_n_rank_path_gloo(scaling):
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import bench
    from cpuperformanceraytracer_amd.config import Workload
    from oracle import pyoracle
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, scaling, q)) for r in range(world)]
    for p in procs:
        p.start()
    res, acc0 = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    wl = Workload("tiny", 64, 36, 3, 8, scaling=scaling)
    Wg, Hg = bench.job_image(wl, world)
    if scaling == "strong":
        assert (Wg, Hg) == (64, 36)                       # the image does not grow with N
    else:
        assert Wg * Hg > 1.9 * 64 * 36
    assert res["scaling"] == scaling and res["n_gpus"] == world
    assert res["config"]["image"] == [Wg, Hg]
    assert res["verified"]["bit_exact"] and len(res["verified"]["rows"]) >= 2
    assert "gather_ms" in res and res["value"] > 0
    assert res["segments_per_sample"] > 0
    # warm-up (1 step) + 2 timed steps + the untimed per-launch pass (2 steps): rank 0's own rows
    # 0::2 hold frames [1, 1 + 5 * spp) -- the same as the single-process oracle render
    frames = 5 * wl.spp
    ref = pyoracle.render(Wg, Hg, frame_first=1, nframes=frames, num_bounces=wl.num_bounces, row_start=0,
                          row_stride=world, nrows=(Hg + 1) // 2, nthreads=2)
    got = acc0[:ref.size].reshape(ref.shape)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    # the verified frame range ends where the timed steps end (1 warm-up + 2 timed steps)
    assert res["verified"]["frames"] == [1, 3 * wl.spp]


def test_bench_ranks_agree_on_the_device_warmup():
    """The device warm-up runs batches until a time budget is spent; the ranks' clocks differ, so the
    number of batches is agreed by all ranks (the largest any rank needs).  Rank 0 alone would stop
    after 4 batches of 10 steps (20 ms at 5 ms each), rank 1 after 1 (25 ms): both run 4, every rank
    accumulates the same frames, and the gathered image passes the bench's own row check.  (Decided
    per rank, this was the row mismatch of the round-4 two-process rehearsals)"""
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    from oracle import pyoracle
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, "weak", q, True)) for r in range(world)]
    for p in procs:
        p.start()
    res, acc0 = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res["device_warmup"]["steps"] == 40
    assert res["verified"]["bit_exact"]
    Wg, Hg = res["config"]["image"]
    frames = (40 + 1 + 2 + 2) * 3      # device warm-up + warm-up + timed + untimed steps of 3 frames
    ref = pyoracle.render(Wg, Hg, frame_first=1, nframes=frames, num_bounces=8, row_start=0, row_stride=world,
                          nrows=(Hg + 1) // 2, nthreads=2)
    got = acc0[:ref.size].reshape(ref.shape)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def _worker_leg(rank, world, port, q):
    """bench.strong_leg (the configs[4] leg of the default line) on a tiny fixed image."""
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import torch.distributed as dist
    import bench
    from cpuperformanceraytracer_amd.config import Workload
    from oracle import pyoracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        wl4 = Workload("tiny_c5", 48, 28, 4, 8, scaling="strong")

        def render_fn(buf, W, H, f, n, rs, st, nr):
            pyoracle.render(W, H, frame_first=f, nframes=n, num_bounces=8, row_start=rs, row_stride=st, nrows=nr,
                            nthreads=2, buf=buf.numpy())

        def count_fn(buf, W, H, f, n, rs, st, nr):
            render_fn(buf, W, H, f, n, rs, st, nr)
            _, c = pyoracle.render_counted(W, H, frame_first=f, nframes=n, num_bounces=8, row_start=rs,
                                           row_stride=st, nrows=nr)
            return {"segments": c["segments"], "samples": c["samples"], "escaped": c["escaped"],
                    "lane_slots": c["segments"], "primary": c["samples"]}

        out = bench.strong_leg(wl4, rank, world, bench.HostOps(), render_fn, count_fn, steps=2)
        if rank == 0:
            q.put(out)
        else:
            assert out is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2])
def test_configs4_leg_of_the_default_line(world):
    """The default line's `configs4` object (bench.strong_leg): the fixed image does not grow with N,
    every step's render and gather are reported apart, and with N > 1 the gathered image passes the
    bench's row check; N = 1 reports the whole-image render alone."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_leg, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out["scaling"] == "strong" and out["n_gpus"] == world
    assert out["config"]["image"] == [48, 28] and out["steps"] == 2
    assert out["value"] > 0 and out["render_ms_per_step"] > 0 and "gather_ms" in out
    if world > 1:
        assert out["verified"]["bit_exact"]
    else:
        assert out["gather_ms"] == 0.0


# ---- `python bench.py --gpus N` without a launcher: bench.spawn_ranks starts the N ranks itself ----
def test_spawn_ranks_runs_the_n_rank_path(capfd):
    """The driver's plain invocation with N > 1 (no torch.distributed.run): spawn_ranks gives each
    rank the launcher's environment, the ranks rendezvous (gloo here, RCCL on the GPUs), and rank 0's
    JSON line is the output -- the weak-scaling image gathered and verified bit for bit."""
    import hashlib
    import json
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import bench
    from cpuperformanceraytracer_amd.config import Workload
    from oracle import pyoracle
    worker = str(Path(__file__).resolve().parent / "bench_rank_worker.py")
    rc = bench.spawn_ranks(2, ["64", "36", "3", "8", "weak"], script=worker)
    out = [ln for ln in capfd.readouterr().out.splitlines() if ln.startswith("{")]   # (gloo logs a line too)
    assert rc == 0
    assert len(out) == 1, out                      # one JSON line, from rank 0 only
    res = json.loads(out[0])
    assert res["n_gpus"] == 2 and res["scaling"] == "weak" and res["verified"]["bit_exact"]
    wl = Workload("tiny", 64, 36, 3, 8, scaling="weak")
    Wg, Hg = bench.job_image(wl, 2)
    ref = pyoracle.render(Wg, Hg, frame_first=1, nframes=5 * wl.spp, num_bounces=8, row_start=0, row_stride=2,
                          nrows=(Hg + 1) // 2, nthreads=2)
    assert res["acc_sha256"] == hashlib.sha256(_pad(ref, Hg, Wg)).hexdigest()


def _pad(ref, Hg, Wg):
    """rank 0's accumulator: max_rows(2, Hg) rows of which its (Hg + 1) // 2 rows are rendered."""
    from cpuperformanceraytracer_amd.shard import max_rows
    buf = np.zeros((max_rows(2, Hg), Wg, 3), np.float32)
    buf[:ref.shape[0]] = ref
    return buf.tobytes()


def test_spawn_ranks_reports_a_failed_rank():
    """A rank that dies makes spawn_ranks end the others (waiting in the rendezvous) and return its
    exit code instead of hanging."""
    import sys
    import time
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import bench
    worker = str(Path(__file__).resolve().parent / "bench_rank_worker.py")
    t0 = time.time()
    rc = bench.spawn_ranks(2, ["64", "36", "3", "8", "weak", "1"], script=worker)
    assert rc == 3 and time.time() - t0 < 120


def test_main_dispatches_to_spawn_ranks(monkeypatch):
    """bench.main with --gpus N > 1 and no WORLD_SIZE goes to spawn_ranks before touching a GPU."""
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import bench
    seen = {}
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench, "spawn_ranks", lambda n, argv, script=None: seen.update(n=n, argv=argv) or 7)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3"])
    with pytest.raises(SystemExit) as ei:
        bench.main()
    assert ei.value.code == 7 and seen == {"n": 4, "argv": ["--gpus", "4", "--steps", "3"]}


def _worker_drive(rank, world, port, q):
    """bench.drive -- main()'s whole post-setup flow (run, launch-variant report, the configs[4]
    strong leg, rank 0's output stage and CPU baseline) -- on CPU with host hooks."""
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import torch.distributed as dist
    import bench
    from cpuperformanceraytracer_amd.config import Workload
    from oracle import pyoracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        wl = Workload("tiny", 64, 36, 3, 8, scaling="weak")
        wl4 = Workload("tiny_c5", 48, 28, 4, 8, scaling="strong")
        args = bench.parse(["--gpus", str(world), "--steps", "2", "--warmup", "1", "--device-warmup-ms", "0"])

        def render_fn(buf, W, H, f, n, rs, st, nr):
            pyoracle.render(W, H, frame_first=f, nframes=n, num_bounces=8, row_start=rs, row_stride=st, nrows=nr,
                            nthreads=2, buf=buf.numpy())

        def count_fn(buf, W, H, f, n, rs, st, nr):
            render_fn(buf, W, H, f, n, rs, st, nr)
            _, c = pyoracle.render_counted(W, H, frame_first=f, nframes=n, num_bounces=8, row_start=rs,
                                           row_stride=st, nrows=nr)
            return {"segments": c["segments"], "samples": c["samples"], "escaped": c["escaped"],
                    "lane_slots": c["segments"], "primary": c["samples"]}

        calls = []
        hooks = bench.Hooks(
            check_errors=lambda: calls.append("check"),
            launch_variant=lambda buf, W, H, rs, st, nr: {"rows": [rs, st, nr], "n": int(buf.numel())},
            output_stage=lambda buf, res: {"pixels": int(buf.numel()) // 3},
            cpu_baseline=lambda: {"value": 1.0})
        out = bench.drive(args, wl, rank, world, bench.HostOps(), render_fn, count_fn, hooks, leg_workload=wl4)
        q.put((rank, out, calls))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2])
def test_drive_completes_on_every_rank(world):
    """main()'s post-run flow on N ranks: ranks 1..N-1 (whose run() result is None) pass the reports
    and take part in the configs[4] leg's gathers; rank 0's object carries launch_variant, the leg,
    the output stage, and (N = 1 only) the CPU baseline.  Round 5's main() crashed every rank but 0
    here, so rank 0 waited in the leg's all-reduce and no N-GPU line was ever printed."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_drive, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, (o, c)) for r, o, c in (q.get(timeout=240) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(1, world):
        assert got[r][0] is None and got[r][1] == ["check", "check"]
    res, calls = got[0]
    assert calls == ["check", "check"]
    assert "_accumulator" not in res
    assert res["launch_variant"]["rows"][1] == world
    assert res["configs4"]["scaling"] == "strong" and res["configs4"]["n_gpus"] == world
    assert res["configs4"]["metric"].endswith("at 48×28; ms/frame")
    assert res["metric"].endswith("at 64×36; ms/frame")
    assert res["output_stage"]["pixels"] > 0
    assert ("cpu_baseline" in res) == (world == 1)
    if world > 1:
        assert res["configs4"]["verified"]["bit_exact"]


def _worker_chain_fallback(port, q):
    """bench.drive with chained steps whose run ends in a chained-launch wait error (guard 13): the line
    is measured again with plain steps and says so."""
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import torch.distributed as dist
    import bench
    from cpuperformanceraytracer_amd._native import PtError
    from cpuperformanceraytracer_amd.config import Workload
    from oracle import pyoracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        wl = Workload("tiny", 64, 36, 3, 8, scaling="weak")
        args = bench.parse(["--steps", "2", "--warmup", "1", "--device-warmup-ms", "0", "--no-configs4",
                            "--no-cpu-baseline"])
        modes, failed = [], []

        def render_fn(buf, W, H, f, n, rs, st, nr, chain=False):
            modes.append(chain)
            pyoracle.render(W, H, frame_first=f, nframes=n, num_bounces=8, row_start=rs, row_stride=st, nrows=nr,
                            nthreads=2, buf=buf.numpy())

        def count_fn(buf, W, H, f, n, rs, st, nr):
            render_fn(buf, W, H, f, n, rs, st, nr)
            _, c = pyoracle.render_counted(W, H, frame_first=f, nframes=n, num_bounces=8, row_start=rs,
                                           row_stride=st, nrows=nr)
            return {"segments": c["segments"], "samples": c["samples"], "escaped": c["escaped"],
                    "lane_slots": c["segments"], "primary": c["samples"]}

        def check_errors():
            if True in modes and not failed:
                failed.append(1)
                raise PtError(-5, "pt_check", "device 0: 9 kernel bounds guard failure(s), the first: guard 13 "
                                              "(chained launch: the previous launch's tile never became ready)")

        hooks = bench.Hooks(check_errors=check_errors, chain_counts=lambda: {"restarts": 0, "continued": 0})
        out = bench.drive(args, wl, 0, 1, bench.HostOps(), render_fn, count_fn, hooks)
        q.put((out["launch_chain"], sorted(set(modes))))
    finally:
        dist.destroy_process_group()


def test_drive_measures_plain_steps_after_a_chain_wait_error():
    """A chained run that ends in guard PT_G_CHAIN_WAIT (residency) is measured again with
    plain launches: the line reports launch_chain.enabled false and the error."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker_chain_fallback, args=(_free_port(), q))
    p.start()
    chain, modes = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert chain["enabled"] is False and "guard 13" in chain["chained_run_failed"], chain
    assert modes == [False, True]
