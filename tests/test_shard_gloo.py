"""Multi-process sharding on CPU (gloo, world_size 2 and 3): each rank renders its row-interleaved
shard (here with the oracle -- the CPU test stands in for the GPU render) and shard.gather_rows
reassembles the image on rank 0.  The result must equal the single-process image bit for bit."""
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


def _worker(rank, world, port, w, h, frames, bounces, q):
    import sys
    from pathlib import Path
    root = str(Path(__file__).resolve().parents[1])
    sys.path.insert(0, root)
    sys.path.insert(0, str(Path(root) / "tests"))
    import torch
    import torch.distributed as dist
    from cpuperformanceraytracer_amd.shard import gather_rows, max_rows, rows_of
    from oracle import pyoracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        r0, stride, n = rows_of(rank, world, h)
        mr = max_rows(world, h)
        sub = np.zeros((mr, w, 3), np.float32)
        if n:
            pyoracle.render(w, h, nframes=frames, num_bounces=bounces, row_start=r0, row_stride=stride, nrows=n,
                            nthreads=2, buf=sub)
        full = gather_rows(torch.from_numpy(sub), w, h, rank, world)
        if rank == 0:
            q.put(full.numpy().copy())
        else:
            assert full is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,h", [(2, 37), (3, 40)])
def test_gloo_row_shards_gather_to_full_image(world, h):
    from oracle import pyoracle
    w, frames, bounces = 48, 2, 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, w, h, frames, bounces, q)) for r in range(world)]
    for p in procs:
        p.start()
    img = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ref = pyoracle.render(w, h, nframes=frames, num_bounces=bounces)
    assert np.array_equal(img.view(np.uint32), ref.view(np.uint32))


def test_rows_of_partition():
    from cpuperformanceraytracer_amd.shard import max_rows, rows_of
    h, world = 1081, 8
    seen = []
    for r in range(world):
        s, st, n = rows_of(r, world, h)
        rows = list(range(s, s + n * st, st))
        assert all(y < h for y in rows) and n <= max_rows(world, h)
        seen += rows
    assert sorted(seen) == list(range(h))
    with pytest.raises(ValueError):
        rows_of(8, 8, 10)
