"""The RCCL calls of the N-GPU bench path, executed on the one GPU of the test box.

bench.py's N-rank runs gather the ranks' sub-images to rank 0 (shard.gather_rows: dist.gather) and
reduce their clocks and work counts (bench.reduce_values: dist.all_reduce, MAX and SUM) on cuda
tensors over RCCL ("nccl").  A one-rank run skips both, and every multi-rank rehearsal used gloo
through host memory -- so before this test those RCCL calls had never run.  Here a one-rank nccl
process group on cuda:0 makes exactly those calls (force_collective) on a rendered sub-image: the
gathered image equals the rendered one and the oracle bit for bit, the reductions return their
inputs.  Reference: the tile fan-out this replaces, demofox_path_tracing_simd_tiled.cpp:549-571."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest

from conftest import bits_equal, mismatch_report
from oracle import pyoracle

pytestmark = pytest.mark.gpu


@pytest.fixture
def nccl_group(monkeypatch):
    import torch
    import torch.distributed as dist
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl"
    yield
    dist.destroy_process_group()


def test_rccl_gather_and_reductions_on_device(nccl_group):
    import sys
    from pathlib import Path
    import torch
    import torch.distributed as dist
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import bench
    from cpuperformanceraytracer_amd.device import render_device
    from cpuperformanceraytracer_amd.shard import gather_rows, max_rows
    W, H, B, S = 320, 180, 8, 3
    buf = torch.zeros(max_rows(1, H) * W * 3, dtype=torch.float32, device="cuda:0")
    render_device(buf, W, H, frame_first=1, nframes=S, num_bounces=B)
    full = gather_rows(buf, W, H, 0, 1, force_collective=True)
    torch.cuda.synchronize()
    assert full.device.type == "cuda" and tuple(full.shape) == (H, W, 3)
    ref = pyoracle.render(W, H, nframes=S, num_bounces=B)
    got = full.cpu().numpy()
    assert bits_equal(got, ref), mismatch_report(got, ref)
    # the reductions bench.run makes (device tensors under nccl): clocks (MAX), work counts (SUM)
    mx = bench.reduce_values([1.5, 0.25, 3.0], dist.ReduceOp.MAX, world=1, dev=torch.device("cuda", 0),
                             force_collective=True)
    sm = bench.reduce_values([123456789, 42, 7], dist.ReduceOp.SUM, world=1, dev=torch.device("cuda", 0),
                             force_collective=True)
    assert mx == [1.5, 0.25, 3.0] and sm == [123456789.0, 42.0, 7.0]
    dist.barrier()
