"""Multi-GPU sharding of one image: row-interleaved partition + gather of sub-images.

Pixels are independent and every sample's RNG seed depends only on the GLOBAL pixel (x, y) and
the frame (demofox_path_tracing_scalar.cpp:332), so any partition of the rows renders bit-identical
pixels.  Rows are dealt round-robin (row Y -> rank Y % world): neighbouring rows cost about the
same (open front vs. box interior varies slowly with Y), so every rank gets the same mix of cheap
and expensive rows -- contiguous bands would not.

Each rank renders its rows into a compact sub-image in its own HBM (pt_render_device with
row_start = rank, row_stride = world).  The only exchange in the whole path is the final gather of
those disjoint sub-images to the root (torch.distributed -> RCCL over xGMI on MI355X; gloo on CPU
in the tests): no reduction, so no all-reduce.
"""
from __future__ import annotations


def rows_of(rank: int, world: int, height: int) -> tuple[int, int, int]:
    """(row_start, row_stride, nrows) of `rank`'s shard of a `height`-row image."""
    if not (0 <= rank < world):
        raise ValueError(f"rank {rank} outside world {world}")
    return rank, world, len(range(rank, height, world))


def max_rows(world: int, height: int) -> int:
    return (height + world - 1) // world


def gather_rows(sub, width: int, height: int, rank: int, world: int, dst: int = 0, group=None,
                force_collective: bool = False):
    """Gather every rank's compact sub-image (nrows x width x 3, rows rank::world) to `dst` and
    un-interleave into the full height x width x 3 image there (None on other ranks).

    `sub` must hold max_rows(world, height) rows (the tail row of shorter shards is padding) so
    that every rank sends the same byte count.  One rank returns its sub-image without a collective,
    unless force_collective (tests: the RCCL call an N-GPU run makes, executed on one GPU)."""
    import torch
    import torch.distributed as dist

    mr = max_rows(world, height)
    sub = sub.reshape(-1)
    if sub.numel() != mr * width * 3:
        raise ValueError(f"sub-image must hold {mr} rows of {width}x3 floats, got {sub.numel()}")
    if world == 1 and not force_collective:
        return sub.view(height, width, 3)
    # the root receives every rank's sub-image into one (world, mr, W*3) tensor; rank r's row k is the
    # global row k * world + r, so the un-interleave is ONE transposing copy (world, mr) -> (mr, world)
    stacked = torch.empty((world, mr, width * 3), dtype=sub.dtype, device=sub.device) if rank == dst else None
    chunks = list(stacked.view(world, mr * width * 3).unbind(0)) if rank == dst else None
    dist.gather(sub, gather_list=chunks, dst=dst, group=group)
    if rank != dst:
        return None
    full = stacked.transpose(0, 1).reshape(mr * world, width * 3)[:height]
    return full.reshape(height, width, 3)
