"""Host model of the continuous ring pool of the diffuse kernel's MULTI launches (pt_kernel.hip,
`RING`): the same hand-out arithmetic (frame-major items, umulhi(i, ceil(2^32 / nh)) for i / nh and
nh = 1 apart, the R-slot ring per pixel with free / reserved / ready marks, in-order hand-out that
stops at the first blocked item, one fold per lane and iteration) on random path lengths.  Every
pool drains (no hang), well inside the kernel's iteration guard, and every pixel folds frames
0..S-1 in order from the slot that holds that very frame."""
from __future__ import annotations

import random

import pytest

R = 7   # CHS of the ambient kernel


def run_pool(nh: int, S: int, B: int, seed: int) -> int:
    rnd = random.Random(seed)
    hit = sorted(rnd.sample(range(64), nh))
    slot = [[-1.0] * R for _ in range(64)]   # x component: -1 free, -2 reserved, >= 0 ready
    frame_in = {}
    total = nh * S
    div_nh = (((1 << 32) + nh - 1) // nh) & 0xFFFFFFFF if nh > 1 else 0
    f_next = i_next = issued = folded = 0
    nfold = [0] * 64
    busy = [0] * 64   # segments left of the lane's item
    item = [None] * 64
    it = 1
    guard = total * (B + 2) + S + 64
    while True:
        idle = [busy[l] == 0 for l in range(64)]
        ntaken = 0
        if any(idle) and issued < total:
            ranks = [l for l in range(64) if idle[l]]
            taken = []
            for rank, l in enumerate(ranks):
                if issued + rank >= total:
                    break
                ii = i_next + rank
                q = ii if nh == 1 else (ii * div_nh) >> 32
                f, s = f_next + q, ii - q * nh
                src = hit[s]
                if not (slot[src][f % R] == -1.0 and q < R):
                    break   # in order: stop at the first blocked item
                taken.append((l, src, f))
            for l, src, f in taken:
                slot[src][f % R] = -2.0
                frame_in[(src, f % R)] = f
                busy[l] = rnd.randint(1, B + 1)
                item[l] = (src, f)
            ntaken = len(taken)
            issued += ntaken
            i_next += ntaken
            while i_next >= nh:
                i_next -= nh
                f_next += 1
        if all(idle) and ntaken == 0 and folded >= total:
            return it
        assert it <= guard, (nh, S, it, guard)
        it += 1
        for l in range(64):
            if busy[l]:
                busy[l] -= 1
                if busy[l] == 0:
                    src, f = item[l]
                    slot[src][f % R] = 0.5
        for p in hit:
            if nfold[p] < S and not slot[p][nfold[p] % R] < 0:
                assert frame_in[(p, nfold[p] % R)] == nfold[p]
                slot[p][nfold[p] % R] = -1.0
                nfold[p] += 1
                folded += 1


@pytest.mark.parametrize("nh", [1, 2, 3, 7, 9, 13, 56, 64])
@pytest.mark.parametrize("S", [9, 64, 256])
def test_ring_pool_drains_in_frame_order(nh, S):
    it = run_pool(nh, S, 8, seed=1000 * nh + S)
    assert it > 0
