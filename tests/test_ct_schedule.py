"""Host model of the continuous-tiles pool (pt_kernel.hip render_body_ct): the wave's control flow
-- chunk stream, the two contexts A / D, hand-out, retire, fold, the guards -- restated in Python on
random tiles and random path lengths, so that its bookkeeping is checked on the CPU:

  * every item of every chunk is handed out once and ends, and no guard fires;
  * a chunk is folded only after its last item ended, and a tile's chunks fold in frame order
    (so every pixel's lerp chain sees its frames in order, :812);
  * the loop ends (no hang) with every tile folded.

The model mirrors the kernel statement by statement (the names are the kernel's); path lengths are
the number of pool iterations an item takes (1 .. B + 1).
"""
from __future__ import annotations

import random

import pytest

KCHUNK = 8


def run_wave(tiles, S, B, rng):
    """tiles: list of 64-bit hit masks (one per tile).  Returns (folds, iterations, items)."""
    queue = list(range(len(tiles)))
    claimed, queue_done = False, False
    tcur, hmcur, nhcur, f0next = None, 0, 0, 0
    cA, hasA, hasD = 0, False, False
    A, Dc = {}, {}
    lanes = [None] * 64          # item: dict(tile, f, ctx, rem)
    dmask = 0                    # lanes holding D's items (set at retire, bits only cleared)
    folds, ended_items = [], []
    iters = 0

    def start_chunk():
        nonlocal tcur, hmcur, nhcur, f0next, hasA, A, queue_done
        while not hasA:
            if tcur is not None and f0next < S:
                nf = min(KCHUNK, S - f0next)
                A = dict(tile=tcur, hm=hmcur, f0=f0next, nf=nf, iss=0, nit=nhcur * nf)
                f0next += nf
                hasA = True
                break
            tcur = None
            if queue_done:
                break
            if not queue:
                queue_done = True
                break
            t = queue.pop(0)
            hm = tiles[t]
            nh = bin(hm).count("1")
            if nh == 0:
                folds.append((t, 0, S, "const"))
                continue
            tcur, hmcur, nhcur, f0next = t, hm, nh, 0

    def fold_D():
        nonlocal hasD
        folds.append((Dc["tile"], Dc["f0"], Dc["nf"], "items"))
        hasD = False

    start_chunk()
    stall_limit, stall, idle_events = B + 8, 0, 0
    fault = False
    while not fault:
        event = False
        if hasD and dmask == 0:
            fold_D()
            event = True
        if hasA and A["iss"] >= A["nit"] and not hasD:
            Dc = A
            hasD, hasA = True, False
            # every earlier chunk is folded: the items in flight are all A's
            assert all(it is None or it["ctx"] == cA for it in lanes)
            dmask = sum(1 << i for i in range(64) if lanes[i] is not None)
            cA ^= 1
            start_chunk()
            event = True
            if dmask == 0:
                continue
        if not hasA and not hasD:
            break
        idle_events = 0 if event else idle_events + 1
        if idle_events > 2:
            fault = True
            break
        while True:
            idle = [i for i in range(64) if lanes[i] is None]
            ntaken = 0
            if idle and hasA and A["iss"] < A["nit"]:
                ntaken = min(len(idle), A["nit"] - A["iss"])
                for r, lane in enumerate(idle[:ntaken]):
                    k = A["iss"] + r
                    slot, fi = k // A["nf"], k % A["nf"]
                    lanes[lane] = dict(tile=A["tile"], f=A["f0"] + fi, ctx=cA, rem=rng.randint(1, B + 1), slot=slot)
                A["iss"] += ntaken
            if not any(lanes) and ntaken == 0:
                break
            iters += 1
            ended = 0
            for i in range(64):
                it = lanes[i]
                if it is None:
                    continue
                it["rem"] -= 1
                if it["rem"] == 0:
                    ended |= 1 << i
                    ended_items.append((it["tile"], it["f"], it["slot"]))
                    lanes[i] = None
            # a lane of dmask holds a D item until it ends (then it is idle or takes A's)
            assert all(lanes[i] is None or lanes[i]["ctx"] != cA for i in range(64) if (dmask >> i) & 1)
            dmask &= ~ended
            stall = 0 if (ntaken or ended) else stall + 1
            if stall > stall_limit:
                fault = True
                break
            if hasD and dmask == 0:
                break
            if hasA and A["iss"] >= A["nit"] and not hasD:
                break
    assert not fault, "a guard fired"
    return folds, iters, ended_items


@pytest.mark.parametrize("S", [1, 3, 8, 9, 16, 20, 64])
@pytest.mark.parametrize("B", [1, 8])
def test_ct_pool_drains_in_frame_order(S, B):
    rng = random.Random(S * 100 + B)
    for trial in range(6):
        ntiles = rng.randint(1, 12)
        tiles = []
        for _ in range(ntiles):
            kind = rng.random()
            if kind < 0.3:
                tiles.append(0)                                  # sky / all-miss tile
            elif kind < 0.5:
                tiles.append(rng.getrandbits(64) & rng.getrandbits(64))   # partial
            else:
                tiles.append((1 << 64) - 1)                       # every pixel hits
        folds, iters, ended = run_wave(tiles, S, B, rng)
        # every tile folded completely, chunks in frame order, tiles in queue order
        by_tile = {}
        for t, f0, nf, kind in folds:
            by_tile.setdefault(t, []).append((f0, nf, kind))
        assert sorted(by_tile) == list(range(ntiles))
        for t, chunks in by_tile.items():
            if chunks[0][2] == "const":
                assert chunks == [(0, S, "const")]
                continue
            assert [c[0] for c in chunks] == list(range(0, S, KCHUNK)), chunks
            assert sum(c[1] for c in chunks) == S
        # every item of every chunk ended exactly once
        want = sorted((t, f, s) for t, hm in enumerate(tiles) if hm for f in range(S)
                      for s in range(bin(hm).count("1")))
        assert sorted(ended) == want


def test_ct_pool_keeps_lanes_busy():
    """With many full tiles the pool's lanes stay busy across tile boundaries (the point of CT):
    items / (64 x iterations) is close to 1, unlike a per-tile pool whose tail idles."""
    rng = random.Random(7)
    tiles = [(1 << 64) - 1] * 40
    S, B = 8, 8
    folds, iters, ended = run_wave(tiles, S, B, rng)
    # path lengths are uniform in 1..9: mean 5 iterations per item
    util = sum(1 for _ in ended) * 5.0 / (64 * iters)
    assert util > 0.9, util


def _claimed(n, old, from_back):
    """pt_tile_queue.h PtTileQueue::claimed: the dynamic position of a claim whose 64-bit counter
    read `old` (low word: front claims, high word: back claims), None past the group's n units."""
    f, b = old & 0xFFFFFFFF, old >> 32
    if f + b >= n:
        return None
    return n - 1 - b if from_back else f


@pytest.mark.parametrize("n", [0, 1, 2, 7, 64])
def test_front_back_claims_partition_the_group(n):
    """Waves claiming a group's units from the front (atomicAdd 1) and from the back (atomicAdd
    2^32) in any interleaving take every unit exactly once, and a claim past the meeting point gets
    none (pt_tile_queue.h: the last-dispatched blocks take the cheapest units)."""
    rng = random.Random(n)
    for trial in range(50):
        counter, taken = 0, []
        for _ in range(n + 10):
            back = rng.random() < 0.3
            old = counter
            counter += (1 << 32) if back else 1
            pos = _claimed(n, old, back)
            if pos is not None:
                taken.append(pos)
        assert sorted(taken) == list(range(n))
