"""Host model of the chained-launch protocol (pt_capi.cpp launch_chain, pt_kernel.hip render_body_ct).

A chain of persistent launches over the same tiles.  Each launch has a grid of blocks; the machine
has a fixed number of block slots (the resident grid), a block holds its slot until it exits.  A
block claims tiles from its launch's queue (longest first, the same order every launch) and, before
it touches tile t's pixels, waits until the previous launch has published t (the tile epochs).  The
stream gate of launch e+1 opens once every block of launch e has started (hipStreamWaitValue64 on the
started counter); without the gate the dispatcher may start launch e+1's blocks first.

The model checks, over random interleavings of dispatch and block steps:
  * with the gate, every launch completes (no deadlock) and every tile is folded by launch e only
    after launch e-1 published it -- each pixel's frames in order (scalar.cpp:812);
  * without the gate, an adversarial dispatch order deadlocks (all slots held by waiting blocks of the
    later launch), which is what the gate prevents;
  * the monotonic started counter: a gate evaluated before a restart's launch has started does not
    pass on a count from an earlier launch (the round-6 bug of a counter reset at each restart).
"""
from __future__ import annotations

import random


class Launch:
    def __init__(self, idx, grid, order):
        self.idx = idx
        self.grid = grid
        self.order = list(order)     # tiles in claim order
        self.next = 0                # queue position
        self.started = 0             # blocks started
        self.exited = 0
        self.published = set()

    def done(self):
        return self.exited == self.grid


def simulate(n_launches, n_tiles, slots, grid, seed, gate=True, adversarial=False, max_steps=200000):
    """Returns (completed, fold_log) where fold_log lists (launch, tile) in fold order."""
    rng = random.Random(seed)
    order = sorted(range(n_tiles), key=lambda t: (-(t % 7), t))   # a fixed "longest first" order
    launches = [Launch(e, grid, order) for e in range(n_launches)]
    blocks = []          # running blocks: dict(launch, tile, phase)
    free = slots
    fold_log = []
    pending = 0          # the next launch whose blocks are not all dispatched
    for _ in range(max_steps):
        if all(L.done() for L in launches):
            return True, fold_log
        # dispatcher: eligible launches -- stream order (launch e after e-2 completes: two streams)
        # and, with the gate, e after every block of e-1 has started
        eligible = []
        for L in launches:
            if L.started == L.grid:
                continue
            e = L.idx
            if e >= 2 and not launches[e - 2].done():
                continue
            if gate and e >= 1 and launches[e - 1].started < launches[e - 1].grid:
                continue
            eligible.append(L)
        if eligible and free > 0:
            L = max(eligible, key=lambda x: x.idx) if adversarial else rng.choice(eligible)
            L.started += 1
            free -= 1
            blocks.append({"L": L, "tile": None})
            continue_dispatch = rng.random() < 0.5
            if continue_dispatch:
                continue
        if not blocks:
            continue
        b = rng.choice(blocks)
        L = b["L"]
        if b["tile"] is None:
            if L.next >= len(L.order):          # queue empty: the block exits
                blocks.remove(b)
                L.exited += 1
                free += 1
                continue
            b["tile"] = L.order[L.next]
            L.next += 1
            continue
        t = b["tile"]
        if L.idx >= 1 and t not in launches[L.idx - 1].published:
            continue                            # waits for the previous launch's epoch (spins)
        fold_log.append((L.idx, t))
        L.published.add(t)
        b["tile"] = None
    return False, fold_log


def _check_order(fold_log, n_launches, n_tiles):
    pos = {}
    for i, (e, t) in enumerate(fold_log):
        pos[(e, t)] = i
    assert len(pos) == n_launches * n_tiles
    for e in range(1, n_launches):
        for t in range(n_tiles):
            assert pos[(e - 1, t)] < pos[(e, t)], (e, t)


def test_gated_chain_completes_in_order():
    for seed in range(300):
        ok, log = simulate(n_launches=6, n_tiles=24, slots=4, grid=4, seed=seed)
        assert ok, seed
        _check_order(log, 6, 24)


def test_gated_chain_adversarial_dispatch_completes():
    for seed in range(100):
        ok, log = simulate(n_launches=5, n_tiles=16, slots=3, grid=3, seed=seed, adversarial=True)
        assert ok, seed
        _check_order(log, 5, 16)


def test_ungated_chain_can_deadlock():
    """Without the gate the later launch can take every slot first and wait forever."""
    dead = 0
    for seed in range(100):
        ok, _ = simulate(n_launches=4, n_tiles=16, slots=3, grid=3, seed=seed, gate=False, adversarial=True,
                         max_steps=20000)
        dead += not ok
    assert dead > 0


def test_started_counter_is_monotonic_across_restarts():
    """launch_chain's gate for the first continuing launch after a restart waits for
    started >= cum (all blocks of every chained launch so far).  A counter reset at the restart
    (on the restart's stream, behind its waits) could still hold the old total when the gate is
    evaluated on the other stream; with the monotonic counter the gate needs the restart's own blocks."""
    grids = [1536, 1536, 1280, 1536, 1536]
    cum = 0
    counter = 0
    for g in grids[:3]:          # a first chain segment: every block started
        cum += g
        counter += g
    # restart: its launch has not started yet when the next launch's gate is evaluated
    restart_grid = grids[3]
    cum += restart_grid
    assert not counter >= cum                  # monotonic: the gate stays closed
    reset_cum = restart_grid                   # the buggy scheme: cum and the counter reset to 0 ...
    assert counter >= reset_cum                # ... but a stale counter passes the gate early
    counter += restart_grid                    # the restart's blocks start
    assert counter >= cum


# ---- residency: a queue preemption that restores the later launch first ---------------
# The gate makes the chain deadlock-free only while a started block stays resident.  A preemption saves
# every running block; if the later launch's queue is restored first, its saved blocks and then its
# not-yet-dispatched ones take the free slots, the earlier launch's saved blocks find none, and the
# later launch's blocks wait for tiles the earlier one can no longer fold.  The remedy modelled here (the
# branch chain-defer-wip's design): a block whose tile stays unready for `defer_after` steps defers it
# and exits, claiming nothing more; the launch's last block to exit first runs the deferred tiles and
# what its queue still holds, waiting as long as it must.

def simulate_preempt(n_launches, n_tiles, slots, grid, seed, preempt_at, defer_after=None, max_steps=60000):
    """Returns (completed, fold_log).  At step `preempt_at` every running block is saved; restoring
    gives priority to the later launch (its saved blocks, then its new dispatches), the earlier
    launch's saved blocks get a slot only when the later one has nothing left to place."""
    rng = random.Random(seed)
    order = sorted(range(n_tiles), key=lambda t: (-(t % 7), t))
    launches = [Launch(e, grid, order) for e in range(n_launches)]
    for L in launches:
        L.deferred = []
    blocks, saved = [], []
    free = slots
    fold_log = []
    for step in range(max_steps):
        if all(L.done() for L in launches):
            return True, fold_log
        if step == preempt_at:
            saved, blocks = blocks, []
            free = slots
        # placement: saved blocks of later launches first, then new dispatches, then older saved blocks
        cands = []
        for b in saved:
            cands.append((b["L"].idx, 1, b))
        for L in launches:
            if L.started == L.grid:
                continue
            e = L.idx
            if e >= 2 and not launches[e - 2].done():
                continue
            if e >= 1 and launches[e - 1].started < launches[e - 1].grid:
                continue
            cands.append((e, 0, L))
        if cands and free > 0:
            e, kind, x = max(cands, key=lambda c: (c[0], c[1]))
            if kind == 1:
                saved.remove(x)
                blocks.append(x)
            else:
                x.started += 1
                blocks.append({"L": x, "tile": None, "wait": 0, "stop": False, "drain": False})
            free -= 1
            if rng.random() < 0.5:
                continue
        if not blocks:
            continue
        b = rng.choice(blocks)
        L = b["L"]
        if b["tile"] is None:
            src = None
            if b["drain"] and L.deferred:
                src = L.deferred.pop(0)
            elif not b["stop"] and L.next < len(L.order):
                src = L.order[L.next]
                L.next += 1
            if src is None:
                # the launch's last block to exit runs what was deferred and what the queue holds
                if (defer_after is not None and not b["drain"] and L.exited + 1 == L.grid
                        and (L.deferred or L.next < len(L.order))):
                    b["drain"], b["stop"] = True, False
                    continue
                blocks.remove(b)
                L.exited += 1
                free += 1
                continue
            b["tile"], b["wait"] = src, 0
            continue
        t = b["tile"]
        if L.idx >= 1 and t not in launches[L.idx - 1].published:
            b["wait"] += 1
            if defer_after is not None and not b["drain"] and b["wait"] > defer_after:
                L.deferred.append(t)                    # defer it, claim nothing more, exit
                b["tile"], b["stop"] = None, True
            continue
        fold_log.append((L.idx, t))
        L.published.add(t)
        b["tile"] = None
    return False, fold_log


def test_preemption_restoring_the_later_launch_first_can_stall_the_chain():
    """The residency gap: with waits that hold their slot, a restore that favours the later launch
    leaves the earlier launch's saved blocks without slots while the later launch's blocks wait on it."""
    stalled = 0
    for seed in range(60):
        ok, _ = simulate_preempt(n_launches=4, n_tiles=24, slots=4, grid=4, seed=seed, preempt_at=40,
                                 max_steps=20000)
        stalled += not ok
    assert stalled > 0


def test_deferral_survives_the_preemption_and_keeps_frame_order():
    """With deferral every launch completes under the same restores, and every tile is still folded by
    launch e only after launch e-1 folded it."""
    for seed in range(60):
        for preempt_at in (25, 40, 70):
            ok, log = simulate_preempt(n_launches=4, n_tiles=24, slots=4, grid=4, seed=seed, preempt_at=preempt_at,
                                       defer_after=30)
            assert ok, (seed, preempt_at)
            _check_order(log, 4, 24)


def test_deferral_without_preemption_keeps_frame_order():
    for seed in range(100):
        ok, log = simulate_preempt(n_launches=5, n_tiles=20, slots=3, grid=3, seed=seed, preempt_at=-1, defer_after=3)
        assert ok, seed
        _check_order(log, 5, 20)
