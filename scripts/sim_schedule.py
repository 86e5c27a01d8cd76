"""Dev tool: a model of the diffuse kernel's tile pool and launch schedule, driven by the exact path
lengths of the scalar path (scripts/sim_lengths.c).  Used to weigh scheduling / pool changes on the
CPU before building them.

    python scripts/sim_schedule.py [--variant base|help] [--chunk 8] [--tile 8]

Model: a wave runs one 8x8 tile at a time (phase A = 1 iteration, phase B = the (pixel, frame) item
pool of pt_kernel.hip's render_body with OWN_LAST, phase C ~ kTileC iterations); every iteration
costs the same; waves share their SIMD's issue rate (5 per SIMD, rate(k) from
profiles/r01_valu_microbench.txt's mixes); tiles in longest-first order from the previous launch's
costs, cut into units of ~12 iterations.
"""
from __future__ import annotations

import argparse
import ctypes
import heapq
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
RATE = {0: 0.0, 1: 0.432, 2: 0.81, 3: 0.83, 4: 0.833, 5: 0.85}   # wave-instr per SIMD per ns
K_TILE_C = 1.5


def lengths(w, h, frame_first, nframes, bounces):
    L = ctypes.CDLL(str(ROOT / "build" / "libsimlen.so"))
    out = np.zeros(w * h * nframes, np.uint8)
    L.sim_lengths(w, h, frame_first, nframes, bounces, out.ctypes.data_as(ctypes.c_void_p), 8)
    return out.reshape(h, w, nframes)


def pool_iterations(rem_own, items, lanes=64):
    """Iterations of the item pool: lanes start with rem_own (0 = idle), then take `items`
    (remaining segments each) in lane order as they free up."""
    rem = np.array(rem_own, np.int64)
    nxt = 0
    n = len(items)
    it = 0
    while True:
        idle = np.nonzero(rem == 0)[0]
        if len(idle) and nxt < n:
            k = min(len(idle), n - nxt)
            rem[idle[:k]] = items[nxt:nxt + k]
            nxt += k
        if not (rem > 0).any():
            return it
        it += 1
        rem = np.maximum(rem - 1, 0)


def tile_costs(Ls, tile=8, chunk=8, per_chunk=False, tile_h=None):
    """Pool iterations per tile (1 + phase B), the kernel's cost record (per_chunk: the phase-B
    iterations of each chunk of `chunk` frames, shape (tiles, chunks)).  tile_h: tile rows (8x4
    half tiles: tile_h=4), tiles numbered row-major."""
    h, w, S = Ls.shape
    tile_h = tile if tile_h is None else tile_h
    th, tw = (h + tile_h - 1) // tile_h, (w + tile - 1) // tile
    cost = np.zeros(th * tw, np.int64)
    chunks = np.zeros((th * tw, (S + chunk - 1) // chunk), np.int64)
    for ty in range(th):
        for tx in range(tw):
            blk = Ls[ty * tile_h:(ty + 1) * tile_h, tx * tile:(tx + 1) * tile].reshape(-1, S).astype(np.int64)
            hit = blk[:, 0] > 1 if S else np.zeros(len(blk), bool)
            # a pixel whose camera ray misses has length 1 in every frame; a hit has >= 2
            total = 1
            for f0 in range(0, S, chunk):
                nf = min(chunk, S - f0)
                own = nf > 1
                sub = blk[hit, f0:f0 + nf] - 1          # segments after bounce 0
                rem_own = np.zeros(64, np.int64)
                if own:
                    lanes = np.nonzero(hit)[0]
                    rem_own[lanes] = sub[:, nf - 1]
                    items = sub[:, :nf - 1].reshape(-1)
                else:
                    items = sub.reshape(-1)
                it = pool_iterations(rem_own, items)
                chunks[ty * tw + tx, f0 // chunk] = it
                total += it
            cost[ty * tw + tx] = total
    return chunks if per_chunk else cost


def units_of(order, cost, unit_cost=12):
    units = []
    i = 0
    n = len(order)
    while i < n:
        c = cost[order[i]]
        per = 1 if (c >= unit_cost or c == 0) else unit_cost // c
        j = i
        while j < n and j - i < per and cost[order[j]] == c:
            j += 1
        units.append(order[i:j])
        i = j
    return units


def prio_rates(simd_of, running, level, nsimd):
    """Per-wave issue rate when waves of higher s_setprio level issue first: the top level's k_t
    waves share RATE[k_t]; each lower level shares what the levels above leave of RATE[k]."""
    r = np.zeros(len(simd_of))
    idx = np.nonzero(running)[0]
    order = np.lexsort((-level[idx], simd_of[idx]))
    idx = idx[order]
    sims = simd_of[idx]
    starts = np.r_[0, np.nonzero(np.diff(sims))[0] + 1, len(idx)]
    for a, b in zip(starts[:-1], starts[1:]):
        ws = idx[a:b]
        lv = level[ws]
        used = 0.0
        k_above = 0
        for L in sorted(set(lv.tolist()), reverse=True):
            g = ws[lv == L]
            k_above += len(g)
            avail = RATE[min(k_above, 5)] - used
            r[g] = max(avail, 0.0) / len(g)
            used = RATE[min(k_above, 5)]
    return r


def simulate(units, waves=5120, per_simd=5, dt_ns=200.0, iter_instr=900.0, deq_ns=0.0, deq_rate=0.0,
             prio=None):
    """prio: cost thresholds for s_setprio levels 1, 2, 3 (None: no priorities)."""
    """units: lists of job costs (iterations).  Time-stepped: each SIMD shares RATE[k] among its k
    busy waves.  Returns (span_us, idle_frac)."""
    nsimd = waves // per_simd
    simd_of = np.arange(waves) % nsimd
    work = np.zeros(waves)              # remaining instructions of the current tile
    level = np.zeros(waves, np.int64)
    def lvl(c):
        return 0 if prio is None else int(sum(c >= t for t in prio))
    queue = [list(u) for u in units]
    uq = 0
    cur = [[] for _ in range(waves)]     # remaining tiles of the wave's unit
    alive = np.zeros(waves, bool)
    for wv in range(waves):              # static first units
        if uq < len(queue):
            cur[wv] = queue[uq][:]
            uq += 1
            c = cur[wv].pop(0)
            work[wv] = c * iter_instr
            level[wv] = lvl(c)
            alive[wv] = True
    t_ns = 0.0
    death = np.zeros(waves)
    stall = np.zeros(waves)
    while alive.any():
        running = alive & (stall <= 0)
        if prio is None:
            k = np.bincount(simd_of[running], minlength=nsimd)
            rate = np.array([RATE[min(x, 5)] / max(x, 1) for x in range(6)])
            r = rate[np.minimum(k[simd_of], 5)] * running
        else:
            r = prio_rates(simd_of, running, level, nsimd)
        work -= r * dt_ns
        stall = np.maximum(stall - dt_ns, 0.0)
        t_ns += dt_ns
        done = np.nonzero(alive & (work <= 0))[0]
        ndeq = 0
        for wv in done:
            if not cur[wv]:
                if uq < len(queue):
                    cur[wv] = queue[uq][:]
                    uq += 1
                    ndeq += 1
                    # a dequeue: the wave waits deq_ns (+ queueing when the counters saturate)
                    q_wait = max(0.0, ndeq / deq_rate - dt_ns) if deq_rate else 0.0
                    stall[wv] = deq_ns + q_wait
            if cur[wv]:
                c = cur[wv].pop(0)
                work[wv] += c * iter_instr
                level[wv] = lvl(c)
            else:
                alive[wv] = False
                death[wv] = t_ns
    span = t_ns
    idle = (span - death).sum() / (waves * span)
    return span / 1000.0, idle


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--w", type=int, default=1920)
    ap.add_argument("--h", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=8)
    ap.add_argument("--bounces", type=int, default=8)
    ap.add_argument("--unit", type=int, default=12)
    ap.add_argument("--split", type=int, default=0, help="split tiles costing more than this into frame halves")
    ap.add_argument("--hsplit", type=int, default=0, help="split tiles costing more than this into 8x4 halves")
    ap.add_argument("--iter-instr", type=float, default=721.0)
    ap.add_argument("--rate-scale", type=float, default=1.3)
    ap.add_argument("--deq-ns", type=float, default=0.0, help="latency of a dequeue")
    ap.add_argument("--deq-rate", type=float, default=0.0, help="dequeues per ns the counters sustain (0: unlimited)")
    ap.add_argument("--tail-unit", type=int, default=0, help="unit cost for the last --tail-tiles tiles")
    ap.add_argument("--tail-tiles", type=int, default=0)
    ap.add_argument("--prio", type=str, default="", help="comma-separated cost thresholds of s_setprio 1,2,3")
    args = ap.parse_args()
    for k in RATE:
        RATE[k] *= args.rate_scale
    S = args.spp
    prev = lengths(args.w, args.h, 1, S, args.bounces)
    cur = lengths(args.w, args.h, 1 + S, S, args.bounces)
    c_prev = tile_costs(prev, chunk=S)
    c_cur = tile_costs(cur, chunk=S)
    if args.hsplit:
        hp = tile_costs(prev, chunk=S, tile_h=4)
        hc = tile_costs(cur, chunk=S, tile_h=4)
        tw = (args.w + 7) // 8
        jobs_prev, jobs_cur = [], []
        for t in range(len(c_cur)):
            ty, tx = divmod(t, tw)
            if c_prev[t] > args.hsplit:
                for k in range(2):
                    jobs_prev.append(hp[(2 * ty + k) * tw + tx] + K_TILE_C)
                    jobs_cur.append(hc[(2 * ty + k) * tw + tx] + K_TILE_C)
            else:
                jobs_prev.append(c_prev[t] + K_TILE_C)
                jobs_cur.append(c_cur[t] + K_TILE_C)
        jp, jc = np.array(jobs_prev), np.array(jobs_cur)
    elif args.split:
        h_prev = tile_costs(prev, chunk=S // 2, per_chunk=True)
        h_cur = tile_costs(cur, chunk=S // 2, per_chunk=True)
        jobs_prev, jobs_cur = [], []
        for t in range(len(c_cur)):
            if c_prev[t] > args.split:
                for k in range(2):
                    jobs_prev.append(1 + h_prev[t, k] + K_TILE_C / 2)
                    jobs_cur.append(1 + h_cur[t, k] + K_TILE_C / 2)
            else:
                jobs_prev.append(c_prev[t] + K_TILE_C)
                jobs_cur.append(c_cur[t] + K_TILE_C)
        jp, jc = np.array(jobs_prev), np.array(jobs_cur)
    else:
        jp, jc = c_prev + K_TILE_C, c_cur + K_TILE_C
    order = np.argsort(-jp, kind="stable")
    cp = np.round(jp).astype(np.int64)
    if args.tail_tiles:
        head, tail = order[:-args.tail_tiles], order[-args.tail_tiles:]
        us = units_of(head, cp, args.unit) + units_of(tail, cp, args.tail_unit)
    else:
        us = units_of(order, cp, args.unit)
    units = [[jc[j] for j in u] for u in us]
    prio = [float(x) for x in args.prio.split(",")] if args.prio else None
    span, idle = simulate(units, iter_instr=args.iter_instr, deq_ns=args.deq_ns, deq_rate=args.deq_rate, prio=prio,
                          dt_ns=500.0 if prio else 200.0)
    print(f"jobs {len(jc)} units {len(units)} work {jc.sum():.0f} max job {jc.max():.0f} "
          f"mean/wave {jc.sum() / 5120:.1f}; span {span:.1f} us, idle at end {idle:.3f}")


if __name__ == "__main__":
    main()
