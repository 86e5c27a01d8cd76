import random
# A wave's continuous-tiles pool on one tile (nh item pixels x nf frames per chunk, `chunks` chunks),
# pixel-major or frame-major hand-out to 64 lanes, item path lengths geometric (mean ~1/p_end
# iterations, capped at B+1 = 9).  Rule "direct": an ended item whose frame is its pixel's next frame
# to fold lerps into the pixel's LDS accumulator at once; others go to the slots; a chunk's fold
# (once every item of it has ended and the previous chunk is folded) folds what remains and sets
# next = the chunk's end.  Reports the fraction of items that never touch the slots.
def sim(order, nh=64, nf=8, chunks=8, seed=1, p_end=0.7, maxlen=9):
    rnd = random.Random(seed)
    items = []
    for c in range(chunks):
        lst = [(c * nf + f, p) for p in range(nh) for f in range(nf)]
        if order == 'frame':
            lst.sort(key=lambda x: (x[0], x[1]))
        items += lst
    lanes = [None] * 64
    nxt = [0] * nh
    left = [nh * nf] * chunks
    folded = 0
    k = direct = total = it = 0
    while k < len(items) or any(lanes):
        it += 1
        for i in range(64):
            if lanes[i] is None and k < len(items):
                fr, p = items[k]; k += 1
                L = 1
                while L < maxlen and rnd.random() > p_end:
                    L += 1
                lanes[i] = [fr, p, L]
        done = []
        for i in range(64):
            if lanes[i] is not None:
                lanes[i][2] -= 1
                if lanes[i][2] == 0:
                    done.append(lanes[i]); lanes[i] = None
        snap = list(nxt)
        for fr, p, _ in done:
            total += 1
            left[fr // nf] -= 1
            if fr == snap[p]:
                direct += 1; nxt[p] = fr + 1
        while folded < chunks and left[folded] == 0:
            for p in range(nh):
                nxt[p] = max(nxt[p], (folded + 1) * nf)
            folded += 1
    return round(direct / total, 3), it
for pe in (0.5, 0.7):
    for order in ('pixel', 'frame'):
        print('p_end', pe, order, sim(order, p_end=pe), 'one chunk:', sim(order, chunks=1, p_end=pe))
