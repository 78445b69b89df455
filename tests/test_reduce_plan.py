"""CPU mirror of the reduce's dispatch plan (src/kernels/reduce.hip lpt_piece):
every block derives, from the map's per-bucket weights, which bucket piece it
reduces.  Checked here for random and skewed weights: every bucket is reduced
exactly once — all its pieces (quarters) present, each on one block, a
bucket's pieces on consecutive blocks starting at its `base` (the partial
slots the last piece merges), nothing past the grid — heavy buckets are split
only while the extra pieces fit the grid, and pieces run heaviest class first."""
import random

RED_SPLIT_MAX_Q = 16


def plan(weights, grid):
    nb = len(weights)
    w = [x + 1 for x in weights]
    W = sum(w)
    n = []
    for x in w:
        n.append(min(RED_SPLIT_MAX_Q, x * (grid - nb) // W + 1))
    P = sum(n)
    if P > grid:
        n = [1] * nb
        P = nb
    cls = [min(7, 4 * x * P // (W * k)) for x, k in zip(w, n)]
    tot = [0] * 8
    first = [0] * nb
    within = [0] * 8
    for b in range(nb):
        first[b] = within[cls[b]]
        within[cls[b]] += n[b]
        tot[cls[b]] += n[b]
    base = []
    for b in range(nb):
        before = sum(tot[k] for k in range(7, cls[b], -1))
        base.append(before + first[b])
    blocks = {}
    for i in range(grid):
        hit = [(b, i - base[b], n[b], base[b]) for b in range(nb) if base[b] <= i < base[b] + n[b]]
        assert len(hit) <= 1
        if hit:
            blocks[i] = hit[0]
    return blocks, n, cls


def test_dispatch_plan():
    rnd = random.Random(7)
    for trial in range(300):
        nb = rnd.choice([64, 128, 256, 512])
        extra = rnd.choice([0, 16, 64]) if nb >= 256 else 512 - nb
        if trial % 3 == 0:  # skewed: a few buckets far above the mean (LONG-heavy buckets)
            weights = [rnd.randint(900, 1100) for _ in range(nb)]
            for _ in range(rnd.randint(1, 6)):
                weights[rnd.randrange(nb)] *= rnd.choice([2, 3, 8, 40])
        else:
            weights = [rnd.choice([0, 1, 50, 1000, 1200]) for _ in range(nb)]
        blocks, n, cls = plan(weights, nb + extra)
        seen = {}
        for i, (b, q, nq, base) in blocks.items():
            assert 0 <= q < nq and i == base + q
            seen.setdefault(b, set()).add(q)
        assert sorted(seen) == list(range(nb))
        assert all(seen[b] == set(range(n[b])) for b in range(nb))
        assert sum(n) <= nb + extra
        if nb < 256 and trial % 3:  # the split regime: pieces of about W / grid each
            W = sum(x + 1 for x in weights)
            for b in range(nb):
                assert (weights[b] + 1) / n[b] <= W / (nb + extra - nb) + 1 or n[b] == RED_SPLIT_MAX_Q
        order = [cls[blocks[i][0]] for i in sorted(blocks)]
        assert order == sorted(order, reverse=True)  # heaviest class first
