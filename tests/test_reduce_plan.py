"""CPU mirror of the balanced reduce's plan (src/kernels/reduce.hip
reduce_planned / plan_lo / plan_block / the weight -> record-range map): with
each bucket padded by ceil(G / buckets), every block's weight interval is
non-empty, a bucket's pieces are exactly the blocks [first, last] its interval
meets (so the piece counter the last piece waits for is reached), and the
pieces' record ranges cover each bucket's Rec16 and 24-byte records exactly
once.  (The first GPU run without the pad lost every bucket of a 56-byte input:
blocks with empty intervals never arrived.)"""
import random

W24 = 12  # kernels.hpp RED_W24


def plan_lo(W, G, i):
    return W * i // G


def plan_block(W, G, y):
    i = y * G // W
    while i + 1 < G and plan_lo(W, G, i + 1) <= y:
        i += 1
    while i > 0 and plan_lo(W, G, i) > y:
        i -= 1
    return i


def r24(x, n16, n24):
    return 0 if x <= n16 else min(n24, (x - n16 + W24 - 1) // W24)


def test_plan_pieces_and_ranges():
    rnd = random.Random(5)
    for _ in range(300):
        nb = rnd.choice([64, 128, 256, 512])
        G = rnd.choice([1, 3, 64, 256, 300])
        n16s = [rnd.choice([0, 0, 1, 7, 300, 5000]) for _ in range(nb)]
        n24s = [rnd.choice([0, 0, 1, 3, 40]) for _ in range(nb)]
        pad = (G + nb - 1) // nb
        w = [a + W24 * b + pad for a, b in zip(n16s, n24s)]
        pre = [0]
        for x in w:
            pre.append(pre[-1] + x)
        W = pre[-1]
        assert W >= G
        arrivals = [0] * nb
        got16 = [[] for _ in range(nb)]
        got24 = [[] for _ in range(nb)]
        for i in range(G):
            lo, hi = plan_lo(W, G, i), plan_lo(W, G, i + 1)
            assert lo < hi
            for b in range(nb):
                if not (pre[b] < hi and pre[b + 1] > lo):
                    continue
                arrivals[b] += 1
                fb, lb = plan_block(W, G, pre[b]), plan_block(W, G, pre[b + 1] - 1)
                first, last = fb == i, lb == i
                x0, x1 = max(lo, pre[b]) - pre[b], min(hi, pre[b + 1]) - pre[b]
                n16, n24 = n16s[b], n24s[b]
                a16, b16 = (0 if first else min(x0, n16)), (n16 if last else min(x1, n16))
                a24, b24 = (0 if first else r24(x0, n16, n24)), (n24 if last else r24(x1, n16, n24))
                got16[b] += range(a16, b16)
                got24[b] += range(a24, b24)
        for b in range(nb):
            fb, lb = plan_block(W, G, pre[b]), plan_block(W, G, pre[b + 1] - 1)
            assert arrivals[b] == lb - fb + 1
            assert sorted(got16[b]) == list(range(n16s[b]))
            assert sorted(got24[b]) == list(range(n24s[b]))
