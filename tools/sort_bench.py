"""Device time of the two first-occurrence orders: radix_sort_pairs (onesweep,
wc_bench_radix_sort) and first_order (the three-launch sample sort of unique
keys, wc_debug_first_order) on first-offset-like keys."""
import ctypes
import sys

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from cuda_mapreduce_amd.ops._lib import check, lib  # noqa: E402

P64 = ctypes.POINTER(ctypes.c_uint64)
P32 = ctypes.POINTER(ctypes.c_uint32)
rng = np.random.default_rng(1)


def first_offsets(n):
    # unique, crowding at the start of the text (Heaps' law), in hash order
    k = np.unique((rng.random(n * 2) ** 2.5 * (1 << 30)).astype(np.uint64))[:n]
    return rng.permutation(k)


for n in [10_000, 100_000, 200_000, 400_000, 1_000_000]:
    keys = first_offsets(n)
    ms = ctypes.c_double(0)
    check(lib.wc_bench_radix_sort(0, keys.ctypes.data_as(P64), len(keys), 30, 5, ctypes.byref(ms)))
    srt = np.empty(len(keys), np.uint64)
    perm = np.empty(len(keys), np.uint32)
    ovf = ctypes.c_int(0)
    ms2 = ctypes.c_double(0)
    if n > 400_000:
        print(f"n={len(keys):>9}: radix {ms.value * 1e3:8.1f} us (no gather)", flush=True)
        continue
    check(lib.wc_debug_first_order(0, keys.ctypes.data_as(P64), len(keys), 6, srt.ctypes.data_as(P64),
                                   perm.ctypes.data_as(P32), ctypes.byref(ovf), ctypes.byref(ms2)))
    ok = np.array_equal(srt, np.sort(keys)) and np.array_equal(keys[perm], srt)
    print(f"n={len(keys):>9}: radix {ms.value * 1e3:8.1f} us (no gather) | sample sort + gather {ms2.value * 1e3:8.1f} us"
          f" ok={ok} overflow={ovf.value}", flush=True)
