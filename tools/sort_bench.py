"""Device time of radix_sort_pairs (onesweep) on n random / first-offset-like keys (wc_bench_radix_sort)."""
import ctypes
import sys

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from cuda_mapreduce_amd.ops._lib import check, lib  # noqa: E402

P64 = ctypes.POINTER(ctypes.c_uint64)
rng = np.random.default_rng(1)
for n, bits in [(100_000, 30), (1_000_000, 30), (100_000, 64), (10_000_000, 32), (47_800_000, 32)]:
    keys = rng.integers(0, 1 << min(bits, 62), n, dtype=np.uint64)
    ms = ctypes.c_double(0)
    check(lib.wc_bench_radix_sort(0, keys.ctypes.data_as(P64), n, bits, 5, ctypes.byref(ms)))
    print(f"n={n:>9} bits={bits}: {ms.value * 1e3:8.1f} us  ({n / ms.value / 1e6:.1f} Mkeys/s)", flush=True)
