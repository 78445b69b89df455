"""Time bitmap_order (wc_debug_order method 1) and first_order on 1M first-offset-like
keys: python tools/bm_probe.py [n] — per-kernel times come from rocprofv3 around it."""
import ctypes
import sys

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))

from cuda_mapreduce_amd.ops._lib import check, lib  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
rng = np.random.default_rng(1)
keys = rng.permutation(np.unique((rng.random(3 * n) ** 4 * (1 << 29)).astype(np.uint64))[:n])
n = len(keys)
srt = np.empty(n, np.uint64)
perm = np.empty(n, np.uint32)
ovf, ms, res = ctypes.c_int(0), ctypes.c_double(0), ctypes.c_uint64(0)
P64, P32 = ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint32)
for method in (1, 0):
    check(lib.wc_debug_order(0, method, keys.ctypes.data_as(P64), n, 10, srt.ctypes.data_as(P64),
                             perm.ctypes.data_as(P32), ctypes.byref(ovf), ctypes.byref(ms), ctypes.byref(res)))
    ok = np.array_equal(srt, np.sort(keys))
    print("method %d n %d: %.1f us/call ovf %d residue %d sorted %s" % (method, n, ms.value * 1e3, ovf.value, res.value, ok))
