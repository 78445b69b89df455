"""A/B of the reduce design: hash-merge (wc_reduce_buckets) against a
sort + segmented-count reduce, priced by its lower bound — ONE stable radix
sort of a pass's records keyed by k0 (64 bits; the k1 digits and the
segmented count/min pass would come on top).

usage: python tools/sort_vs_hash.py [vocab]   (markdown on stdout)"""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cuda_mapreduce_amd import ops  # noqa: E402
from cuda_mapreduce_amd.ops._lib import check, lib  # noqa: E402

vocab = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
e = ops.Engine(device=0)
e.synth_device(1 << 30, seed=1, vocab=vocab)
for _ in range(3):
    e.reset()
    e.count_resident(1 << 30)
    e.finalize_device()
st = e.stats()
records = int(st["records"])
e.close()
# random 64-bit keys, as many as the pass's records (the hash reduce's kernel time: tools/kstats.sh)
rng = np.random.default_rng(1)
keys = rng.integers(0, 1 << 63, records, dtype=np.uint64)
P64 = ctypes.POINTER(ctypes.c_uint64)
out = {}
for bits in (32, 64):
    ms = ctypes.c_double(0)
    check(lib.wc_bench_radix_sort(0, keys.ctypes.data_as(P64), records, bits, 4, ctypes.byref(ms)))
    out[bits] = ms.value
print(f"| vocab | records / GiB | radix sort, 32-bit keys (ms) | radix sort, 64-bit keys (ms) |")
print(f"|---|---:|---:|---:|")
print(f"| {vocab} | {records} | {out[32]:.3f} | {out[64]:.3f} |", flush=True)
