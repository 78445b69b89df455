"""Key-for-key validation of a job's result against an independent oracle.

The reference's output contract is the word table in first-occurrence order
plus the total (/root/reference/main.cu:208-218).  `synthetic_oracle` builds
the exact expected table of a benchmark configuration from the synthetic
generator's own word walk (``cpu_count_synth``: no tokenizer involved), also
for the host-staged configs whose ranks replay a pool of chunks;
`compare_results` checks words, order, counts, first offsets and the total.
"""
from __future__ import annotations

import numpy as np

from ..ops import Result, cpu_count_synth

SEG = 1024  # synthetic segment size (src/kernels/synth.hpp)


def compare_results(got: Result, want: Result) -> str:
    """'' if identical, else a short description of the first difference."""
    if got.total != want.total:
        return f"total {got.total} != {want.total}"
    if len(got) != len(want):
        return f"{len(got)} distinct words != {len(want)}"
    if got.words != want.words:
        i = next(i for i, (a, b) in enumerate(zip(got.words, want.words)) if a != b)
        return f"row {i}: word {got.words[i]!r} != {want.words[i]!r}"
    if not np.array_equal(got.counts, want.counts):
        i = int(np.nonzero(got.counts != want.counts)[0][0])
        return f"row {i} ({got.words[i]!r}): count {int(got.counts[i])} != {int(want.counts[i])}"
    if not np.array_equal(got.first_off, want.first_off):
        i = int(np.nonzero(got.first_off != want.first_off)[0][0])
        return f"row {i} ({got.words[i]!r}): first offset {int(got.first_off[i])} != {int(want.first_off[i])}"
    return ""


def merge_results(parts) -> Result:
    """Union of per-shard tables: counts add, first offset = min, first-occurrence order."""
    acc = {}
    for r in parts:
        for w, c, f in zip(r.words, r.counts, r.first_off):
            e = acc.get(w)
            if e is None:
                acc[w] = [int(c), int(f)]
            else:
                e[0] += int(c)
                e[1] = min(e[1], int(f))
    rows = sorted(acc.items(), key=lambda kv: kv[1][1])
    return Result([w for w, _ in rows], np.array([v[0] for _, v in rows], np.uint64),
                  np.array([v[1] for _, v in rows], np.uint64), sum(v[0] for _, v in rows))


def synthetic_oracle(world: int, nbytes: int, seed: int, vocab: int, zipf: float, pool_bytes: int = 0,
                     chunk: int = 0, threads: int = 16, long_frac: float = 0.0) -> Result:
    """Expected table of a benchmark run: rank r owns segments [r*nseg, (r+1)*nseg) of one
    logical stream (global offset r*nbytes).  Device-resident configs count that stream;
    host-staged configs (pool_bytes > 0) replay rank r's first pool_bytes in chunks of
    `chunk` up to nbytes (chunk k from pool offset k*chunk mod pool_bytes)."""
    nseg = nbytes // SEG
    if not pool_bytes:
        return cpu_count_synth(world * nbytes, 0, seed, vocab, zipf, 0, threads, long_frac)
    parts = []
    reps, rem = divmod(nbytes, pool_bytes)
    assert chunk and pool_bytes % chunk == 0 and rem % SEG == 0
    for r in range(world):
        base = r * nbytes
        full = cpu_count_synth(pool_bytes, r * nseg, seed, vocab, zipf, base, threads, long_frac)
        if reps:
            full.counts = full.counts * np.uint64(reps)
            full.total *= reps
            parts.append(full)
        if rem:  # a last partial pass over the pool's head
            parts.append(cpu_count_synth(rem, r * nseg, seed, vocab, zipf, base + reps * pool_bytes, threads,
                                         long_frac))
    return merge_results(parts) if len(parts) > 1 else parts[0]
