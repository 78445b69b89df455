"""Word-count job definitions: the BASELINE.json configurations.

The reference has one fixed "model": count the words of ./test.txt
(/root/reference/main.cu:164-222).  BASELINE.json names five configurations;
each is a `JobConfig` here and `run_job` executes it on the calling rank
(one process per GPU; see parallel/dist.py for the rendezvous).
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field
from typing import Optional

GiB = 1 << 30
SEG = 1024  # synthetic segment size (src/kernels/synth.hpp)


@dataclass(frozen=True)
class JobConfig:
    name: str
    description: str
    bytes_per_gpu: int = GiB
    gpus: int = 1
    source: str = "device"  # device | host-staged | file | cpu
    chunk_bytes: int = GiB
    pool_bytes: int = 4 * GiB  # host-staged replay pool per rank
    vocab: int = 100000
    zipf_s: float = 1.0
    seed: int = 1
    long_frac: float = 0.0  # share of the vocabulary drawn as 16..64-byte words (LONG-key path)
    path: Optional[str] = None
    merge: str = "shuffle"  # cross-GPU merge: shuffle (all-to-all to hash owners) | dense (reduce-scatter + all-gather)

    @property
    def merge_mode(self) -> int:
        return {"shuffle": 0, "dense": 1}[self.merge]


CONFIGS = {
    c.name: c
    for c in [
        JobConfig("cpu-test", "test.txt word count on CPU reference path (single-thread hash map, no GPU)",
                  source="cpu", path=os.path.join(os.path.dirname(__file__), "..", "..", "tests", "data", "test.txt")),
        JobConfig("1gb", "1 GB synthetic ASCII text per MI355X (map/shuffle/reduce HIP kernels end-to-end; "
                  "N > 1: shuffle merge — all-to-all to hash owners over xGMI)"),
        JobConfig("64gb", "64 GB synthetic text, single MI355X (HBM-resident, chunked)", bytes_per_gpu=64 * GiB,
                  chunk_bytes=2 * GiB),
        # shuffle merge: per-rank merge cost measured at W = 1 / 2 / 4 / 8 (kernel traces + wire bytes,
        # profiles/r5_merge_rank_cost.md) predicts it 26-34 % below the dense reduce-scatter protocol at
        # 100k and 1M keys / rank on an 8-GPU xGMI node (fewer kernels, 3 collectives instead of 5,
        # 30-45 % fewer bytes); --merge dense still selects the reduce-scatter protocol
        JobConfig("256gb-8gpu", "256 GB synthetic text sharded across 8x MI355X, RCCL all-to-all (shuffle) merge",
                  bytes_per_gpu=32 * GiB, gpus=8, chunk_bytes=2 * GiB, merge="shuffle"),
        JobConfig("1tb-8gpu-host-staged", "1 TB synthetic text, 8x MI355X, host-staged pinned hipMemcpyAsync",
                  bytes_per_gpu=128 * GiB, gpus=8, source="host-staged", chunk_bytes=GiB),
    ]
}


@dataclass
class JobResult:
    config: str
    rank: int
    world: int
    bytes: int
    tokens: int
    distinct: int
    seconds: float
    stats: dict = field(default_factory=dict)

    @property
    def gb_per_s(self) -> float:
        return self.bytes / self.seconds / 1e9


def run_job(cfg: JobConfig, rank: int = 0, world: int = 1, local_rank: int = 0, comm=None, engine=None) -> JobResult:
    """Run one configuration on this rank.  Synthetic shards are segment-aligned
    slices of ONE logical stream, so results are independent of `world`."""
    from ..ops import Engine, HostPool, cpu_count

    if cfg.source == "cpu":
        data = open(cfg.path, "rb").read()
        t0 = time.perf_counter()
        res = cpu_count(data)
        return JobResult(cfg.name, rank, world, len(data), res.total, len(res), time.perf_counter() - t0)

    nbytes = cfg.bytes_per_gpu // SEG * SEG
    first_seg = rank * (nbytes // SEG)
    base = rank * nbytes
    own = engine is None
    eng = engine or Engine(device=local_rank, chunk_bytes=cfg.chunk_bytes, merge_mode=cfg.merge_mode)
    try:
        eng.reset()
        if cfg.source == "device":
            eng.synth_device(nbytes, first_segment=first_seg, seed=cfg.seed, vocab=cfg.vocab, zipf_s=cfg.zipf_s,
                             long_frac=cfg.long_frac)
            t0 = time.perf_counter()
            eng.count_resident(nbytes, global_base=base)
        elif cfg.source == "host-staged":
            pool_bytes = max(cfg.chunk_bytes, min(cfg.pool_bytes, nbytes) // cfg.chunk_bytes * cfg.chunk_bytes)
            pool = HostPool(pool_bytes, first_segment=first_seg, seed=cfg.seed, vocab=cfg.vocab, zipf_s=cfg.zipf_s,
                            long_frac=cfg.long_frac)
            t0 = time.perf_counter()
            eng.count_pool(pool, nbytes, global_base=base)
        else:
            raise ValueError(f"unknown source {cfg.source}")
        distinct = eng.finalize_device(comm)
        dt = time.perf_counter() - t0
        st = eng.stats()
        return JobResult(cfg.name, rank, world, nbytes, st["tokens"], distinct, dt, st)
    finally:
        if own:
            eng.close()
