#!/usr/bin/env python3
"""Headline benchmark: GB/s of text ingested (whole node) + words/s.

BASELINE.json metric "GB/s text ingested (whole node) + words/sec at 1/2/4/8
MI355X"; default config "1 GB synthetic ASCII text" per GPU (weak scaling:
every rank owns a fixed 1 GiB shard of one logical synthetic stream).

One process per GPU.  For N > 1 the driver launches
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
and ranks merge their key tables with RCCL (reduce-scatter + all-gather over
xGMI) through the native communicator; torch.distributed (backend "nccl" =
RCCL) carries the rendezvous, the RCCL unique id and the timing barriers.

A timed step is the full job on the resident shard: map (tokenize + combine),
shuffle, reduce into the running table, compaction, cross-GPU merge and the
first-occurrence ordering of the final table on device.  Text is generated on
the device once before timing (synthetic data, random-free: a Zipf(1.0)
vocabulary of 100k words); nothing inside the timed region is cached between
steps (the table is cleared at the start of every step).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def parse():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--gb-per-gpu", type=float, default=1.0, help="GiB of synthetic text per GPU")
    ap.add_argument("--vocab", type=int, default=100000)
    ap.add_argument("--zipf", type=float, default=1.0)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--chunk-gb", type=float, default=1.0)
    ap.add_argument("--json-out", default="")
    return ap.parse_args()


def main() -> int:
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus and rank == 0:
        print(f"bench: WORLD_SIZE={world} but --gpus {a.gpus}; using WORLD_SIZE", file=sys.stderr)

    import torch
    import torch.distributed as dist

    from cuda_mapreduce_amd.ops import Comm, Engine

    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    def barrier():
        if world > 1:
            dist.barrier()

    nbytes = int(a.gb_per_gpu * (1 << 30))
    seg = 1024
    nbytes = nbytes // seg * seg
    chunk = int(a.chunk_gb * (1 << 30))
    eng = Engine(device=local, chunk_bytes=chunk)
    comm = None
    if world > 1:
        uid = [Comm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        comm = Comm(uid[0], rank, world, local)

    # rank r owns segments [r*nseg, (r+1)*nseg) of the logical stream
    first_seg = rank * (nbytes // seg)
    eng.synth_device(nbytes, first_segment=first_seg, seed=a.seed, vocab=a.vocab, zipf_s=a.zipf)
    base = rank * nbytes

    def step():
        eng.reset()
        eng.count_resident(nbytes, global_base=base)
        return eng.finalize_device(comm)

    for _ in range(a.warmup):
        step()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    keys = 0
    for _ in range(a.steps):
        keys = step()
    barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st = eng.stats()
    ms = dt / max(a.steps, 1) * 1e3
    tokens = st["tokens"]
    if world > 1:
        t = torch.tensor([ms, float(tokens)], dtype=torch.float64, device="cuda")
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = t.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        ms, tokens_total = float(mx[0]), float(sm[1])
    else:
        tokens_total = float(tokens)
    total_bytes = nbytes * world
    gbps = total_bytes / (ms / 1e3) / 1e9
    words = tokens_total / (ms / 1e3)
    if rank == 0:
        out = {
            "metric": "GB/s text ingested (whole node)",
            "value": round(gbps, 3),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8 text / u64 counts",
            "data": f"synthetic (device-generated Zipf({a.zipf}) text, {a.vocab}-word vocabulary, seed {a.seed})",
            "words_per_s": round(words, 1),
            "distinct_words": keys,
            "config": {
                "model": "wordcount-mapreduce",
                "global_batch": total_bytes,
                "seq_len": nbytes,
                "parallelism": f"dp{world}",
                "bytes_per_gpu": nbytes,
                "chunk_bytes": chunk,
            },
            "stages": st,
        }
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    if comm is not None:
        comm.close()
    eng.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
