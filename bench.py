#!/usr/bin/env python3
"""Headline benchmark: GB/s of text ingested (whole node) + words/s.

BASELINE.json metric "GB/s text ingested (whole node) + words/sec at 1/2/4/8
MI355X"; default config "1 GB synthetic ASCII text" per GPU (weak scaling:
every rank owns a fixed 1 GiB shard of one logical synthetic stream).

One process per GPU.  For N > 1 the driver launches
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
and ranks merge their key tables with RCCL over xGMI through the native
communicator (default: the MapReduce shuffle — all-to-all of every key to its
hash owner, owner-side merge, gather to rank 0; `merge_mode=1`: reduce-scatter
+ all-gather of dense count vectors); torch.distributed (backend "nccl" =
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
    ap.add_argument("--steps", type=int, default=1000,
                    help="timed steps (default ~1.4 s of GPU work at 1 GiB: long enough for an external utilisation sampler)")
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="1gb", help="BASELINE config (cuda_mapreduce_amd.models.CONFIGS)")
    ap.add_argument("--gb-per-gpu", type=float, default=None, help="override: GiB of synthetic text per GPU")
    ap.add_argument("--vocab", type=int, default=None)
    ap.add_argument("--zipf", type=float, default=None)
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--chunk-gb", type=float, default=None)
    ap.add_argument("--pool-gb", type=float, default=None, help="host-staged: replay pool per GPU")
    ap.add_argument("--merge", choices=["shuffle", "dense"], default=None,
                    help="cross-GPU merge: shuffle (all-to-all to hash owners) or dense (reduce-scatter + all-gather);"
                         " default: the config's (dense: SURVEY §5.8 reduce-scatter; shuffle is ~0.06 ms faster at W = 8)")
    ap.add_argument("--no-oracle", action="store_true",
                    help="skip the key-for-key check against the generator-walk oracle (sum check only)")
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

    import resource

    from cuda_mapreduce_amd.models import CONFIGS
    from cuda_mapreduce_amd.ops import Comm, Engine, HostPool
    from cuda_mapreduce_amd.utils import compare_results, synthetic_oracle

    cfg = CONFIGS[a.config]
    gib = 1 << 30
    per_gpu = int(a.gb_per_gpu * gib) if a.gb_per_gpu is not None else cfg.bytes_per_gpu
    vocab = a.vocab if a.vocab is not None else cfg.vocab
    zipf = a.zipf if a.zipf is not None else cfg.zipf_s
    seed = a.seed if a.seed is not None else cfg.seed
    chunk = int(a.chunk_gb * gib) if a.chunk_gb is not None else cfg.chunk_bytes
    host_staged = cfg.source == "host-staged"

    torch.cuda.set_device(local)
    # WC_MERGE_ALWAYS=1 runs the RCCL communicator and the merge protocol even at
    # world size 1 (launcher / unique-id broadcast / native Comm end to end).
    use_comm = world > 1 or os.environ.get("WC_MERGE_ALWAYS", "0") not in ("", "0")
    if use_comm:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    def barrier():
        if world > 1:
            dist.barrier()

    seg = 1024
    nbytes = per_gpu // seg * seg
    chunk = min(chunk, nbytes) // seg * seg
    merge = a.merge or cfg.merge
    merge_mode = {"shuffle": 0, "dense": 1}[merge]
    eng = Engine(device=local, chunk_bytes=chunk, merge_mode=merge_mode)
    comm = None
    if use_comm:
        uid = [Comm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        comm = Comm(uid[0], rank, world, local)

    # rank r owns segments [r*nseg, (r+1)*nseg) of the logical stream
    first_seg = rank * (nbytes // seg)
    base = rank * nbytes
    pool_bytes = 0
    pool_info = None
    if host_staged:
        # page-locked host pool of whole chunks replayed over PCIe (1 TB config: 128 GiB per GPU),
        # generated natively in place on 16 threads (no pageable copy)
        pool_bytes = int((a.pool_gb if a.pool_gb is not None else cfg.pool_bytes / gib) * gib)
        pool_bytes = max(chunk, pool_bytes // chunk * chunk)
        def rss_now():
            with open("/proc/self/statm") as f:
                return int(f.read().split()[1]) * os.sysconf("SC_PAGE_SIZE")

        rss_before = rss_now()  # interpreter + torch + HIP runtime, before the pool exists
        pool = HostPool(pool_bytes, first_segment=first_seg, seed=seed, vocab=vocab, zipf_s=zipf, threads=16)
        peak = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss * 1024
        pool_info = {"pool_bytes": pool_bytes, "build_s": round(pool.build_seconds, 3),
                     "rss_before_pool_bytes": rss_before, "peak_rss_bytes": peak,
                     "pool_rss_ratio": round((peak - rss_before) / pool_bytes, 4)}
    else:
        eng.synth_device(nbytes, first_segment=first_seg, seed=seed, vocab=vocab, zipf_s=zipf)

    def step():
        eng.reset()
        if host_staged:
            eng.count_pool(pool, nbytes, global_base=base)
        else:
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
    # Validation (untimed): the merged table must equal, key for key (words,
    # first-occurrence order, counts, first offsets, total), the exact table of
    # the whole logical stream computed on the CPU from the synthetic
    # generator's own word walk — independent of every GPU stage and of any
    # tokenizer; and its counts must sum to the words the map kernels counted.
    res = eng.result(comm)
    valid = True
    check = {}
    if rank == 0:
        valid = int(res.total) == int(tokens_total) and int(res.counts.sum()) == int(tokens_total)
        if not valid:
            print(f"bench: VALIDATION FAILED: table total {int(res.total)} (rows sum {int(res.counts.sum())}) "
                  f"!= tokens {int(tokens_total)}", file=sys.stderr, flush=True)
        if not a.no_oracle:
            t1 = time.perf_counter()
            want = synthetic_oracle(world, nbytes, seed, vocab, zipf, pool_bytes=pool_bytes, chunk=chunk)
            diff = compare_results(res, want)
            check = {"oracle": "generator word walk (cpu_count_synth)", "identical": not diff,
                     "seconds": round(time.perf_counter() - t1, 2)}
            if diff:
                valid = False
                print(f"bench: VALIDATION FAILED vs oracle: {diff}", file=sys.stderr, flush=True)
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
            "data": (f"synthetic ({'host pool replayed over PCIe' if host_staged else 'device-generated'} "
                     f"Zipf({zipf}) text, {vocab}-word vocabulary, seed {seed})"),
            "words_per_s": round(words, 1),
            "validated": valid,
            "validation": check or {"oracle": "skipped (--no-oracle): token-sum check only"},
            "distinct_words": keys,
            "config": {
                "model": f"wordcount-mapreduce/{cfg.name}",
                "global_batch": total_bytes,
                "seq_len": nbytes,
                "parallelism": f"dp{world}",
                "bytes_per_gpu": nbytes,
                "chunk_bytes": chunk,
                "merge": merge,
            },
            "stages": st,
        }
        if pool_info:
            out["host_pool"] = pool_info
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    if comm is not None:
        comm.close()
    eng.close()
    if use_comm:
        dist.destroy_process_group()
    return 0 if valid else 1


if __name__ == "__main__":
    sys.exit(main())
