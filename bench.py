#!/usr/bin/env python3
"""Headline benchmark: GB/s of text ingested (whole node) + words/s.

BASELINE.json metric "GB/s text ingested (whole node) + words/sec at 1/2/4/8
MI355X"; default config "1 GB synthetic ASCII text" per GPU (weak scaling:
every rank owns a fixed 1 GiB shard of one logical synthetic stream).

One process per GPU, each loading only the native engine (/opt/rocm's HIP and
RCCL; torch is never imported, so no second runtime shares the process):
  * `python bench.py --gpus N` with no WORLD_SIZE in the environment: this
    process is a launcher that touches no GPU — it checks that N GPUs are
    visible (KFD topology + *_VISIBLE_DEVICES), starts N fresh rank processes
    with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*, relays rank 0's JSON line
    and fails fast (first failing rank -> siblings stopped, its code returned);
  * under `python -m torch.distributed.run --nproc-per-node N ... bench.py`
    (WORLD_SIZE set) each rank runs directly.
Ranks share rank 0's RCCL unique id through a job-private file
(cuda_mapreduce_amd/parallel/launch.py); from then on the job's own RCCL
communicator carries everything: the key-table merge over xGMI, the timing
barriers (RCCL all-reduce + hipDeviceSynchronize on both sides of the timed
loop) and the max-over-ranks step time.

Cross-GPU merge (`--merge`, default: the config's): `shuffle` = the MapReduce
shuffle (all-to-all of every key to its hash owner, owner-side merge, gather to
rank 0); `dense` = owner-numbered dictionary, reduce-scatter of dense count
vectors + all-gather.

A timed step is the full job on the resident shard: map (tokenize + combine),
shuffle, reduce into the running table, compaction, cross-GPU merge and the
first-occurrence ordering of the final table on device.  Text is generated on
the device once before timing (synthetic data: a Zipf(1.0) vocabulary of 100k
words); nothing inside the timed region is cached between steps (the table is
cleared at the start of every step).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def parse(argv=None):
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
    ap.add_argument("--long-frac", type=float, default=None,
                    help="share of the vocabulary that is 16-64-byte words (LONG-key path under load)")
    ap.add_argument("--chunk-gb", type=float, default=None)
    ap.add_argument("--pool-gb", type=float, default=None, help="host-staged: replay pool per GPU")
    ap.add_argument("--merge", choices=["shuffle", "dense"], default=None,
                    help="cross-GPU merge: shuffle (all-to-all to hash owners) or dense (reduce-scatter + all-gather);"
                         " default: the config's")
    ap.add_argument("--no-oracle", action="store_true",
                    help="skip the key-for-key check against the generator-walk oracle (sum check only)")
    ap.add_argument("--json-out", default="")
    ap.add_argument("--virtual-ranks", type=int, default=0,
                    help="W > 0: W engines (threads) on GPU 0 with the stream-ordered loopback communicator, each "
                         "on its own shard of the stream, the merge at world size W — a merge-cost curve on one "
                         "GPU, not a scaling number")
    ap.add_argument("--dry-launch", action="store_true",
                    help="launcher test: ranks report their environment and exit without touching a GPU")
    return ap.parse_args(argv)


def launch(a) -> int:
    """Parent of N rank processes; never loads the engine (no GPU initialised here)."""
    from cuda_mapreduce_amd.parallel import launch as L

    visible = L.visible_gpus()
    if visible < a.gpus:
        print(f"bench: {a.gpus} GPUs requested, {visible} visible", file=sys.stderr, flush=True)
        return 2
    return L.spawn([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], a.gpus)


def dry_rank(rank: int) -> int:
    keys = ["RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "WC_RDZV_DIR",
            "WC_COMM_TIMEOUT_S", "HSA_ENABLE_IPC_MODE_LEGACY"]
    print(json.dumps({"dry_rank": rank, "env": {k: os.environ.get(k) for k in keys},
                      "torch_loaded": "torch" in sys.modules}), flush=True)
    fail = os.environ.get("WC_DRY_FAIL_RANK")
    if fail is not None and int(fail) == rank:
        return 3
    if os.environ.get("WC_DRY_HANG_RANK") not in (None, "") and int(os.environ["WC_DRY_HANG_RANK"]) == rank:
        time.sleep(600)
    return 0


def loaded_runtime() -> dict:
    """HIP runtime / RCCL / engine objects mapped into this process (one of each expected)."""
    libs = {"hip": set(), "rccl": set(), "engine": set(), "torch": "torch" in sys.modules}
    with open("/proc/self/maps") as f:
        for line in f:
            path = line.split()[-1] if "/" in line else ""
            base = os.path.basename(path)
            if base.startswith("libamdhip64.so"):
                libs["hip"].add(path)
            elif base.startswith("librccl.so"):
                libs["rccl"].add(path)
            elif base == "libwc.so":
                libs["engine"].add(path)
    return {k: sorted(v) if isinstance(v, set) else v for k, v in libs.items()}


def run_virtual(a) -> int:
    """--virtual-ranks W: the merged step at world size W on one GPU (all ranks share it)."""
    from cuda_mapreduce_amd.models import CONFIGS
    from cuda_mapreduce_amd.ops import virtual_bench
    from cuda_mapreduce_amd.utils import compare_results, synthetic_oracle

    cfg = CONFIGS[a.config]
    gib = 1 << 30
    W = a.virtual_ranks
    per = (int(a.gb_per_gpu * gib) if a.gb_per_gpu is not None else cfg.bytes_per_gpu) // 1024 * 1024
    vocab = a.vocab if a.vocab is not None else cfg.vocab
    zipf = a.zipf if a.zipf is not None else cfg.zipf_s
    seed = a.seed if a.seed is not None else cfg.seed
    long_frac = a.long_frac if a.long_frac is not None else cfg.long_frac
    chunk = min(int(a.chunk_gb * gib) if a.chunk_gb is not None else cfg.chunk_bytes, per) // 1024 * 1024
    merge = a.merge or cfg.merge
    res, ranks = virtual_bench(W, per, seed=seed, vocab=vocab, zipf_s=zipf, long_frac=long_frac, steps=a.steps,
                               warmup=a.warmup, chunk_bytes=chunk, merge_mode={"shuffle": 0, "dense": 1}[merge])
    tokens = sum(r["tokens"] for r in ranks)
    valid = int(res.total) == int(tokens) and int(res.counts.sum()) == int(tokens)
    check = {"oracle": "skipped (--no-oracle): token-sum check only"}
    if not a.no_oracle:
        t1 = time.perf_counter()
        want = synthetic_oracle(W, per, seed, vocab, zipf, chunk=chunk, long_frac=long_frac)
        diff = compare_results(res, want)
        check = {"oracle": "generator word walk (cpu_count_synth)", "identical": not diff,
                 "seconds": round(time.perf_counter() - t1, 2)}
        valid = valid and not diff
        if diff:
            print(f"bench: VALIDATION FAILED vs oracle: {diff}", file=sys.stderr, flush=True)
    ms = max(r["ms_per_step"] for r in ranks)
    out = {
        "metric": "merged step at W virtual ranks on one GPU (merge-cost curve, not scaling)",
        "virtual_ranks": W, "value": round(W * per / (ms / 1e3) / 1e9, 3), "unit": "GB/s (all ranks share one GPU)",
        "ms_per_step": round(ms, 4), "steps": a.steps, "warmup": a.warmup, "validated": valid, "validation": check,
        "distinct_words": len(res.words),
        "merge_ms": [round(r["merge"], 4) for r in ranks],
        "merges_planned_rank0": int(ranks[0]["merges_planned"]), "merge_redos_rank0": int(ranks[0]["merge_redos"]),
        "stage_ms_rank0": {k: round(ranks[0][k], 4) for k in ("map", "reduce", "finalize", "merge", "idle")},
        "keys_per_rank": [int(r["keys"]) for r in ranks],
        "merge_wire": [{k: int(r[k]) for k in ("merge_collectives", "merge_sent_bytes", "merge_peer_bytes",
                                               "merge_root_recv_bytes")} for r in ranks],
        "config": {"model": f"wordcount-mapreduce/{cfg.name}", "bytes_per_rank": per, "chunk_bytes": chunk,
                   "merge": merge, "vocab": vocab, "long_frac": long_frac,
                   "communicator": "stream-ordered loopback (src/dist/comm.cpp)"},
    }
    line = json.dumps(out)
    print(line, flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            f.write(line + "\n")
    return 0 if valid else 1


def run_rank(a) -> int:
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.dry_launch:
        return dry_rank(rank)
    if world != a.gpus and rank == 0:
        print(f"bench: WORLD_SIZE={world} but --gpus {a.gpus}; using WORLD_SIZE", file=sys.stderr)
    os.environ.setdefault("WC_COMM_TIMEOUT_S", "120")  # read by the native communicator's watchdog

    import resource

    from cuda_mapreduce_amd.models import CONFIGS
    from cuda_mapreduce_amd.ops import Comm, Engine, HostPool, device_count
    from cuda_mapreduce_amd.parallel import launch as L
    from cuda_mapreduce_amd.utils import compare_results, synthetic_oracle

    ndev = device_count()
    if local >= ndev:
        print(f"bench: rank {rank}: LOCAL_RANK {local} but {ndev} GPU(s) visible", file=sys.stderr, flush=True)
        return 2
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if world > 1 and local_world > ndev:
        # RCCL refuses two ranks on one GPU ("Duplicate GPU detected", ncclInvalidUsage:
        # profiles/r6_rccl_one_gpu.md): fail before any rank waits in the rendezvous
        print(f"bench: rank {rank}: {local_world} local ranks but {ndev} GPU(s) visible; RCCL allows one rank per "
              f"GPU (\"Duplicate GPU detected\") — use --virtual-ranks for several ranks on one GPU",
              file=sys.stderr, flush=True)
        return 2

    cfg = CONFIGS[a.config]
    gib = 1 << 30
    per_gpu = int(a.gb_per_gpu * gib) if a.gb_per_gpu is not None else cfg.bytes_per_gpu
    vocab = a.vocab if a.vocab is not None else cfg.vocab
    zipf = a.zipf if a.zipf is not None else cfg.zipf_s
    seed = a.seed if a.seed is not None else cfg.seed
    long_frac = a.long_frac if a.long_frac is not None else cfg.long_frac
    chunk = int(a.chunk_gb * gib) if a.chunk_gb is not None else cfg.chunk_bytes
    host_staged = cfg.source == "host-staged"
    # WC_MERGE_ALWAYS=1 runs the RCCL communicator and the merge protocol even at
    # world size 1 (rendezvous / native Comm / merge end to end on one GPU).
    use_comm = world > 1 or os.environ.get("WC_MERGE_ALWAYS", "0") not in ("", "0")

    seg = 1024
    nbytes = per_gpu // seg * seg
    chunk = min(chunk, nbytes) // seg * seg
    merge = a.merge or cfg.merge
    merge_mode = {"shuffle": 0, "dense": 1}[merge]
    eng = Engine(device=local, chunk_bytes=chunk, merge_mode=merge_mode)
    comm = None
    if use_comm:
        timeout = float(os.environ["WC_COMM_TIMEOUT_S"])
        uid = L.rendezvous_uid(rank, Comm.unique_id, timeout_s=timeout)
        comm = Comm(uid, rank, world, local)
        comm.barrier()  # every rank holds its communicator: the id file may go
        if rank == 0:
            L.rendezvous_cleanup()

    def barrier():
        eng.sync()
        if comm is not None:
            comm.barrier()

    # rank r owns segments [r*nseg, (r+1)*nseg) of the logical stream
    first_seg = rank * (nbytes // seg)
    base = rank * nbytes
    pool_bytes = 0
    pool_info = None
    synth = dict(seed=seed, vocab=vocab, zipf_s=zipf, long_frac=long_frac)
    if host_staged:
        # page-locked host pool of whole chunks replayed over PCIe (1 TB config: 128 GiB per GPU),
        # generated natively in place on 16 threads (no pageable copy)
        pool_bytes = int((a.pool_gb if a.pool_gb is not None else cfg.pool_bytes / gib) * gib)
        pool_bytes = max(chunk, min(pool_bytes, nbytes) // chunk * chunk)

        def rss_now():
            with open("/proc/self/statm") as f:
                return int(f.read().split()[1]) * os.sysconf("SC_PAGE_SIZE")

        rss_before = rss_now()  # interpreter + HIP runtime, before the pool exists
        pool = HostPool(pool_bytes, first_segment=first_seg, threads=16, device=local, **synth)
        peak = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss * 1024
        pool_info = {"pool_bytes": pool_bytes, "build_s": round(pool.build_seconds, 3), "numa_node": pool.numa_node,
                     "rss_before_pool_bytes": rss_before, "peak_rss_bytes": peak,
                     "pool_rss_ratio": round((peak - rss_before) / pool_bytes, 4)}
    else:
        eng.synth_device(nbytes, first_segment=first_seg, **synth)

    def step():  # one whole job: reset, count, finalize (ordered device table)
        if host_staged:
            eng.reset()
            eng.count_pool(pool, nbytes, global_base=base)
            return eng.finalize_device(comm)
        return eng.job_resident(nbytes, global_base=base, comm=comm)

    for _ in range(a.warmup):
        step()
    # stage timing marks cost the GPU ~4.5 us each (profiles/r4_session3.md §9):
    # off in the timed loop; one more untimed step with them on gives "stages"
    eng.set_stage_events(False)
    barrier()
    t0 = time.perf_counter()
    keys = 0
    for _ in range(a.steps):
        keys = step()
    barrier()
    dt = time.perf_counter() - t0
    eng.set_stage_events(True)
    step()
    st = eng.stats()
    ms = dt / max(a.steps, 1) * 1e3
    tokens = st["tokens"]
    if comm is not None:
        ms = comm.allreduce_f64([ms], "max")[0]
        tokens_total = comm.allreduce_f64([float(tokens)], "sum")[0]
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
            want = synthetic_oracle(world, nbytes, seed, vocab, zipf, pool_bytes=pool_bytes, chunk=chunk,
                                    long_frac=long_frac)
            diff = compare_results(res, want)
            check = {"oracle": "generator word walk (cpu_count_synth)", "identical": not diff,
                     "seconds": round(time.perf_counter() - t1, 2)}
            if diff:
                valid = False
                print(f"bench: VALIDATION FAILED vs oracle: {diff}", file=sys.stderr, flush=True)
    if comm is not None:  # every rank exits with rank 0's verdict
        valid = comm.allreduce_f64([0.0 if valid else 1.0], "max")[0] == 0.0
    total_bytes = nbytes * world
    gbps = total_bytes / (ms / 1e3) / 1e9
    words = tokens_total / (ms / 1e3)
    if rank == 0:
        data = (f"synthetic ({'host pool replayed over PCIe' if host_staged else 'device-generated'} "
                f"Zipf({zipf}) text, {vocab}-word vocabulary, seed {seed}"
                + (f", {long_frac:g} of the vocabulary 16-64-byte words" if long_frac else "") + ")")
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
            "data": data,
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
            "control_plane": "native RCCL communicator (file rendezvous), no torch" if comm else "single process",
            "runtime": loaded_runtime(),
            "stages": st,  # from one extra untimed step with the stage marks on
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
    return 0 if valid else 1


def main() -> int:
    a = parse()
    if a.virtual_ranks > 0:
        return run_virtual(a)
    if "WORLD_SIZE" not in os.environ and (a.gpus > 1 or a.dry_launch):
        return launch(a)
    return run_rank(a)


if __name__ == "__main__":
    sys.exit(main())
