"""One-process-per-GPU data parallelism.

* Rendezvous and control: torch.distributed (``nccl`` backend = RCCL on ROCm,
  ``gloo`` on CPU).
* Data plane on GPUs: the native engine's RCCL communicator (src/dist/comm.cpp),
  created from a unique id that rank 0 broadcasts through torch.distributed;
  the merge (src/dist/merge.cpp) then runs reduce-scatter + all-gather over
  xGMI on device buffers.
* CPU ranks (tests, hosts without GPUs): the same owner-partitioned merge
  protocols (shuffle / dense) on host data (``host_merge``) over gloo.
* bench.py does not use this module: its ranks never import torch
  (parallel/launch.py: file rendezvous, then the native communicator).

Input sharding: rank r owns every token whose first byte lies in its byte
range (``shard_range``), so shards need no halo exchange.
"""
from __future__ import annotations

import datetime
import os
import struct
from dataclasses import dataclass
from typing import Optional

import numpy as np

from ..ops import Comm, Engine, Result, cpu_count, shard_range, shard_range_file


@dataclass
class DistEnv:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    backend: str = "none"


class CommFault(RuntimeError):
    """A simulated communication failure (``WC_COMM_FAULT``) or a failed peer."""


def comm_timeout_s() -> float:
    """Collective timeout (``WC_COMM_TIMEOUT_S``, default 300 s) — shared with the native RCCL watchdog."""
    try:
        t = float(os.environ.get("WC_COMM_TIMEOUT_S", "300"))
    except ValueError:
        t = 300.0
    return t if t > 0 else 300.0


_calls = 0


def _fault_tick(rank: int) -> None:
    """Fault injection, same contract as src/dist/comm.cpp: ``WC_COMM_FAULT=<rank>[:<n>]``
    makes rank <rank> fail its n-th collective (default the first)."""
    global _calls
    spec = os.environ.get("WC_COMM_FAULT", "")
    _calls += 1
    if not spec:
        return
    r, _, n = spec.partition(":")
    if int(r) == rank and _calls == (int(n) if n else 1):
        raise CommFault(f"injected comm fault (WC_COMM_FAULT) at collective {_calls} of rank {rank}")


def init_from_env(backend: Optional[str] = None) -> DistEnv:
    """Initialise torch.distributed from RANK/WORLD_SIZE/LOCAL_RANK (127.0.0.1 rendezvous).

    Collectives time out after ``comm_timeout_s()`` instead of hanging when a
    peer dies (the reference has no failure handling at all)."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1:
        return DistEnv(rank, world, local, "none")
    import torch
    import torch.distributed as dist

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if not dist.is_initialized():
        timeout = datetime.timedelta(seconds=comm_timeout_s())
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local), timeout=timeout)
        else:
            dist.init_process_group(backend, timeout=timeout)
    return DistEnv(rank, world, local, backend)


def rccl_comm(env: DistEnv, device: int) -> Optional[Comm]:
    """Native RCCL communicator over the ranks of the torch.distributed world."""
    if env.world == 1:
        return None
    import torch.distributed as dist

    uid = [Comm.unique_id() if env.rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    return Comm(uid[0], env.rank, env.world, device)


def _reduce_scatter(t, op):
    """reduce-scatter of a 1-D tensor (len divisible by world); gloo lacks it, so all-reduce + slice."""
    import torch
    import torch.distributed as dist

    world, rank = dist.get_world_size(), dist.get_rank()
    n = t.numel() // world
    if dist.get_backend() == "gloo":
        dist.all_reduce(t, op=op)
        return t[rank * n : (rank + 1) * n].clone()
    out = torch.empty(n, dtype=t.dtype, device=t.device)
    dist.reduce_scatter_tensor(out, t, op=op)
    return out


_M32, _M64 = (1 << 32) - 1, (1 << 64) - 1
_FNV_OFFSET, _FNV_PRIME = 0xCBF29CE484222325, 0x100000001B3


def _fmix64(k: int) -> int:
    k ^= k >> 33
    k = (k * 0xFF51AFD7ED558CCD) & _M64
    k ^= k >> 33
    k = (k * 0xC4CEB9FE1A85EC53) & _M64
    return k ^ (k >> 33)


def key_of(word: bytes):
    """(k0, k1) of a word: src/kernels/keys.hpp key_of (SHORT / MEDIUM exact, LONG hashed)."""
    n = len(word)
    k0 = int.from_bytes(word[:8].ljust(8, b"\0"), "little")
    if n <= 8:
        return k0, n
    if n <= 15:
        return k0, int.from_bytes(word[8:].ljust(8, b"\0"), "little") | (n << 56)
    h = _FNV_OFFSET
    for c in range(8, n, 8):
        h = ((h ^ int.from_bytes(word[c:c + 8].ljust(8, b"\0"), "little")) * _FNV_PRIME) & _M64
    return k0, (1 << 63) | (_fmix64(h ^ n) & ((1 << 62) - 1))


def _mix32(x: int) -> int:
    x ^= x >> 16
    x = (x * 0x7FEB352D) & _M32
    x ^= x >> 15
    x = (x * 0x846CA68B) & _M32
    return x ^ (x >> 16)


def place_hash(k0: int, k1: int) -> int:
    """keys.hpp place_hash: 32-bit placement hash of a packed key."""
    c = (k1 & _M32) ^ (k1 >> 32)
    return _mix32((k0 & _M32) ^ (((k0 >> 32) * 0x9E3779B1) & _M32) ^ ((c * 0x85EBCA77) & _M32))


def _owner(word: bytes, world: int) -> int:
    """Merge owner of a word: keys.hpp owner_of, the rule src/dist/merge.cpp partitions by
    (high bits of the placement hash)."""
    return (place_hash(*key_of(word)) * world) >> 32


def _pack(rows) -> bytes:
    """(word, count, first) rows -> one byte string: per row u32 length, word, u64 count, u64 first."""
    out = bytearray()
    for w, c, f in rows:
        out += struct.pack("<I", len(w)) + w + struct.pack("<QQ", int(c), int(f))
    return bytes(out)


def _unpack(buf: bytes):
    rows, i = [], 0
    while i < len(buf):
        (n,) = struct.unpack_from("<I", buf, i)
        w = bytes(buf[i + 4 : i + 4 + n])
        c, f = struct.unpack_from("<QQ", buf, i + 4 + n)
        rows.append((w, c, f))
        i += 4 + n + 16
    return rows


def _alltoallv_bytes(parts) -> list:
    """Personalised exchange of byte strings: parts[p] goes to rank p; returns what each rank sent here."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size()
    send_sizes = torch.tensor([len(b) for b in parts], dtype=torch.int64)
    recv_sizes = torch.empty(world, dtype=torch.int64)
    dist.all_to_all_single(recv_sizes, send_sizes)
    send = torch.frombuffer(bytearray(b"".join(parts)) or bytearray(1), dtype=torch.uint8)[: int(send_sizes.sum())]
    recv = torch.empty(int(recv_sizes.sum()), dtype=torch.uint8)
    dist.all_to_all_single(recv, send, output_split_sizes=recv_sizes.tolist(), input_split_sizes=send_sizes.tolist())
    raw, out, o = recv.numpy().tobytes(), [], 0
    for n in recv_sizes.tolist():
        out.append(raw[o : o + n])
        o += n
    return out


def host_merge(local: Result, dense: bool = False) -> Result:
    """Merge per-rank results on the host over torch.distributed (CPU ranks over
    gloo): a Python mirror of the owner-partitioned protocols of
    src/dist/merge.cpp (the native merge runs HIP kernels and RCCL, so CPU
    ranks cannot run it):

    1. owner(word) = high bits of the word's placement hash (keys.hpp owner_of,
       the native rule); rows are packed by owner
    2. all-to-all (personalised exchange) of the packed rows
    3. each owner merges what it received (counts add, first offset = min)
    shuffle: 4. the owners' merged rows are gathered to every rank
    dense:   4. owners' sizes all-gathered -> global id = owner base + index;
             5. ids go back to the senders (reverse all-to-all); every rank
                scatters its counts / first offsets into dense vectors by id;
             6. reduce-scatter (sum / min) + all-gather of the vectors; the
                dictionary rows are gathered to every rank
    Every rank returns the merged table in first-occurrence order."""
    import torch
    import torch.distributed as dist

    world, rank = dist.get_world_size(), dist.get_rank()
    rows = list(zip(local.words, (int(c) for c in local.counts), (int(f) for f in local.first_off)))
    by_owner = [[] for _ in range(world)]
    for r in rows:
        by_owner[_owner(r[0], world)].append(r)
    _fault_tick(rank)
    received = _alltoallv_bytes([_pack(b) for b in by_owner])
    merged = {}
    for buf in received:
        for w, c, f in _unpack(buf):
            e = merged.get(w)
            if e is None:
                merged[w] = [c, f]
            else:
                e[0] += c
                e[1] = min(e[1], f)
    own = sorted(merged.items())  # owner slice in a deterministic order (dense: its id order)
    _fault_tick(rank)
    slices = [None] * world
    dist.all_gather_object(slices, [w for w, _ in own])  # the dictionary (sizes give the id bases)
    if not dense:
        vals = [None] * world
        _fault_tick(rank)
        dist.all_gather_object(vals, [v for _, v in own])
        words = [w for sl in slices for w in sl]
        cnt = [v[0] for vl in vals for v in vl]
        first = [v[1] for vl in vals for v in vl]
    else:
        base = np.cumsum([0] + [len(sl) for sl in slices])
        ids = {w: int(base[rank]) + i for i, (w, _) in enumerate(own)}
        # ids back to the senders: for each sender, the ids of the rows it sent here, in its order
        back = [_pack([(w, ids[w], 0) for w, _, _ in _unpack(buf)]) for buf in received]
        _fault_tick(rank)
        mine = _alltoallv_bytes(back)
        G = int(base[-1])
        vpad = max(world, -(-G // world) * world)
        vc = torch.zeros(vpad, dtype=torch.int64)
        vf = torch.full((vpad,), 1 << 62, dtype=torch.int64)
        for p in range(world):
            for (w, c, f), (w2, gid, _) in zip(by_owner[p], _unpack(mine[p])):
                assert w == w2
                vc[gid] = c
                vf[gid] = f
        _fault_tick(rank)
        scnt = _reduce_scatter(vc, dist.ReduceOp.SUM)
        _fault_tick(rank)
        sfirst = _reduce_scatter(vf, dist.ReduceOp.MIN)
        full_cnt = [torch.empty_like(scnt) for _ in range(world)]
        full_first = [torch.empty_like(sfirst) for _ in range(world)]
        _fault_tick(rank)
        dist.all_gather(full_cnt, scnt)
        _fault_tick(rank)
        dist.all_gather(full_first, sfirst)
        words = [w for sl in slices for w in sl]
        cnt = torch.cat(full_cnt)[:G].tolist()
        first = torch.cat(full_first)[:G].tolist()
    order = np.argsort(np.asarray(first, dtype=np.uint64), kind="stable")
    c = np.asarray(cnt, dtype=np.uint64)
    return Result(
        words=[words[i] for i in order],
        counts=c[order],
        first_off=np.asarray(first, dtype=np.uint64)[order],
        total=int(c.sum()),
    )


def gather_merge(local: Result) -> Result:
    """Every rank receives every rank's (small) host table and folds them in rank order:
    counts add, first offset = min, rows in first-occurrence order.  Works on any
    process-group backend (the object all-gather goes through the device for nccl)."""
    import torch.distributed as dist

    world, rank = dist.get_world_size(), dist.get_rank()
    tabs = [None] * world
    _fault_tick(rank)
    dist.all_gather_object(tabs, (list(local.words), [int(c) for c in local.counts],
                                  [int(f) for f in local.first_off]))
    acc = {}
    for words, counts, firsts in tabs:
        for w, c, f in zip(words, counts, firsts):
            if w in acc:
                acc[w][0] += c
                acc[w][1] = min(acc[w][1], f)
            else:
                acc[w] = [c, f]
    rows = sorted(acc.items(), key=lambda kv: kv[1][1])
    return Result(
        words=[w for w, _ in rows],
        counts=np.array([v[0] for _, v in rows], dtype=np.uint64),
        first_off=np.array([v[1] for _, v in rows], dtype=np.uint64),
        total=sum(v[0] for _, v in rows),
    )


class DistributedWordCount:
    """Count one logical input across all ranks; rank 0 (or all) gets the result."""

    def __init__(self, env: DistEnv, use_gpu: bool = True, **engine_opts):
        self.env = env
        self.use_gpu = use_gpu
        self.dense = engine_opts.get("merge_mode", 0) == 1  # CPU ranks: the same protocol choice
        self.engine = Engine(device=env.local_rank, **engine_opts) if use_gpu else None
        self.comm = rccl_comm(env, env.local_rank) if use_gpu else None

    def close(self):
        if self.comm is not None:
            self.comm.close()
        if self.engine is not None:
            self.engine.close()

    def count_bytes(self, data: bytes) -> Result:
        b, e = shard_range(data, self.env.rank, self.env.world)
        return self._count(lambda eng: eng.count_bytes(data[b:e], global_base=b), lambda: cpu_count(data[b:e], b))

    def count_file(self, path: str, checkpoint: str = "", interval: int = 4 << 30, resume: bool = True) -> Result:
        """Count a file sharded over the ranks.  With `checkpoint`, every rank counts its
        shard resumably (src/io/checkpoint.cpp; file `<checkpoint>.r<rank>of<world>`) and
        the per-rank host tables are merged with gather_merge."""
        b, e = shard_range_file(path, self.env.rank, self.env.world)
        if checkpoint:
            if self.use_gpu:
                local = self.engine.count_file_checkpointed(path, checkpoint, interval, resume, b, e,
                                                            self.env.rank, self.env.world)
            else:
                from ..ops.engine import _count_file_checkpointed

                local = _count_file_checkpointed(None, path, checkpoint, interval, resume, b, e,
                                                 self.env.rank, self.env.world)
            return local if self.env.world == 1 else gather_merge(local)

        def host():
            with open(path, "rb") as fh:
                fh.seek(b)
                return cpu_count(fh.read(e - b), b)

        return self._count(lambda eng: eng.count_file(path, b, e), host)

    def _count(self, gpu_fn, cpu_fn) -> Result:
        if self.use_gpu:
            self.engine.reset()
            gpu_fn(self.engine)
            return self.engine.result(self.comm)
        local = cpu_fn()
        if self.env.world == 1:
            return local
        return host_merge(local, dense=self.dense)
