"""Python face of the native engine (src/engine/engine.cpp) and CPU paths.

Reference parity: the whole reference pipeline is ``runMapReduce``
(/root/reference/main.cu:133-162) fed by the host tokenizer (main.cu:181-206);
``Engine.count_*`` + ``Engine.result`` are its MI355X-native equivalent.
"""
from __future__ import annotations

import ctypes
import json
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

from ._lib import Options, check, check_ptr, lib

_P8 = ctypes.POINTER(ctypes.c_uint8)
_P64 = ctypes.POINTER(ctypes.c_uint64)


def _u8ptr(buf) -> "ctypes._Pointer":
    arr = np.frombuffer(buf, dtype=np.uint8) if not isinstance(buf, np.ndarray) else buf
    return arr.ctypes.data_as(_P8), arr


@dataclass
class Result:
    """Distinct words in first-occurrence order with their counts."""

    words: List[bytes] = field(default_factory=list)
    counts: np.ndarray = field(default_factory=lambda: np.zeros(0, np.uint64))
    first_off: np.ndarray = field(default_factory=lambda: np.zeros(0, np.uint64))
    total: int = 0

    def __len__(self) -> int:
        return len(self.words)

    def as_dict(self) -> dict:
        return {w: int(c) for w, c in zip(self.words, self.counts)}

    def rows(self):
        return list(zip(self.words, (int(c) for c in self.counts)))

    @classmethod
    def _from_native(cls, p) -> "Result":
        try:
            n = lib.wc_result_size(p)
            nb = lib.wc_result_bytes(p)
            counts = np.zeros(n, np.uint64)
            first = np.zeros(n, np.uint64)
            offs = np.zeros(n + 1, np.uint64)
            blob = ctypes.create_string_buffer(max(nb, 1))
            lib.wc_result_export(p, counts.ctypes.data_as(_P64), first.ctypes.data_as(_P64), offs.ctypes.data_as(_P64), blob)
            raw = blob.raw
            words = [raw[int(offs[i]) : int(offs[i + 1])] for i in range(n)]
            res = cls(words, counts, first, int(lib.wc_result_total(p)))
            return res
        finally:
            lib.wc_result_free(p)


def format_output(res: Result, echo: Optional[bytes] = None, list_rows: bool = True, top_k: int = 0) -> bytes:
    """Reference-identical framing (/root/reference/main.cu:166-218)."""
    out = bytearray(b"Input Data:\n")
    if echo:
        out += echo
    out += b"-" * 26 + b"\n"
    if list_rows:
        idx = range(len(res))
        if top_k and top_k < len(res):
            order = sorted(range(len(res)), key=lambda i: (-int(res.counts[i]), int(res.first_off[i])))
            idx = order[:top_k]
        for i in idx:
            out += res.words[i] + b"\t" + str(int(res.counts[i])).encode() + b"\n"
    out += b"-" * 26 + b"\n"
    out += b"Total Count:" + str(res.total).encode() + b"\n"
    return bytes(out)


def default_options(**kw) -> Options:
    o = Options()
    lib.wc_default_options(ctypes.byref(o))
    for k, v in kw.items():
        if not hasattr(o, k):
            raise TypeError(f"unknown engine option {k!r}")
        setattr(o, k, v)
    return o


def device_count() -> int:
    return int(lib.wc_device_count())


class Comm:
    """RCCL communicator owned by the native engine (one rank per GPU)."""

    def __init__(self, unique_id: bytes, rank: int, size: int, device: int):
        buf = ctypes.create_string_buffer(unique_id, 128)
        self._p = check_ptr(lib.wc_comm_rccl_create(buf, rank, size, device))
        self.rank, self.size = rank, size

    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(128)
        check(lib.wc_rccl_unique_id(buf))
        return buf.raw

    def barrier(self) -> None:
        """Every rank reaches this point (an RCCL all-reduce waited for under the watchdog)."""
        check(lib.wc_comm_barrier(self._p))

    def allgather_host(self, data: bytes) -> List[bytes]:
        """Rank r's ``data`` (same length on every rank) for every r, over the communicator."""
        n = len(data)
        send = ctypes.create_string_buffer(data, max(n, 1))
        recv = ctypes.create_string_buffer(max(n * self.size, 1))
        check(lib.wc_comm_allgather_host(self._p, send, n, recv))
        raw = recv.raw
        return [raw[r * n:(r + 1) * n] for r in range(self.size)]

    def allreduce_f64(self, values: Sequence[float], op: str = "max") -> List[float]:
        """Element-wise max / sum over ranks of a few host doubles (all-gather + fold)."""
        a = np.asarray(values, dtype=np.float64)
        parts = [np.frombuffer(b, dtype=np.float64) for b in self.allgather_host(a.tobytes())]
        m = np.stack(parts)
        return list((m.max(axis=0) if op == "max" else m.sum(axis=0)).tolist())

    def close(self) -> None:
        if getattr(self, "_p", None):
            lib.wc_comm_destroy(self._p)
            self._p = None

    def __del__(self):
        self.close()


class Engine:
    """One GPU's MapReduce engine: count text, then merge / order / download."""

    def __init__(self, device: int = 0, **opts):
        self.options = default_options(device=device, **opts)
        self._p = check_ptr(lib.wc_engine_create(ctypes.byref(self.options)))
        self._resident = 0

    def close(self) -> None:
        if getattr(self, "_p", None):
            lib.wc_engine_destroy(self._p)
            self._p = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def reset(self) -> None:
        check(lib.wc_engine_reset(self._p))

    def set_stage_events(self, on: bool) -> None:
        """Stage timing marks (stats()["device_ms"]); each costs the GPU ~4.5 us."""
        if hasattr(lib, "wc_engine_set_stage_events"):  # an older A/B variant build (WC_LIB) keeps them on
            check(lib.wc_engine_set_stage_events(self._p, int(bool(on))))

    def count_bytes(self, data: bytes, global_base: int = 0) -> None:
        """Host text, streamed through the pinned ring (H2D overlapped)."""
        ptr, keep = _u8ptr(data)
        check(lib.wc_count_host(self._p, ptr, len(keep), global_base))

    def count_file(self, path: str, begin: int = 0, end: Optional[int] = None, global_base: Optional[int] = None) -> None:
        import os

        if end is None:
            end = os.path.getsize(path)
        check(lib.wc_count_file(self._p, path.encode(), begin, end, begin if global_base is None else global_base))

    def count_file_checkpointed(self, path: str, checkpoint: str = "", interval: int = 4 << 30, resume: bool = True,
                                begin: int = 0, end: Optional[int] = None, rank: int = 0, world: int = 1) -> "Result":
        """Resumable count of [begin, end) of a file: delimiter-aligned intervals,
        each finalised on the GPU and folded into a host table that is saved with the next byte
        offset to `checkpoint` (per-rank suffix when world > 1).  Returns this rank's table; the
        engine's running table is left empty."""
        return _count_file_checkpointed(self._p, path, checkpoint, interval, resume, begin, end, rank, world)

    def count_replay(self, pool: np.ndarray, total: int, global_base: int = 0) -> None:
        """Replay a host pool of self-contained chunks until `total` bytes (host-staged config)."""
        ptr, keep = _u8ptr(pool)
        check(lib.wc_count_replay(self._p, ptr, len(keep), total, global_base))

    def count_replay_pinned(self, pool: np.ndarray, total: int, global_base: int = 0) -> None:
        """Host-staged path at PCIe speed: the pool (whole chunks, each ending with a
        delimiter) is page-locked once and DMA'd straight to HBM, overlapped with compute."""
        ptr, keep = _u8ptr(pool)
        self._pool = keep  # must stay alive (and registered) while the engine uses it
        check(lib.wc_count_pinned_replay(self._p, ptr, len(keep), total, global_base))

    def count_pool(self, pool: "HostPool", total: int, global_base: int = 0) -> None:
        """Host-staged path from a native page-locked pool (HostPool): no registration, no copies."""
        check(lib.wc_count_pool(self._p, pool._p, total, global_base))

    def synth_device(self, nbytes: int, first_segment: int = 0, seed: int = 1, vocab: int = 100000, zipf_s: float = 1.0,
                     long_frac: float = 0.0) -> None:
        """Generate synthetic text directly in HBM (no host/PCIe involvement)."""
        check(lib.wc_synth_device(self._p, nbytes, first_segment, seed, vocab, zipf_s, long_frac))
        self._resident = nbytes

    def count_resident(self, nbytes: Optional[int] = None, global_base: int = 0) -> None:
        check(lib.wc_count_resident(self._p, self._resident if nbytes is None else nbytes, global_base))

    def finalize_device(self, comm: Optional[Comm] = None) -> int:
        n = ctypes.c_uint64(0)
        check(lib.wc_finalize_device(self._p, comm._p if comm else None, ctypes.byref(n)))
        return int(n.value)

    def job_resident(self, nbytes: Optional[int] = None, global_base: int = 0, comm: Optional[Comm] = None) -> int:
        """reset() + count_resident() + finalize_device() in one native call."""
        nbytes = self._resident if nbytes is None else nbytes
        if not hasattr(lib, "wc_job_resident"):  # an older A/B variant build (WC_LIB)
            self.reset()
            self.count_resident(nbytes, global_base)
            return self.finalize_device(comm)
        n = ctypes.c_uint64(0)
        check(lib.wc_job_resident(self._p, nbytes, global_base, comm._p if comm else None, ctypes.byref(n)))
        return int(n.value)

    def result(self, comm: Optional[Comm] = None, all_ranks: bool = False) -> Result:
        return Result._from_native(check_ptr(lib.wc_engine_result(self._p, comm._p if comm else None, int(all_ranks))))

    def sync(self) -> None:
        """hipDeviceSynchronize on the engine's device (the bench's timing brackets)."""
        check(lib.wc_engine_sync(self._p))

    def stats(self) -> dict:
        buf = ctypes.create_string_buffer(2048)
        lib.wc_engine_stats_json(self._p, buf, len(buf))
        return json.loads(buf.value.decode())


def _count_file_checkpointed(eng, path, checkpoint, interval, resume, begin, end, rank, world) -> "Result":
    import os

    if end is None:
        end = os.path.getsize(path)
    return Result._from_native(check_ptr(lib.wc_count_file_checkpointed(
        eng, path.encode(), begin, end, rank, world, checkpoint.encode(), interval, int(resume))))


# ---------------------------------------------------------------- CPU paths --
def cpu_count_file_checkpointed(path: str, checkpoint: str = "", interval: int = 4 << 30, resume: bool = True,
                                begin: int = 0, end: Optional[int] = None) -> Result:
    """CPU-oracle twin of Engine.count_file_checkpointed (same checkpoint file format)."""
    return _count_file_checkpointed(None, path, checkpoint, interval, resume, begin, end, 0, 1)


def cpu_count(data: bytes, global_base: int = 0) -> Result:
    """Single-thread CPU oracle (BASELINE config 1)."""
    ptr, keep = _u8ptr(data)
    return Result._from_native(check_ptr(lib.wc_cpu_count(ptr, len(keep), global_base)))


def cpu_count_compat(data: bytes) -> Result:
    """The reference program's exact quirks."""
    ptr, keep = _u8ptr(data)
    return Result._from_native(check_ptr(lib.wc_cpu_count_compat(ptr, len(keep))))


def synth_host(nbytes: int, first_segment: int = 0, seed: int = 1, vocab: int = 100000, zipf_s: float = 1.0,
               threads: int = 1, long_frac: float = 0.0) -> bytes:
    """Host copy of the synthetic stream (bit-identical to the device generator)."""
    return synth_host_array(nbytes, first_segment, seed, vocab, zipf_s, threads, long_frac).tobytes()


def synth_host_array(nbytes: int, first_segment: int = 0, seed: int = 1, vocab: int = 100000, zipf_s: float = 1.0,
                     threads: int = 8, long_frac: float = 0.0) -> np.ndarray:
    """The synthetic stream generated in place into a numpy array on `threads` threads."""
    out = np.empty(nbytes, np.uint8)
    check(lib.wc_synth_host_mt(out.ctypes.data_as(_P8), nbytes, first_segment, seed, vocab, zipf_s, long_frac,
                               threads))
    return out


def cpu_count_synth(nbytes: int, first_segment: int = 0, seed: int = 1, vocab: int = 100000, zipf_s: float = 1.0,
                    global_base: int = 0, threads: int = 0, long_frac: float = 0.0) -> Result:
    """Exact counts of the synthetic stream from the generator's own word walk (full-scale
    benchmark oracle): independent of every tokenizer."""
    return Result._from_native(check_ptr(lib.wc_cpu_count_synth(nbytes, first_segment, seed, vocab, zipf_s,
                                                                 long_frac, global_base, threads)))


class HostPool:
    """Page-locked synthetic replay pool (host-staged configs), generated in place natively."""

    def __init__(self, nbytes: int, first_segment: int = 0, seed: int = 1, vocab: int = 100000,
                 zipf_s: float = 1.0, threads: int = 16, long_frac: float = 0.0, device: int = -1):
        """device >= 0: the pool's pages and generator threads on that GPU's NUMA node."""
        self._p = check_ptr(lib.wc_pool_create(nbytes, first_segment, seed, vocab, zipf_s, long_frac, threads, device))
        self.nbytes = nbytes
        self.build_seconds = float(lib.wc_pool_build_seconds(self._p))
        self.numa_node = int(lib.wc_pool_numa_node(self._p))

    def close(self) -> None:
        if getattr(self, "_p", None):
            lib.wc_pool_destroy(self._p)
            self._p = None

    def __del__(self):
        self.close()


def numa_of_pci(bus_id: str, sysfs_root: str = "/sys"):
    """(node, cpus) of a PCI device from a sysfs tree (src/io/numa.cpp); node -1 if unknown."""
    node = ctypes.c_int(-1)
    cpus = (ctypes.c_int * 4096)()
    n = lib.wc_numa_of_pci(sysfs_root.encode(), bus_id.encode(), ctypes.byref(node), cpus, 4096)
    return node.value, list(cpus[:min(n, 4096)])


def h2d_bench(device: int = 0, node: int = -1, nbytes: int = 1 << 30, reps: int = 8):
    """Pinned H2D GB/s from a pool on host NUMA node `node` (-1: the GPU's own) -> (GB/s, node used)."""
    g, used = ctypes.c_double(0), ctypes.c_int(-1)
    check(lib.wc_h2d_bench(device, node, nbytes, reps, ctypes.byref(g), ctypes.byref(used)))
    return g.value, used.value


def file_read_bench(path: str, piece: int = 64 << 20, device: int = 0):
    """Host read rate of the file path (pread_parallel into page-locked memory, no GPU copy) -> (GB/s, bytes)."""
    g, n = ctypes.c_double(0), ctypes.c_uint64(0)
    check(lib.wc_file_read_bench(path.encode(), piece, device, ctypes.byref(g), ctypes.byref(n)))
    return g.value, n.value


def shard_range(data: bytes, rank: int, world: int):
    """Ownership-adjusted [begin, end) of shard `rank` (token owned by its first byte)."""
    ptr, keep = _u8ptr(data)
    b, e = ctypes.c_uint64(), ctypes.c_uint64()
    check(lib.wc_shard_range_mem(ptr, len(keep), rank, world, ctypes.byref(b), ctypes.byref(e)))
    return int(b.value), int(e.value)


def shard_range_file(path: str, rank: int, world: int):
    b, e = ctypes.c_uint64(), ctypes.c_uint64()
    check(lib.wc_shard_range_file(path.encode(), rank, world, ctypes.byref(b), ctypes.byref(e)))
    return int(b.value), int(e.value)


def virtual_bench(ranks: int, nbytes: int, seed: int = 1, vocab: int = 100000, zipf_s: float = 1.0,
                  long_frac: float = 0.0, steps: int = 20, warmup: int = 3, device: int = 0, **opts):
    """`ranks` virtual ranks (threads, stream-ordered loopback communicator) on
    one GPU run bench.py's step on their own resident shards of one synthetic
    stream.  Returns (rank 0's merged Result, per-rank dicts of wall ms/step and
    the last job's device stage times)."""
    o = default_options(**opts)
    out = (ctypes.c_double * (14 * ranks))()
    res = Result._from_native(check_ptr(lib.wc_virtual_bench(ctypes.byref(o), ranks, device, nbytes, seed, vocab,
                                                             zipf_s, long_frac, steps, warmup, out)))
    keys = ("ms_per_step", "map", "reduce", "finalize", "merge", "idle", "tokens", "keys", "merges_planned",
            "merge_redos", "merge_collectives", "merge_sent_bytes", "merge_peer_bytes", "merge_root_recv_bytes")
    return res, [{k: out[14 * r + i] for i, k in enumerate(keys)} for r in range(ranks)]


def loopback_count(data: bytes, ranks: int, devices: Optional[Sequence[int]] = None, all_ranks: bool = False,
                   resident: bool = False, warm: Optional[bytes] = None, **opts) -> Result:
    """`ranks` virtual ranks (threads) on `devices` count shards and merge in-process.

    Returns rank 0's table; with ``all_ranks`` every rank receives the merged
    table and the native side checks that they all equal rank 0's.  With
    ``resident`` each shard is counted from HBM and the merge runs behind the
    pending last pass (the bench's speculative merged finalize).  ``warm``: a
    first job on that text (its result dropped), so the merge of ``data``
    plans from the caps it learned."""
    ptr, keep = _u8ptr(data)
    wptr, wkeep = _u8ptr(warm) if warm is not None else (None, b"")
    devs = (ctypes.c_int * ranks)(*(devices if devices is not None else [0] * ranks))
    o = default_options(**opts)
    return Result._from_native(
        check_ptr(lib.wc_loopback_count(ptr, len(keep), ranks, devs, ctypes.byref(o), int(all_ranks), int(resident),
                                        wptr, len(wkeep))))
