"""One process per GPU without a second GPU runtime: launcher + rendezvous.

The reference runs on one device in one process (/root/reference/main.cu:133-162).
Here every rank is a fresh process that loads ONLY the native engine
(``lib/libwc.so``: /opt/rocm's HIP runtime and RCCL); nothing in a rank imports
torch, so exactly one HIP runtime and one RCCL live in each process.

* ``visible_gpus()``   counts the GPUs this process may use from the KFD
  topology in sysfs and the *_VISIBLE_DEVICES masks — no HIP call, so the
  launcher itself never initialises a GPU (it may then start children freely).
* ``spawn(argv, n)``   starts n children with RANK / LOCAL_RANK / WORLD_SIZE /
  MASTER_ADDR / MASTER_PORT (the torch.distributed.run contract), relays their
  output, and fails fast: the first child that exits non-zero gets every
  sibling terminated and its exit code returned.
* ``rendezvous_uid()`` shares rank 0's 128-byte RCCL unique id through a file in
  a directory private to the job (``WC_RDZV_DIR``, set by ``spawn``; under
  torch.distributed.run the agent's pid keys it, since every local rank is its
  child).  After ``Comm`` creation the job's own communicator carries the
  control plane (``Comm.barrier``, ``Comm.allgather_host``).
"""
from __future__ import annotations

import glob
import os
import signal
import socket
import subprocess
import sys
import tempfile
import time
from typing import Dict, List, Optional, Sequence

_MASKS = ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")


def kfd_gpu_nodes(root: str = "/sys/class/kfd/kfd/topology/nodes") -> int:
    """GPU agents in the KFD topology (nodes with SIMDs; CPU nodes have none)."""
    n = 0
    for props in glob.glob(os.path.join(root, "*", "properties")):
        try:
            with open(props) as f:
                for line in f:
                    k, _, v = line.partition(" ")
                    if k == "simd_count" and int(v) > 0:
                        n += 1
                        break
        except (OSError, ValueError):
            continue
    return n


def visible_gpus(env: Optional[Dict[str, str]] = None) -> int:
    """GPUs a child process would see: the KFD GPU count, narrowed by every
    visibility mask that is set (WC_FAKE_VISIBLE_GPUS overrides, for tests)."""
    env = os.environ if env is None else env
    fake = env.get("WC_FAKE_VISIBLE_GPUS")
    if fake is not None:
        return int(fake)
    n = kfd_gpu_nodes()
    for m in _MASKS:
        v = env.get(m)
        if v is not None:
            ids = [x for x in v.split(",") if x.strip() != ""]
            n = min(n, len(ids))
    return n


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_env(rank: int, world: int, port: int, rdzv_dir: str, base: Optional[Dict[str, str]] = None) -> Dict[str, str]:
    env = dict(os.environ if base is None else base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WC_RDZV_DIR=rdzv_dir)
    env.setdefault("WC_COMM_TIMEOUT_S", "120")  # a dead peer ends the job instead of hanging it
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL across processes)
    return env


def spawn(argv: Sequence[str], world: int, grace_s: float = 10.0) -> int:
    """Run ``argv`` as ranks 0..world-1 (stdout / stderr inherited: rank 0 alone
    prints the result line).  Returns 0 if every rank succeeded, else the exit
    code of the first rank that failed (128 + signal for a killed rank)."""
    rdzv = tempfile.mkdtemp(prefix="wc_rdzv_")
    port = free_port()
    procs: List[subprocess.Popen] = []
    rc = 0
    try:
        for r in range(world):
            procs.append(subprocess.Popen(list(argv), env=rank_env(r, world, port, rdzv)))
        live = set(range(world))
        while live:
            for r in sorted(live):
                code = procs[r].poll()
                if code is None:
                    continue
                live.discard(r)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    print(f"launch: rank {r} exited with {code}; stopping the other ranks", file=sys.stderr,
                          flush=True)
                    _stop(procs, live, grace_s)
                    live.clear()
                    break
            time.sleep(0.02)
    except BaseException:
        _stop(procs, set(range(len(procs))), grace_s)
        raise
    finally:
        for f in glob.glob(os.path.join(rdzv, "*")):
            try:
                os.unlink(f)
            except OSError:
                pass
        try:
            os.rmdir(rdzv)
        except OSError:
            pass
    return rc


def _stop(procs: List[subprocess.Popen], ranks, grace_s: float) -> None:
    for r in ranks:
        if procs[r].poll() is None:
            procs[r].send_signal(signal.SIGTERM)
    t0 = time.time()
    for r in ranks:
        try:
            procs[r].wait(timeout=max(0.1, grace_s - (time.time() - t0)))
        except subprocess.TimeoutExpired:
            procs[r].kill()
            procs[r].wait()


def _proc_start_epoch(pid: int) -> float:
    """Start time of a process (seconds since the epoch) from /proc; 0 if unknown."""
    try:
        with open(f"/proc/{pid}/stat") as f:
            ticks = int(f.read().rsplit(")", 1)[1].split()[19])
        with open("/proc/stat") as f:
            btime = next(int(l.split()[1]) for l in f if l.startswith("btime"))
        return btime + ticks / os.sysconf("SC_CLK_TCK")
    except (OSError, ValueError, StopIteration, IndexError):
        return 0.0


def rdzv_dir() -> str:
    d = os.environ.get("WC_RDZV_DIR")
    if d:
        return d
    # torch.distributed.run: every local rank is a child of the same agent; the
    # file rendezvous is node-local, so a multi-node job is refused (the RCCL
    # id would have to travel through the agent's store instead)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if world > local:
        raise RuntimeError(f"WORLD_SIZE {world} > LOCAL_WORLD_SIZE {local}: the file rendezvous of the RCCL id is "
                           "single-node only (set WC_RDZV_DIR to a shared directory to override)")
    run = os.environ.get("TORCHELASTIC_RUN_ID", "")
    tag = run if run and run != "none" else str(os.getppid())
    d = os.path.join(tempfile.gettempdir(), f"wc_rdzv_{tag}_{os.environ.get('MASTER_PORT', '0')}")
    os.makedirs(d, exist_ok=True)
    return d


def rendezvous_uid(rank: int, make_uid, timeout_s: float = 120.0, name: str = "rccl_uid") -> bytes:
    """Rank 0 publishes ``make_uid()`` (atomic rename); the others wait for it.

    A file left by an earlier job with the same directory (same agent pid and
    port, crashed before its cleanup) is older than this job's agent: ranks
    ignore any id file written before their parent process started."""
    path = os.path.join(rdzv_dir(), name)
    if rank == 0:
        uid = make_uid()
        tmp = path + f".tmp{os.getpid()}"
        with open(tmp, "wb") as f:
            f.write(uid)
        os.replace(tmp, path)
        return uid
    not_before = _proc_start_epoch(os.getppid()) - 1.0 if not os.environ.get("WC_RDZV_DIR") else 0.0
    t0 = time.time()
    while True:
        try:
            fresh = os.stat(path).st_mtime >= not_before
            with open(path, "rb") as f:
                uid = f.read()
            if fresh and len(uid) == 128:
                return uid
        except FileNotFoundError:
            pass
        if time.time() - t0 > timeout_s:
            raise TimeoutError(f"rank {rank}: no RCCL unique id from rank 0 at {path} after {timeout_s:.0f} s")
        time.sleep(0.005)


def rendezvous_cleanup(name: str = "rccl_uid") -> None:
    """Rank 0, after every rank has created its communicator."""
    d = rdzv_dir()
    try:
        os.unlink(os.path.join(d, name))
    except OSError:
        pass
    if not os.environ.get("WC_RDZV_DIR"):
        try:
            os.rmdir(d)
        except OSError:
            pass
