"""Multi-process data-parallel word count on CPU (gloo, world_size 2, 3 and 8):
shard ownership (the native shard splitter, wc_shard_range_*) + the Python
mirror of the owner-partitioned merge protocols
(cuda_mapreduce_amd/parallel/dist.py host_merge — shuffle: all-to-all to hash
owners; dense: owner-numbered dictionary + reduce-scatter / all-gather) must
give exactly the single-process result.  The mirror partitions by the native
owner rule (keys.hpp owner_of, checked against the library below); the native
merge itself (src/dist/merge.cpp: HIP kernels + RCCL) is covered by the GPU
tests (tests/test_gpu_engine.py loopback ranks, tests/test_gpu_launcher.py)."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, path, q, ckpt="", dense=False):
    sys.path.insert(0, ROOT)
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from cuda_mapreduce_amd.parallel import DistributedWordCount, init_from_env

    env = init_from_env("gloo")
    job = DistributedWordCount(env, use_gpu=False, merge_mode=1 if dense else 0)
    res = job.count_file(path, checkpoint=ckpt, interval=20000) if ckpt else job.count_file(path)
    q.put((rank, res.words, [int(c) for c in res.counts], [int(f) for f in res.first_off], res.total))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,ckpt,dense", [(2, False, False), (3, False, True), (8, False, False),
                                              (8, False, True), (2, True, False)])
def test_gloo_data_parallel_matches_single(tmp_path, world, ckpt, dense):
    from cuda_mapreduce_amd.ops import cpu_count, synth_host

    text = synth_host(300_000, seed=5, vocab=4000) + b"tail-without-newline"
    p = tmp_path / "in.txt"
    p.write_bytes(text)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ck = str(tmp_path / "ck") if ckpt else ""
    procs = [ctx.Process(target=_worker, args=(r, world, port, str(p), q, ck, dense)) for r in range(world)]
    for pr in procs:
        pr.start()
    outs = [q.get(timeout=120) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    if ckpt:  # one checkpoint file per rank, each finished at the end of its shard
        assert sorted(os.listdir(tmp_path)) == sorted(["in.txt"] + [f"ck.r{r}of{world}" for r in range(world)])
    want = cpu_count(text)
    for rank, words, counts, first, total in outs:
        assert total == want.total
        assert words == want.words
        assert counts == [int(c) for c in want.counts]
        assert first == [int(f) for f in want.first_off]


def _fault_worker(rank, world, port, path, q):
    sys.path.insert(0, ROOT)
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), WC_COMM_FAULT="1:2", WC_COMM_TIMEOUT_S="15")
    from cuda_mapreduce_amd.parallel import CommFault, DistributedWordCount, init_from_env

    env = init_from_env("gloo")
    job = DistributedWordCount(env, use_gpu=False)
    try:
        job.count_file(path)
        q.put((rank, "ok", ""))
    except CommFault as ex:
        q.put((rank, "fault", str(ex)))
        q.close()
        q.join_thread()  # flush the queue before the hard exit
        os._exit(3)  # the failed rank leaves without tearing down the group, like a crash
    except Exception as ex:  # peers: gloo reports the lost rank or times out
        q.put((rank, "error", type(ex).__name__))
        q.close()
        q.join_thread()
        os._exit(4)


def test_gloo_injected_comm_fault_fails_every_rank(tmp_path):
    """a rank whose collective fails (WC_COMM_FAULT=1:2 — rank 1, 2nd
    collective of the merge) ends the job on EVERY rank with an error within the
    collective timeout; nobody hangs and nobody reports a (wrong) result."""
    from cuda_mapreduce_amd.ops import synth_host

    p = tmp_path / "in.txt"
    p.write_bytes(synth_host(50_000, seed=2, vocab=500))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fault_worker, args=(r, 2, port, str(p), q)) for r in range(2)]
    for pr in procs:
        pr.start()
    outs = dict((r, (kind, msg)) for r, kind, msg in (q.get(timeout=90) for _ in range(2)))
    for pr in procs:
        pr.join(timeout=30)
    assert outs[1][0] == "fault" and "injected comm fault" in outs[1][1]
    assert outs[0][0] == "error"
    assert [pr.exitcode for pr in procs] == [4, 3]


def test_owner_rule_matches_native():
    """dist._owner (Python) == wc_key_owner (keys.hpp owner_of of place_hash), for
    SHORT, MEDIUM and LONG words and several world sizes."""
    import ctypes
    import random

    from cuda_mapreduce_amd.ops import _lib
    from cuda_mapreduce_amd.parallel import dist

    lib = _lib.lib
    rng = random.Random(7)
    words = [b"a", b"Hello", b"12345678", b"123456789", b"fifteen-bytes!!", b"sixteen-bytes!!!",
             b"x" * 64, b"tab\there", b"nul\0byte", b"\xff" * 23]
    words += [bytes(rng.randrange(1, 256) for _ in range(rng.randrange(1, 80))) for _ in range(400)]
    for w in words:
        buf = (ctypes.c_uint8 * len(w)).from_buffer_copy(w)
        for world in (1, 2, 3, 8, 64):
            assert dist._owner(w, world) == lib.wc_key_owner(buf, len(w), world), (w, world)
