"""Multi-process data-parallel word count on CPU (gloo, world_size 2 and 3):
shard ownership + the merge protocol (reduce-scatter / all-gather) must give
exactly the single-process result."""
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


def _worker(rank, world, port, path, q):
    sys.path.insert(0, ROOT)
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from cuda_mapreduce_amd.parallel import DistributedWordCount, init_from_env

    env = init_from_env("gloo")
    job = DistributedWordCount(env, use_gpu=False)
    res = job.count_file(path)
    q.put((rank, res.words, [int(c) for c in res.counts], [int(f) for f in res.first_off], res.total))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_data_parallel_matches_single(tmp_path, world):
    from cuda_mapreduce_amd.ops import cpu_count, synth_host

    text = synth_host(300_000, seed=5, vocab=4000) + b"tail-without-newline"
    p = tmp_path / "in.txt"
    p.write_bytes(text)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, str(p), q)) for r in range(world)]
    for pr in procs:
        pr.start()
    outs = [q.get(timeout=120) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    want = cpu_count(text)
    for rank, words, counts, first, total in outs:
        assert total == want.total
        assert words == want.words
        assert counts == [int(c) for c in want.counts]
        assert first == [int(f) for f in want.first_off]
