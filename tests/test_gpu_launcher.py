"""bench.py under torch.distributed.run (one process per GPU, the driver's N>1
launch form) at --nproc-per-node 1 with the native RCCL communicator forced on
(WC_MERGE_ALWAYS=1): rendezvous, unique-id broadcast, Comm creation and both
merge protocols run end to end and the bench's key-for-key validation passes."""
import json
import os
import random
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.parametrize("merge", ["shuffle", "dense"])
def test_torchrun_world1_rccl_merge(merge):
    env = dict(os.environ, WC_MERGE_ALWAYS="1", MASTER_ADDR="127.0.0.1")
    port = 29500 + random.randint(100, 900)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--steps", "2", "--warmup", "1", "--gb-per-gpu", "0.125", "--merge", merge]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [l for l in p.stdout.splitlines() if l.startswith("{")][-1]
    d = json.loads(line)
    assert d["validated"] is True
    assert d["config"]["merge"] == merge
    assert d["n_gpus"] == 1 and d["distinct_words"] > 0


@pytest.mark.gpu
def test_bench_self_launch_refuses_missing_gpus():
    # `bench.py --gpus N` launches N ranks itself; with fewer GPUs visible it must
    # fail at once, before any rank starts
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    from cuda_mapreduce_amd.parallel.launch import visible_gpus

    n = visible_gpus()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n + 1), "--steps", "1"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=60)
    assert p.returncode == 2
    assert f"{n + 1} GPUs requested, {n} visible" in p.stderr


@pytest.mark.gpu
def test_bench_one_runtime_per_rank():
    # the rank loads only /opt/rocm's HIP runtime and RCCL (no torch, no second copy)
    env = dict(os.environ, WC_MERGE_ALWAYS="1")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "2", "--warmup", "1",
                        "--gb-per-gpu", "0.125"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    rt = d["runtime"]
    assert rt["torch"] is False
    assert len(rt["hip"]) == 1 and rt["hip"][0].startswith("/opt/rocm"), rt
    assert len(rt["rccl"]) == 1 and rt["rccl"][0].startswith("/opt/rocm"), rt
    assert d["validated"] is True and d["control_plane"].startswith("native RCCL")
