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


_DUP_RANK = r"""
import os, sys
sys.path.insert(0, os.environ["WC_ROOT"])
from cuda_mapreduce_amd.ops import Comm
from cuda_mapreduce_amd.parallel import launch as L
rank = int(os.environ["RANK"])
uid = L.rendezvous_uid(rank, Comm.unique_id, timeout_s=60)
try:
    c = Comm(uid, rank, 2, 0)
except Exception as e:
    print("REFUSED", e, flush=True)
    sys.exit(3)
print("ACCEPTED", flush=True)
c.close()
"""


@pytest.mark.gpu
def test_rccl_two_ranks_on_one_gpu_refused(tmp_path):
    """SURVEY §4.3 item 6 / VERDICT r5 item 3: two RCCL ranks on ONE GPU.  RCCL
    2.27 refuses them at ncclCommInitRank ("Duplicate GPU detected",
    ncclInvalidUsage; profiles/r6_rccl_one_gpu.md): both ranks fail at once
    with the engine's one-rank-per-GPU message, nothing hangs."""
    port = str(29500 + random.randint(100, 900))
    procs = []
    for r in (0, 1):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK="0", WORLD_SIZE="2", LOCAL_WORLD_SIZE="2",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port, WC_RDZV_DIR=str(tmp_path), WC_ROOT=ROOT,
                   WC_COMM_TIMEOUT_S="60", HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, "-c", _DUP_RANK], cwd=ROOT, env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=100) for p in procs]
    for p, (out, err) in zip(procs, outs):
        assert p.returncode == 3, (out[-2000:], err[-2000:])
        assert "REFUSED" in out and "one rank per GPU" in out, out[-2000:]


@pytest.mark.gpu
def test_bench_refuses_more_local_ranks_than_gpus():
    # the same refusal before any rendezvous when the rank's own view shows it
    from cuda_mapreduce_amd.parallel.launch import visible_gpus

    n = visible_gpus()
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE=str(n + 1), LOCAL_WORLD_SIZE=str(n + 1),
               MASTER_ADDR="127.0.0.1", MASTER_PORT="29999")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n + 1), "--steps", "1"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=60)
    assert p.returncode == 2
    assert "one rank per GPU" in p.stderr
