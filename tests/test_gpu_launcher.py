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
