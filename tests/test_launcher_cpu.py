"""bench.py's own N-rank launcher and the torch-free rendezvous (CPU, no GPU).

`python bench.py --gpus N` without WORLD_SIZE starts N fresh rank processes
(cuda_mapreduce_amd/parallel/launch.py); `--dry-launch` ranks only report their
environment, so the launch contract, fail-fast and the visibility check are
testable here.  WC_FAKE_VISIBLE_GPUS stands in for the KFD GPU count."""
import json
import os
import subprocess
import sys
import threading
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT", "WC_RDZV_DIR")}
    env.update({k: str(v) for k, v in kw.items()})
    return env


def _run(args, timeout=60, **env):
    return subprocess.run([sys.executable, BENCH] + args, cwd=ROOT, env=_env(**env), capture_output=True, text=True,
                          timeout=timeout)


def test_dry_launch_three_ranks():
    p = _run(["--gpus", "3", "--dry-launch"], WC_FAKE_VISIBLE_GPUS=3)
    assert p.returncode == 0, p.stderr
    lines = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    assert sorted(d["dry_rank"] for d in lines) == [0, 1, 2]
    ports = {d["env"]["MASTER_PORT"] for d in lines}
    dirs = {d["env"]["WC_RDZV_DIR"] for d in lines}
    assert len(ports) == 1 and len(dirs) == 1  # one job: one rendezvous
    for d in lines:
        e = d["env"]
        assert e["RANK"] == e["LOCAL_RANK"] == str(d["dry_rank"])
        assert e["WORLD_SIZE"] == e["LOCAL_WORLD_SIZE"] == "3"
        assert e["MASTER_ADDR"] == "127.0.0.1"
        assert e["WC_COMM_TIMEOUT_S"] == "120"
        assert e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
        assert d["torch_loaded"] is False
    assert not os.path.exists(dirs.pop())  # rendezvous directory removed at the end


def test_fail_fast_propagates_rank_code():
    # rank 1 fails, rank 2 would hang for 10 minutes: the launcher stops it and returns rank 1's code
    t0 = time.time()
    p = _run(["--gpus", "3", "--dry-launch"], timeout=60, WC_FAKE_VISIBLE_GPUS=3, WC_DRY_FAIL_RANK=1,
             WC_DRY_HANG_RANK=2)
    assert p.returncode == 3, (p.returncode, p.stderr)
    assert "rank 1 exited with 3" in p.stderr
    assert time.time() - t0 < 30


def test_too_few_gpus_fails_at_once():
    t0 = time.time()
    p = _run(["--gpus", "2", "--steps", "1"], WC_FAKE_VISIBLE_GPUS=1)
    assert p.returncode == 2
    assert "2 GPUs requested, 1 visible" in p.stderr
    assert time.time() - t0 < 30


def test_visible_gpus_masks(tmp_path):
    from cuda_mapreduce_amd.parallel import launch as L

    nodes = tmp_path / "nodes"
    for i, simd in enumerate([0, 256, 256, 256]):  # one CPU node + three GPU nodes
        d = nodes / str(i)
        d.mkdir(parents=True)
        (d / "properties").write_text(f"cpu_cores_count 8\nsimd_count {simd}\n")
    assert L.kfd_gpu_nodes(str(nodes)) == 3
    assert L.visible_gpus({"WC_FAKE_VISIBLE_GPUS": "8", "HIP_VISIBLE_DEVICES": "0"}) == 8
    n = L.kfd_gpu_nodes()
    assert L.visible_gpus({}) == n
    assert L.visible_gpus({"HIP_VISIBLE_DEVICES": ""}) == 0
    assert L.visible_gpus({"ROCR_VISIBLE_DEVICES": "0,1"}) == min(n, 2)


def test_file_rendezvous(tmp_path, monkeypatch):
    from cuda_mapreduce_amd.parallel import launch as L

    monkeypatch.setenv("WC_RDZV_DIR", str(tmp_path))
    uid = bytes(range(128))
    got = {}

    def peer(r):
        got[r] = L.rendezvous_uid(r, lambda: b"x" * 128, timeout_s=10)

    th = [threading.Thread(target=peer, args=(r,)) for r in (1, 2)]
    for t in th:
        t.start()
    time.sleep(0.1)
    assert L.rendezvous_uid(0, lambda: uid) == uid
    for t in th:
        t.join(10)
    assert got == {1: uid, 2: uid}
    L.rendezvous_cleanup()
    assert not os.path.exists(tmp_path / "rccl_uid")
    with pytest.raises(TimeoutError):
        L.rendezvous_uid(1, lambda: uid, timeout_s=0.2)


def test_rendezvous_ignores_stale_id_and_refuses_multinode(tmp_path, monkeypatch):
    """Under torch.distributed.run (no WC_RDZV_DIR): the directory is keyed on the
    job (TORCHELASTIC_RUN_ID, else the agent pid) and the port; an id file older
    than the agent (a crashed earlier job's) is ignored; a multi-node world is
    refused (the file rendezvous is node-local)."""
    from cuda_mapreduce_amd.parallel import launch as L

    monkeypatch.delenv("WC_RDZV_DIR", raising=False)
    monkeypatch.setattr(L.tempfile, "gettempdir", lambda: str(tmp_path))
    monkeypatch.setenv("MASTER_PORT", "29999")
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "job42")
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "2")
    d = L.rdzv_dir()
    assert os.path.basename(d) == "wc_rdzv_job42_29999"
    stale = os.path.join(d, "rccl_uid")
    with open(stale, "wb") as f:
        f.write(b"s" * 128)
    os.utime(stale, (1, 1))  # written long before this process's parent started
    with pytest.raises(TimeoutError):
        L.rendezvous_uid(1, lambda: b"x" * 128, timeout_s=0.2)
    fresh = bytes(range(128))
    assert L.rendezvous_uid(0, lambda: fresh) == fresh
    assert L.rendezvous_uid(1, lambda: b"x" * 128, timeout_s=2) == fresh
    monkeypatch.setenv("WORLD_SIZE", "16")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    with pytest.raises(RuntimeError, match="single-node"):
        L.rdzv_dir()


def test_launcher_imports_no_engine():
    # the launcher half of bench.py must not load libwc.so (no HIP runtime in the parent)
    code = ("import sys; sys.path.insert(0, %r); import bench; a = bench.parse(['--gpus', '2']);"
            "from cuda_mapreduce_amd.parallel import launch;"
            "print('libwc' in open('/proc/self/maps').read(), 'torch' in sys.modules)") % ROOT
    p = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    assert p.stdout.split() == ["False", "False"]
