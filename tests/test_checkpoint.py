"""Checkpoint / resume (the reference has none — main.cu:133-162 is
one in-memory pass).  The CLI counts FILE in delimiter-aligned intervals and
saves the running table + next byte offset after each; WC_CKPT_STOP_AFTER=N
simulates a crash after the N-th checkpoint.  Resumed output must be
byte-identical to an uninterrupted run."""
import os
import random
import struct
import subprocess

import pytest

from conftest import ROOT

EXE = os.path.join(ROOT, "wordcount")


def make_text(path, n=40000, seed=3, long_every=0):
    rng = random.Random(seed)
    parts = []
    for i in range(n):
        w = "w%d" % rng.randint(0, 400)
        if long_every and i % long_every == 0:
            w = "L" * rng.randint(300, 3000)  # longer than the interval
        parts.append(w)
        parts.append(rng.choice([" ", " ", "\n", "\r\n", "  "]))
    data = "".join(parts).encode()
    path.write_bytes(data)
    return data


def run(args, cwd, env_extra=None):
    env = dict(os.environ)
    env.pop("WC_CKPT_STOP_AFTER", None)
    env.update(env_extra or {})
    return subprocess.run([EXE] + args, cwd=cwd, env=env, capture_output=True, timeout=120)


def crash_then_resume(tmp_path, mode, every, stops, every_resume=None):
    """Uninterrupted output vs. a run stopped after `stops` checkpoints then resumed."""
    base = run(["t.txt", "--no-echo"] + mode, tmp_path)
    assert base.returncode == 0, base.stderr
    ck = ["--checkpoint", "ck.bin", "--checkpoint-every", str(every)]
    crashed = run(["t.txt", "--no-echo"] + mode + ck, tmp_path, {"WC_CKPT_STOP_AFTER": str(stops)})
    assert crashed.returncode == 1 and b"stopped after" in crashed.stderr
    ck2 = ["--checkpoint", "ck.bin", "--checkpoint-every", str(every_resume or every), "--resume"]
    resumed = run(["t.txt", "--no-echo"] + mode + ck2, tmp_path)
    assert resumed.returncode == 0, resumed.stderr
    assert b"resumes at byte" in resumed.stderr
    assert resumed.stdout == base.stdout
    return base.stdout


@pytest.mark.parametrize("every,stops,every_resume", [(5000, 1, None), (7001, 9, 13000), (65536, 2, 1000)])
def test_cpu_crash_resume_identical(tmp_path, every, stops, every_resume):
    make_text(tmp_path / "t.txt")
    crash_then_resume(tmp_path, ["--cpu"], every, stops, every_resume)


def test_cpu_checkpointed_equals_plain_with_long_words(tmp_path):
    # words longer than the interval widen the read instead of being split
    make_text(tmp_path / "t.txt", n=5000, long_every=97)
    a = run(["t.txt", "--no-echo", "--cpu"], tmp_path)
    b = run(["t.txt", "--no-echo", "--cpu", "--checkpoint", "c", "--checkpoint-every", "256"], tmp_path)
    assert a.returncode == 0 and b.returncode == 0 and a.stdout == b.stdout


def test_checkpoint_golden_with_echo(tmp_path, golden_text):
    (tmp_path / "test.txt").write_bytes(golden_text)
    a = run(["--cpu"], tmp_path)
    b = run(["--cpu", "--checkpoint", "c", "--checkpoint-every", "5"], tmp_path)
    assert b.returncode == 0 and a.stdout == b.stdout


def test_corrupt_and_foreign_checkpoints_are_refused(tmp_path):
    make_text(tmp_path / "t.txt", n=3000)
    ck = ["--cpu", "--no-echo", "--checkpoint", "ck.bin", "--checkpoint-every", "4000"]
    assert run(["t.txt"] + ck, tmp_path, {"WC_CKPT_STOP_AFTER": "1"}).returncode == 1
    raw = bytearray((tmp_path / "ck.bin").read_bytes())
    assert raw[:8] == b"WCCKPT01"
    raw[40] ^= 1
    (tmp_path / "ck.bin").write_bytes(bytes(raw))
    bad = run(["t.txt", "--resume"] + ck, tmp_path)
    assert bad.returncode == 1 and b"checksum" in bad.stderr
    # a valid checkpoint of another input is refused
    assert run(["t.txt"] + ck, tmp_path, {"WC_CKPT_STOP_AFTER": "1"}).returncode == 1
    (tmp_path / "t.txt").write_bytes((tmp_path / "t.txt").read_bytes() + b"extra ")
    other = run(["t.txt", "--resume"] + ck, tmp_path)
    assert other.returncode == 1 and b"another input" in other.stderr


def test_checkpoint_layout(tmp_path):
    data = make_text(tmp_path / "t.txt", n=2000)
    r = run(["t.txt", "--cpu", "--no-echo", "--checkpoint", "ck.bin", "--checkpoint-every", "100M"], tmp_path)
    assert r.returncode == 0
    raw = (tmp_path / "ck.bin").read_bytes()
    ver, rank, world, intervals = struct.unpack_from("<4I", raw, 8)
    size, begin, end, nxt, fp, total, rows = struct.unpack_from("<7Q", raw, 24)
    assert (ver, rank, world, intervals) == (2, 0, 1, 1)
    assert (size, begin, end, nxt) == (len(data), 0, len(data), len(data))
    assert fp != 0  # prefix fingerprint of the counted bytes
    assert total == len(data.split()) and rows == len(set(data.split()))
    assert not os.path.exists(tmp_path / "ck.bin.tmp")


def test_resume_without_checkpoint_path_is_an_error(tmp_path):
    r = run(["--cpu", "--resume"], tmp_path)
    assert r.returncode == 1 and b"--resume needs" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("every,stops", [(6000, 3), (100000, 1)])
def test_gpu_crash_resume_identical(tmp_path, every, stops):
    make_text(tmp_path / "t.txt", n=60000)
    out = crash_then_resume(tmp_path, [], every, stops)
    cpu = run(["t.txt", "--no-echo", "--cpu"], tmp_path)
    assert out == cpu.stdout  # GPU checkpointed run == CPU oracle


@pytest.mark.gpu
def test_gpu_resume_from_cpu_checkpoint(tmp_path):
    # the file format is engine-independent: a CPU-written checkpoint resumes on the GPU
    make_text(tmp_path / "t.txt", n=30000)
    ck = ["--checkpoint", "ck.bin", "--checkpoint-every", "9000"]
    assert run(["t.txt", "--no-echo", "--cpu"] + ck, tmp_path, {"WC_CKPT_STOP_AFTER": "4"}).returncode == 1
    g = run(["t.txt", "--no-echo", "--resume"] + ck, tmp_path)
    assert g.returncode == 0, g.stderr
    assert g.stdout == run(["t.txt", "--no-echo", "--cpu"], tmp_path).stdout


@pytest.mark.gpu
def test_gpu_bench_json_stages(tmp_path):
    import json

    data = make_text(tmp_path / "t.txt", n=20000)
    r = run(["t.txt", "--no-echo", "--no-list", "--bench-json", "b.json"], tmp_path, {"WC_LOG": "debug"})
    assert r.returncode == 0, r.stderr
    d = json.loads((tmp_path / "b.json").read_text())
    assert d["path"] == "gpu" and d["tokens"] == len(data.split()) and d["chunks"] >= 1
    assert d["device_ms"]["map"] > 0 and d["device_ms"]["reduce"] > 0 and d["device_ms"]["finalize"] > 0
    assert b"[wc debug" in r.stderr and b"finalize" in r.stderr


def test_python_cpu_checkpointed_api(tmp_path):
    ops = pytest.importorskip("cuda_mapreduce_amd.ops")
    data = make_text(tmp_path / "t.txt", n=20000)
    want = ops.cpu_count(data)
    ck = str(tmp_path / "py.ck")
    got = ops.cpu_count_file_checkpointed(str(tmp_path / "t.txt"), ck, interval=3000)
    assert got.words == want.words and list(got.counts) == list(want.counts) and got.total == want.total
    assert list(got.first_off) == list(want.first_off)
    # a finished checkpoint resumes to the same table without reading anything
    again = ops.cpu_count_file_checkpointed(str(tmp_path / "t.txt"), ck, interval=3000, resume=True)
    assert again.words == want.words and list(again.counts) == list(want.counts)
    with pytest.raises(ops.WcError):
        ops.cpu_count_file_checkpointed(str(tmp_path / "t.txt"), ck, interval=3000, begin=5)


@pytest.mark.gpu
def test_python_gpu_checkpointed_api(tmp_path):
    ops = pytest.importorskip("cuda_mapreduce_amd.ops")
    data = make_text(tmp_path / "t.txt", n=50000)
    want = ops.cpu_count(data)
    with ops.Engine(device=0) as eng:
        got = eng.count_file_checkpointed(str(tmp_path / "t.txt"), str(tmp_path / "g.ck"), interval=40000)
        assert got.words == want.words and list(got.counts) == list(want.counts)
        assert list(got.first_off) == list(want.first_off) and got.total == want.total
        # the engine is reusable afterwards
        eng.count_bytes(data)
        assert eng.result().words == want.words


@pytest.mark.gpu
def test_gpu_checkpointed_long_words(tmp_path):
    # words longer than the interval (and than the map's short-key window) on the GPU path
    make_text(tmp_path / "t.txt", n=6000, long_every=53)
    a = run(["t.txt", "--no-echo", "--cpu"], tmp_path)
    b = run(["t.txt", "--no-echo", "--checkpoint", "c", "--checkpoint-every", "4096"], tmp_path)
    assert b.returncode == 0, b.stderr
    assert a.stdout == b.stdout


def test_resume_refuses_input_modified_in_place(tmp_path):
    """Same size, different bytes in the already-counted prefix: the checkpoint's
    prefix fingerprint no longer matches, so --resume refuses instead of mixing
    stale and new counts."""
    data = make_text(tmp_path / "t.txt", n=6000)
    ck = ["--cpu", "--no-echo", "--checkpoint", "ck.bin", "--checkpoint-every", "4000"]
    assert run(["t.txt"] + ck, tmp_path, {"WC_CKPT_STOP_AFTER": "2"}).returncode == 1
    # flip one word near the start (same length, delimiters untouched)
    i = data.index(b"w")
    mod = bytearray(data)
    mod[i] = ord(b"x")
    (tmp_path / "t.txt").write_bytes(bytes(mod))
    r = run(["t.txt"] + ck + ["--resume"], tmp_path)
    assert r.returncode != 0 and b"changed since it was written" in r.stderr
    # the untouched file resumes fine
    (tmp_path / "t.txt").write_bytes(data)
    r = run(["t.txt"] + ck + ["--resume"], tmp_path)
    assert r.returncode == 0 and b"resumes at byte" in r.stderr
