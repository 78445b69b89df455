"""GPU numerics tests of the native engine against the CPU oracle (exact equality).

Every case compares words, first-occurrence order, counts and total with
``cpu_count`` (a byte-keyed hash map), so the GPU's packed-key scheme, the LDS
combiner, the shuffle partitioning, the running table, its splits and the
merge are all checked end to end.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLDEN_OUTPUT, ROOT

pytestmark = pytest.mark.gpu

ops = pytest.importorskip("cuda_mapreduce_amd.ops")


def assert_same(got, want):
    assert got.total == want.total
    assert len(got) == len(want)
    assert got.words == want.words
    assert np.array_equal(got.counts, want.counts)
    assert np.array_equal(got.first_off, want.first_off)


@pytest.fixture(scope="module")
def eng():
    e = ops.Engine(device=0, chunk_bytes=1 << 22)
    yield e
    e.close()


def run(eng, text):
    eng.reset()
    eng.count_bytes(text)
    return eng.result()


def random_text(rng, n, alphabet=b"abcd ,\n\r\tXY", long_words=0):
    a = np.frombuffer(alphabet, np.uint8)
    buf = a[rng.integers(0, len(a), n)].copy()
    for _ in range(long_words):  # plant words longer than lanes / halo / tiles
        L = int(rng.choice([9, 31, 33, 255, 257, 4000, 20000]))
        if n > L + 2:
            p = int(rng.integers(0, n - L))
            buf[p : p + L] = np.frombuffer(b"q", np.uint8)[0]
            buf[p + L - 1] = ord("z")
    return buf.tobytes()


def test_golden(eng, golden_text):
    res = run(eng, golden_text)
    assert ops.format_output(res, echo=golden_text) == GOLDEN_OUTPUT


def test_empty_and_delims(eng):
    for t in [b"", b" ", b"\n\n\r  \n", b"a", b"a ", b" a", b"\r\na\r\n"]:
        assert_same(run(eng, t), ops.cpu_count(t))


@pytest.mark.parametrize("seed", range(12))
def test_random_vs_oracle(eng, seed):
    rng = np.random.default_rng(seed)
    n = int(rng.choice([1, 17, 1000, 16383, 16384, 16385, 70000, 300000, 2_000_000]))
    text = random_text(rng, n, long_words=3)
    assert_same(run(eng, text), ops.cpu_count(text))


def test_chunk_and_tile_boundaries():
    # 32 KiB chunks: words straddle lanes (32 B), tiles (16 KiB), halo and chunks
    rng = np.random.default_rng(5)
    text = random_text(rng, 1_000_003, alphabet=b"abcdefgh   \n", long_words=20)
    with ops.Engine(device=0, chunk_bytes=1 << 15) as e:
        e.count_bytes(text)
        got = e.result()
    assert_same(got, ops.cpu_count(text))


def test_synthetic_device_matches_host():
    n = 8 << 20
    with ops.Engine(device=0, chunk_bytes=1 << 22) as e:
        e.synth_device(n, first_segment=3, seed=11, vocab=20000)
        e.count_resident(n, global_base=0)
        got = e.result()
    assert_same(got, ops.cpu_count(ops.synth_host(n, first_segment=3, seed=11, vocab=20000)))


def test_job_resident_one_call():
    """wc_job_resident (reset + count + finalize in one call, the bench's step)
    leaves the same ordered table as the three calls, job after job."""
    n = 8 << 20
    want = ops.cpu_count(ops.synth_host(n, first_segment=2, seed=5, vocab=30000))
    with ops.Engine(device=0) as e:
        e.synth_device(n, first_segment=2, seed=5, vocab=30000)
        for _ in range(3):
            assert e.job_resident(n) == len(want)
            assert_same(e.result(), want)


def test_table_split_large_vocab():
    # 2 buckets x 4096 slots to start; ~60k distinct words force several splits
    words = [f"w{i:x}".encode() for i in range(60000)]
    rng = np.random.default_rng(3)
    text = b" ".join(words[i] for i in rng.integers(0, len(words), 300000)) + b"\n"
    with ops.Engine(device=0, chunk_bytes=1 << 20, log2_rec_buckets=1, log2_tab_buckets=1) as e:
        e.count_bytes(text)
        got = e.result()
        st = e.stats()
    assert st["table_splits"] >= 3
    assert_same(got, ops.cpu_count(text))


def test_combiner_flat_vocabulary():
    """A near-flat 1M-word vocabulary over 96 MiB: the map blocks' read-only hot
    tables (the sampled HOT_K most frequent candidates, map.hip wc_map) cover
    few tokens, so most tokens become shuffle records (> half of them here) and
    the reduce merges them; counts and first occurrences must stay exact."""
    text = ops.synth_host(96 << 20, seed=21, vocab=1000000, zipf_s=0.4)
    with ops.Engine(device=0) as e:
        e.count_bytes(text)
        got = e.result()
        st = e.stats()
    assert st["records"] > st["tokens"] // 2  # mostly direct records
    assert_same(got, ops.cpu_count(text))


def test_combiner_vocabulary_drift():
    """The frequent keys change every 32 KiB (alternate pieces are upper-cased),
    so a map block's hot table, sampled once per job from a few units of its
    range, holds words of both halves and misses the rest: hits and records of
    the same word mix in every block — counts and first occurrences must stay
    exact."""
    half = ops.synth_host(48 << 20, seed=5, vocab=20000)
    upper = bytes.maketrans(b"abcdefghijklmnopqrstuvwxyz", b"ABCDEFGHIJKLMNOPQRSTUVWXYZ")
    n = len(half) // 2
    # alternate 32 KiB pieces (whole 1 KiB synthetic segments, which end in a
    # delimiter) so every map block's ~190 KiB share switches hot sets
    piece = 32 << 10
    text = b"".join(half[i:i + piece] + half[i:i + piece].translate(upper) for i in range(0, n, piece))
    with ops.Engine(device=0) as e:
        e.count_bytes(text)
        got = e.result()
    assert_same(got, ops.cpu_count(text))


def test_region_overflow_reruns():
    rng = np.random.default_rng(9)
    text = b" ".join(f"k{i}".encode() for i in rng.integers(0, 200000, 200000))
    with ops.Engine(device=0, chunk_bytes=1 << 20, min_records=16384, records_per_byte=0.001) as e:
        e.count_bytes(text)
        got = e.result()
        st = e.stats()
    assert st["map_reruns"] >= 1
    assert_same(got, ops.cpu_count(text))


@pytest.mark.parametrize("root_rows", [None, "0", "1000000000"])
@pytest.mark.parametrize("merge_mode", [0, 1])
@pytest.mark.parametrize("ranks", [1, 2, 3, 4, 8])
def test_loopback_merge(ranks, merge_mode, root_rows, monkeypatch):
    """Sharding + cross-rank merge at N virtual ranks: shuffle (all-to-all by key
    owner, gather to rank 0, broadcast with all_ranks; with WC_MERGE_ROOT_ROWS
    set and fewer total rows, every rank sends straight to rank 0 instead — by
    default the exact merge takes the owner path, which learns the planned
    merge's caps) and dense (dictionary union + reduce-scatter + all-gather)
    protocols."""
    if root_rows is not None:
        monkeypatch.setenv("WC_MERGE_ROOT_ROWS", root_rows)  # 0: always the owner exchange
    rng = np.random.default_rng(ranks)
    text = random_text(rng, 400_000, alphabet=b"abcdefg  \n", long_words=4) + ops.synth_host(1 << 20, seed=2, vocab=3000)
    for all_ranks in (False, True):
        got = ops.loopback_count(text, ranks, chunk_bytes=1 << 20, merge_mode=merge_mode, all_ranks=all_ranks)
        assert_same(got, ops.cpu_count(text))


def test_loopback_stream_ordered():
    """The loopback communicator only enqueues, as RCCL does: with rank 1's
    stream held, both ranks' allgather calls return on the host, rank 0's
    stream stays busy until rank 1's stream reaches the collective, and the
    gathered data is right once it is released (src/dist/comm.cpp LoopbackComm)."""
    import ctypes

    from cuda_mapreduce_amd.ops import _lib

    ret, pend, ok = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_int(0)
    _lib.check(_lib.lib.wc_debug_loopback_async(0, ctypes.byref(ret), ctypes.byref(pend), ctypes.byref(ok)))
    assert ret.value == 1, "a collective call waited on the host for a peer's stream"
    assert pend.value == 1, "rank 0's collective completed before rank 1's stream reached it"
    assert ok.value == 1


@pytest.mark.parametrize("merge_mode", [0, 1])
@pytest.mark.parametrize("ranks", [1, 3, 8])
def test_planned_merge_virtual_ranks(ranks, merge_mode):
    """The planned merge (fixed exchange regions learned from the first exact
    merge, no host round trip; dist/merge.cpp merge_cols_planned) at W virtual
    ranks: every job after the first runs planned, and the validated job's
    table equals the oracle of the whole stream (WC_MERGE_ALWAYS covers W = 1
    in a child process)."""
    per = 6 << 20
    code = (
        "import sys\n"
        "from cuda_mapreduce_amd import ops\n"
        f"res, rk = ops.virtual_bench({ranks}, {per}, seed=5, vocab=30000, steps=3, warmup=1, "
        f"chunk_bytes=2 << 20, merge_mode={merge_mode})\n"
        f"want = ops.cpu_count_synth({ranks} * {per}, 0, seed=5, vocab=30000)\n"
        "assert res.words == want.words and res.counts.tolist() == want.counts.tolist(), 'table'\n"
        "assert res.first_off.tolist() == want.first_off.tolist(), 'first offsets'\n"
        "assert rk[0]['merges_planned'] >= 4 and rk[0]['merge_redos'] == 0, rk[0]\n"
        "print('ok')\n"
    )
    env = dict(os.environ, WC_MERGE_ALWAYS="1")
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, timeout=120)
    assert out.returncode == 0 and b"ok" in out.stdout, out.stderr.decode()[-2000:]


@pytest.mark.parametrize("merge_mode", [0, 1])
def test_planned_merge_larger_job_redoes_on_every_rank(merge_mode):
    """A job larger than the one the planned merge learned its caps from
    (WC_VB_GROW_SEGS: the last rank's validation job counts 2 MiB more): its
    max first offset passes the caps' global max end.  Every rank checks the
    gathered offsets against that SAME bound (dist/merge.cpp key_bound), so all
    of them redo exactly together — before, ranks whose own max end was lower
    redid alone and waited in collectives the last rank never joined."""
    per, grow = 4 << 20, 2048
    code = (
        "from cuda_mapreduce_amd import ops\n"
        f"res, rk = ops.virtual_bench(3, {per}, seed=8, vocab=20000, steps=2, warmup=1, chunk_bytes=2 << 20, "
        f"merge_mode={merge_mode})\n"
        f"want = ops.cpu_count_synth(3 * {per} + {grow} * 1024, 0, seed=8, vocab=20000)\n"
        "assert res.words == want.words and res.counts.tolist() == want.counts.tolist(), 'table'\n"
        "assert res.first_off.tolist() == want.first_off.tolist(), 'first offsets'\n"
        "assert rk[0]['merge_redos'] >= 1, rk[0]\n"
        "print('ok')\n"
    )
    env = dict(os.environ, WC_VB_GROW_SEGS=str(grow), WC_COMM_TIMEOUT_S="20")
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, timeout=110)
    assert out.returncode == 0 and b"ok" in out.stdout, out.stderr.decode()[-2000:]


@pytest.mark.parametrize("resident", [True, False])
def test_loopback_count_mismatch_fails_every_rank(resident):
    """A rank whose compacted key count disagrees with its owner-count sum
    (injected: WC_MERGE_FAULT_COUNT=1 biases rank 1's count word) is seen by
    EVERY rank in the gathered plan matrix, so all of them fail at once — the
    speculative finalize used to throw on that rank alone while the peers
    entered the merge's collectives and waited for the watchdog."""
    code = (
        "import time\n"
        "from cuda_mapreduce_amd import ops\n"
        "text = ops.synth_host(3 << 20, seed=4, vocab=20000)\n"
        "t0 = time.time()\n"
        "try:\n"
        f"    ops.loopback_count(text, 3, chunk_bytes=1 << 20, resident={resident})\n"
        "    print('no error')\n"
        "except RuntimeError as ex:\n"
        "    print('failed', round(time.time() - t0, 2), str(ex)[:200])\n"
    )
    env = dict(os.environ, WC_MERGE_FAULT_COUNT="1", WC_COMM_TIMEOUT_S="60")
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, timeout=100)
    line = out.stdout.decode().strip().splitlines()[-1] if out.stdout.strip() else out.stderr.decode()[-1500:]
    assert line.startswith("failed"), line
    assert "key count" in line, line
    assert float(line.split()[1]) < 5.0, line


@pytest.mark.parametrize("merge_mode", [0, 1])
def test_planned_merge_overflow_redo(merge_mode):
    """Fixed regions too small (WC_MERGE_CAP_ROWS=64, a test switch): every
    planned merge overflows, all ranks see it in the gathered words and redo
    the merge exactly — the result stays exact."""
    per = 4 << 20
    code = (
        "from cuda_mapreduce_amd import ops\n"
        f"res, rk = ops.virtual_bench(4, {per}, seed=6, vocab=20000, steps=2, warmup=1, chunk_bytes=2 << 20, "
        f"merge_mode={merge_mode})\n"
        f"want = ops.cpu_count_synth(4 * {per}, 0, seed=6, vocab=20000)\n"
        "assert res.words == want.words and res.counts.tolist() == want.counts.tolist(), 'table'\n"
        "assert res.first_off.tolist() == want.first_off.tolist(), 'first offsets'\n"
        "assert rk[0]['merge_redos'] >= 3, rk[0]\n"
        "print('ok')\n"
    )
    env = dict(os.environ, WC_MERGE_CAP_ROWS="64")
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, timeout=120)
    assert out.returncode == 0 and b"ok" in out.stdout, out.stderr.decode()[-2000:]


def test_loopback_merge_host_waits():
    """A merge's host waits do not grow with its collectives: every collective
    of the stream-ordered loopback is enqueue-only, the merge waits only where
    the protocol needs host values (owner plan, merged counts, the result)."""
    import ctypes

    from cuda_mapreduce_amd.ops import _lib

    def counters():
        c, w = ctypes.c_uint64(0), ctypes.c_uint64(0)
        _lib.lib.wc_debug_comm_counters(ctypes.byref(c), ctypes.byref(w))
        return c.value, w.value

    text = ops.synth_host(2 << 20, seed=9, vocab=20000)
    want = ops.cpu_count(text)
    for merge_mode in (0, 1):
        c0, w0 = counters()
        assert_same(ops.loopback_count(text, 4, chunk_bytes=1 << 20, merge_mode=merge_mode, all_ranks=True), want)
        c1, w1 = counters()
        assert c1 - c0 >= 4 * 6, (c1 - c0)  # >= 6 collectives per rank (owner exchange + gather + broadcast)
        assert (w1 - w0) <= 4 * 4, (w1 - w0)  # <= 4 host waits per rank


@pytest.mark.parametrize("merge_mode", [0, 1])
@pytest.mark.parametrize("ranks", [2, 5, 8])
def test_loopback_merge_many_long_words(ranks, merge_mode):
    """Both merges with many >8-byte words (owner byte payloads, arena offsets,
    dense ids returned to the senders)."""
    rng = np.random.default_rng(40 + ranks)
    words = [bytes(rng.integers(97, 123, int(rng.integers(9, 40))).astype(np.uint8)) for _ in range(5000)]
    picks = rng.integers(0, len(words), 200_000)
    text = b" ".join(words[i] for i in picks) + b"\n"
    want = ops.cpu_count(text)
    for all_ranks in (False, True):  # rank-0 gather path | owner exchange + broadcast
        assert_same(ops.loopback_count(text, ranks, chunk_bytes=1 << 20, merge_mode=merge_mode, all_ranks=all_ranks),
                    want)


@pytest.mark.parametrize("merge_mode", [0, 1])
@pytest.mark.parametrize("ranks", [1, 3, 8])
@pytest.mark.parametrize("opts", [dict(chunk_bytes=8 << 20), dict(log2_rec_buckets=1, log2_tab_buckets=1, chunk_bytes=8 << 20),
                                  dict(min_records=16384, records_per_byte=0.001, chunk_bytes=1 << 20)])
def test_loopback_merge_speculative(ranks, merge_mode, opts, monkeypatch):
    """HBM-resident shards: each rank's last pass stays pending and the merged
    finalize runs behind it (merge_cols_speculative: compaction + owner plan +
    all-gather, one host wait).  With a 2-bucket starting table (table splits)
    or tiny shuffle regions (pass re-runs) ranks flag recovery in the gathered
    matrix and all of them fall back to the synchronous protocol together."""
    monkeypatch.setenv("WC_MERGE_ROOT_ROWS", "0")  # the owner exchange
    rng = np.random.default_rng(70 + ranks)
    text = random_text(rng, 300_000, alphabet=b"abcdefgh  \n", long_words=6) + ops.synth_host(3 << 20, seed=4,
                                                                                              vocab=40000)
    want = ops.cpu_count(text)
    for all_ranks in (False, True):
        got = ops.loopback_count(text, ranks, merge_mode=merge_mode, all_ranks=all_ranks, resident=True, **opts)
        assert_same(got, want)


def test_file_stream(tmp_path):
    rng = np.random.default_rng(21)
    text = random_text(rng, 3_000_000, long_words=10)
    p = tmp_path / "in.txt"
    p.write_bytes(text)
    with ops.Engine(device=0, chunk_bytes=1 << 18) as e:
        e.count_file(str(p))
        got = e.result()
    assert_same(got, ops.cpu_count(text))


def test_replay_host_staged():
    pool = np.frombuffer(ops.synth_host(1 << 20, seed=4, vocab=1000), np.uint8)
    with ops.Engine(device=0, chunk_bytes=1 << 18) as e:
        e.count_replay(pool, total=5 << 20)
        got = e.result()
    one = ops.cpu_count(pool.tobytes())
    assert got.total == 5 * one.total
    assert dict(zip(got.words, got.counts.tolist())) == {w: 5 * int(c) for w, c in zip(one.words, one.counts)}


def test_rccl_world1():
    uid = ops.Comm.unique_id()
    comm = ops.Comm(uid, 0, 1, 0)
    with ops.Engine(device=0, chunk_bytes=1 << 20) as e:
        text = ops.synth_host(1 << 18, seed=1, vocab=500)
        e.count_bytes(text)
        got = e.result(comm)
    comm.close()
    assert_same(got, ops.cpu_count(text))


@pytest.mark.parametrize("merge_mode", [0, 1])
def test_rccl_merge_protocol_world1(merge_mode):
    """The full RCCL merge (grouped send/recv, allgather, broadcast / reduce-scatter)
    on one rank: WC_MERGE_ALWAYS makes finalize run it even at world size 1 (the
    only RCCL world a one-GPU box can build).  Runs in a child process so the
    env switch does not leak into other tests."""
    code = (
        "import os, sys\n"
        "from cuda_mapreduce_amd import ops\n"
        "uid = ops.Comm.unique_id(); comm = ops.Comm(uid, 0, 1, 0)\n"
        f"e = ops.Engine(device=0, chunk_bytes=1 << 20, merge_mode={merge_mode})\n"
        "text = ops.synth_host(3 << 18, seed=2, vocab=3000, zipf_s=0.8)\n"
        "e.count_bytes(text)\n"
        "for all_ranks in (False, True):\n"
        "    got = e.result(comm, all_ranks=all_ranks)\n"
        "    want = ops.cpu_count(text)\n"
        "    assert got.words == want.words and got.counts.tolist() == want.counts.tolist(), 'mismatch'\n"
        "assert e.stats()['device_ms']['merge'] > 0\n"
        "e.close(); comm.close(); print('ok')\n"
    )
    env = dict(os.environ, WC_MERGE_ALWAYS="1")
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, timeout=120)
    assert out.returncode == 0 and b"ok" in out.stdout, out.stderr.decode()[-2000:]


@pytest.mark.parametrize("merge_mode", [0, 1])
def test_planned_merge_outgrown_owner_table_redoes(merge_mode):
    """The planned merge sizes each owner's table from the learned merged-row
    cap (2 x cap, not 2 x rows received).  Caps learned on a shared vocabulary
    (every owner sees each word from every rank: ~V / W distinct keys), then a
    job whose four ranks hold DISJOINT vocabularies (~V distinct per owner, the
    rows per sender unchanged, so no fixed region overflows): the owner table
    fills, the insert's bounded probes end instead of spinning, the compaction
    counts more merged rows than the cap and the merge is redone exactly."""
    warm = ops.synth_host(4 << 20, seed=11, vocab=3000)
    data = b"".join(ops.synth_host(1 << 20, seed=21 + r, vocab=3000) for r in range(4))
    got = ops.loopback_count(data, 4, resident=True, warm=warm, chunk_bytes=1 << 20, merge_mode=merge_mode)
    assert_same(got, ops.cpu_count(data))


@pytest.mark.parametrize("fault", ["1:1", "2:3", "0:2"])
@pytest.mark.parametrize("merge_mode", [0, 1])
def test_loopback_injected_comm_fault(fault, merge_mode, monkeypatch):
    """one rank's collective fails (WC_COMM_FAULT=<rank>:<n>); every
    rank must leave its merge with an error — the failed rank aborts the
    communicator, which wakes the peers blocked in the collective — instead of
    hanging or returning a partial table.  A fresh job afterwards is unaffected."""
    text = ops.synth_host(1 << 20, seed=3, vocab=3000)
    monkeypatch.setenv("WC_MERGE_ROOT_ROWS", "0")  # the owner exchange: most collectives
    monkeypatch.setenv("WC_COMM_FAULT", fault)
    with pytest.raises(RuntimeError, match="injected comm fault"):
        ops.loopback_count(text, 3, chunk_bytes=1 << 20, merge_mode=merge_mode, all_ranks=True)
    monkeypatch.delenv("WC_COMM_FAULT")
    assert_same(ops.loopback_count(text, 3, chunk_bytes=1 << 20, merge_mode=merge_mode), ops.cpu_count(text))


def test_rccl_injected_fault_aborts_communicator():
    """RCCL path of the failure handling: the injected fault aborts the
    communicator (ncclCommAbort) and raises; a later merge on it raises at once
    ('failed earlier') instead of issuing collectives on a dead communicator.
    Child process: the env switches must not leak into other tests."""
    code = (
        "from cuda_mapreduce_amd import ops\n"
        "uid = ops.Comm.unique_id(); comm = ops.Comm(uid, 0, 1, 0)\n"
        "e = ops.Engine(device=0, chunk_bytes=1 << 20)\n"
        "e.count_bytes(ops.synth_host(1 << 18, seed=1, vocab=500))\n"
        "msgs = []\n"
        "for _ in range(2):\n"
        "    try:\n"
        "        e.result(comm)\n"
        "    except RuntimeError as ex:\n"
        "        msgs.append(str(ex))\n"
        "assert len(msgs) == 2 and 'injected comm fault' in msgs[0] and 'failed earlier' in msgs[1], msgs\n"
        "e.close(); comm.close(); print('ok')\n"
    )
    env = dict(os.environ, WC_MERGE_ALWAYS="1", WC_COMM_FAULT="0:1")
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, timeout=120)
    assert out.returncode == 0 and b"ok" in out.stdout, out.stderr.decode()[-2000:]


def test_cli_golden(tmp_path, golden_text):
    exe = os.path.join(ROOT, "wordcount")
    (tmp_path / "test.txt").write_bytes(golden_text)
    out = subprocess.run([exe], cwd=tmp_path, capture_output=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout == GOLDEN_OUTPUT
    out = subprocess.run([exe, str(tmp_path / "test.txt")], capture_output=True, timeout=120)
    assert out.stdout == GOLDEN_OUTPUT


@pytest.mark.parametrize("merge", ["shuffle", "dense"])
@pytest.mark.parametrize("ranks", [2, 4])
def test_cli_virtual_ranks(tmp_path, merge, ranks):
    """The CLI's thread-per-rank path (tools/wordcount.cpp) with W loopback ranks
    on one GPU: byte-identical output to --cpu, JSON reports 1 GPU and W ranks."""
    import json

    exe = os.path.join(ROOT, "wordcount")
    rng = np.random.default_rng(ranks)
    text = random_text(rng, 300_000, long_words=5) + ops.synth_host(2 << 20, seed=8, vocab=20000)
    f = tmp_path / "in.txt"
    f.write_bytes(text)
    want = subprocess.run([exe, str(f), "--cpu", "--no-echo"], capture_output=True, timeout=120)
    assert want.returncode == 0, want.stderr
    bj = tmp_path / "b.json"
    got = subprocess.run([exe, str(f), "--no-echo", "--virtual-ranks", str(ranks), "--merge", merge, "--chunk-bytes",
                          "1M", "--bench-json", str(bj)], capture_output=True, timeout=120)
    assert got.returncode == 0, got.stderr
    assert got.stdout == want.stdout
    js = json.loads(bj.read_text())
    assert js["gpus"] == 1 and js["ranks"] == ranks and js["virtual_ranks"] is True


def test_pinned_replay_host_staged():
    pool = np.frombuffer(ops.synth_host(1 << 20, seed=6, vocab=2000), np.uint8).copy()
    with ops.Engine(device=0, chunk_bytes=1 << 18) as e:
        e.count_replay_pinned(pool, total=(5 << 20) + (1 << 18))
        got = e.result()
    one = ops.cpu_count(pool.tobytes())
    q = ops.cpu_count(pool[: 1 << 18].tobytes())
    want = {w: 5 * int(c) for w, c in zip(one.words, one.counts)}
    for w, c in zip(q.words, q.counts):
        want[w] = want.get(w, 0) + int(c)
    assert got.total == 5 * one.total + q.total
    assert dict(zip(got.words, got.counts.tolist())) == want


@pytest.mark.parametrize("n", [1, 2, 5, 2047, 2048, 2049, 100_003, 1_000_000])
@pytest.mark.parametrize("bits", [8, 13, 30, 64])
def test_radix_sort_kernel(n, bits):
    """Kernel unit test: onesweep wc_os_hist / wc_os_pass (decoupled look-back) against
    numpy's stable argsort (many equal keys, so stability is checked too)."""
    import ctypes

    from cuda_mapreduce_amd.ops._lib import check, lib

    rng = np.random.default_rng(n * 131 + bits)
    hi = (1 << bits) - 1 if bits < 64 else (1 << 64) - 1
    keys = rng.integers(0, 1 << 62, n, dtype=np.uint64) * np.uint64(4) + rng.integers(0, 4, n, dtype=np.uint64)
    keys &= np.uint64(hi)
    if n > 10:
        keys[: n // 3] = keys[n // 3 : 2 * (n // 3)] % np.uint64(97)  # duplicates
    out = np.zeros(n, np.uint64)
    perm = np.zeros(n, np.uint32)
    P64 = ctypes.POINTER(ctypes.c_uint64)
    check(lib.wc_debug_radix_sort(0, keys.ctypes.data_as(P64), n, bits, out.ctypes.data_as(P64),
                                  perm.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))))
    want = np.argsort(keys, kind="stable")
    assert np.array_equal(perm, want.astype(np.uint32))
    assert np.array_equal(out, keys[want])
