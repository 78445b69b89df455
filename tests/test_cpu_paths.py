"""CPU-only tests: output contract, reference-quirk emulation, synthetic stream,
shard ownership.  Run everywhere (no GPU needed)."""
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN_OUTPUT, ROOT

ops = pytest.importorskip("cuda_mapreduce_amd.ops")


def table(res):
    return [(w, int(c)) for w, c in zip(res.words, res.counts)]


def test_golden_oracle(golden_text):
    res = ops.cpu_count(golden_text)
    assert ops.format_output(res, echo=golden_text) == GOLDEN_OUTPUT


def test_golden_cli_cpu(tmp_path, golden_text):
    exe = os.path.join(ROOT, "wordcount")
    (tmp_path / "test.txt").write_bytes(golden_text)
    out = subprocess.run([exe, "--cpu"], cwd=tmp_path, capture_output=True, timeout=60)
    assert out.returncode == 0 and out.stdout == GOLDEN_OUTPUT
    out = subprocess.run([exe, "--compat=reference"], cwd=tmp_path, capture_output=True, timeout=60)
    assert out.stdout == GOLDEN_OUTPUT


def test_cli_missing_file_matches_reference(tmp_path):
    # reference: prints the empty framing and exits 0 (main.cu:174)
    exe = os.path.join(ROOT, "wordcount")
    out = subprocess.run([exe, "--cpu"], cwd=tmp_path, capture_output=True, timeout=60)
    assert out.returncode == 0
    assert out.stdout == b"Input Data:\n" + b"-" * 26 + b"\n" + b"-" * 26 + b"\nTotal Count:0\n"


def test_cli_format_tab_and_first_occurrence_order():
    res = ops.cpu_count(b"b a b c a b\n")
    assert table(res) == [(b"b", 3), (b"a", 2), (b"c", 1)]
    assert b"b\t3\n" in ops.format_output(res)


# the reference's verified behaviour on its edge cases.
COMPAT_CASES = [
    (b"a  b\nb a\n", [(b"a", 3), (b"b", 2)]),
    (b" a b\n", [(b"a", 1), (b"b", 1)]),
    (b"x \ny\n", [(b"x", 2), (b"y", 1)]),
    (b"Good Go\n", [(b"Good", 2)]),
    (b"Go Good\n", [(b"Go", 1), (b"Good", 1)]),
    (b"Hello hello, hello\n", [(b"Hello", 1), (b"hello,", 2)]),
    (b"a\tb a\n", [(b"a\tb", 2)]),
    (b"a b\r\nb c\r\n", [(b"a", 1), (b"b", 2), (b"c", 1)]),
    (b"a\rb c\nd\n", [(b"a", 1), (b"d", 1)]),
    (b"x y\nlast word", [(b"x", 1), (b"y", 1), (b"last", 1)]),
    (b"a b\n\nc d\n", [(b"a", 1), (b"b", 1)]),
    (b"a\n" * 9, [(b"a", 9)]),
]


@pytest.mark.parametrize("text,want", COMPAT_CASES)
def test_reference_compat_quirks(text, want):
    assert table(ops.cpu_count_compat(text)) == want


def test_clean_semantics_differ_from_quirks():
    assert table(ops.cpu_count(b"Good Go\n")) == [(b"Good", 1), (b"Go", 1)]
    assert table(ops.cpu_count(b"x y\nlast word")) == [(b"x", 1), (b"y", 1), (b"last", 1), (b"word", 1)]
    assert table(ops.cpu_count(b"a\rb c\nd\n")) == [(b"a", 1), (b"b", 1), (b"c", 1), (b"d", 1)]


def test_compat_equals_clean_inside_envelope(golden_text):
    rng = np.random.default_rng(0)
    vocab = [b"alpha", b"beta", b"gamma", b"delta", b"eps"]  # no word is a prefix of another
    for _ in range(50):
        lines = []
        for _ in range(rng.integers(1, 9)):
            lines.append(b" ".join(vocab[i] for i in rng.integers(0, 5, rng.integers(1, 8))) + b"\n")
        t = b"".join(lines)
        assert table(ops.cpu_count_compat(t)) == table(ops.cpu_count(t))


def test_synth_is_segment_addressable():
    full = ops.synth_host(64 * 1024, first_segment=0, seed=3, vocab=1000)
    part = ops.synth_host(16 * 1024, first_segment=20, seed=3, vocab=1000)
    assert full[20 * 1024 : 36 * 1024] == part
    assert all(full[i * 1024 + 1023] in b" \n" for i in range(64))  # segments end on a delimiter


def test_synth_zipf_shape():
    res = ops.cpu_count(ops.synth_host(4 << 20, seed=1, vocab=100000))
    c = np.sort(res.counts)[::-1]
    assert res.total > 600_000 and len(res) > 20000, (res.total, len(res))
    assert c[0] > 20 * c[100]  # heavy head


@pytest.mark.parametrize("world", [1, 2, 3, 5, 8])
def test_shard_ownership_partitions_tokens(world):
    rng = np.random.default_rng(world)
    a = np.frombuffer(b"ab c\n", np.uint8)
    text = a[rng.integers(0, 5, 10007)].tobytes()
    pieces = []
    for r in range(world):
        b, e = ops.shard_range(text, r, world)
        pieces.append(ops.cpu_count(text[b:e], global_base=b))
    merged = {}
    for p in pieces:
        for w, c, f in zip(p.words, p.counts, p.first_off):
            cnt, first = merged.get(w, (0, 1 << 62))
            merged[w] = (cnt + int(c), min(first, int(f)))
    want = ops.cpu_count(text)
    assert sum(p.total for p in pieces) == want.total
    assert {w: v for w, v in merged.items()} == {w: (int(c), int(f)) for w, c, f in zip(want.words, want.counts, want.first_off)}


def test_shard_range_file_matches_mem(tmp_path):
    text = ops.synth_host(50_000, seed=9, vocab=300)[:49_999]
    p = tmp_path / "x.txt"
    p.write_bytes(text)
    for world in (2, 4, 7):
        for r in range(world):
            assert ops.shard_range_file(str(p), r, world) == ops.shard_range(text, r, world)


def test_cli_synthetic_cpu_matches_python_oracle(tmp_path):
    exe = os.path.join(ROOT, "wordcount")
    out = subprocess.run([exe, "--cpu", "--synthetic", "64K:3:500", "--bench-json", str(tmp_path / "b.json")],
                         capture_output=True, timeout=60)
    assert out.returncode == 0, out.stderr
    want = ops.format_output(ops.cpu_count(ops.synth_host(64 * 1024, seed=3, vocab=500)))
    assert out.stdout == want
    import json

    j = json.loads((tmp_path / "b.json").read_text())
    assert j["bytes"] == 64 * 1024 and j["path"] == "cpu"


def test_cli_top_k(tmp_path):
    exe = os.path.join(ROOT, "wordcount")
    p = tmp_path / "t.txt"
    p.write_bytes(b"a b a c a b d\n")
    out = subprocess.run([exe, str(p), "--cpu", "--no-echo", "--top", "2"], capture_output=True, timeout=60)
    assert out.stdout.split(b"-" * 26 + b"\n")[1] == b"a\t3\nb\t2\n"
    assert out.stdout.endswith(b"Total Count:7\n")


def test_cli_bench_json_and_log_levels(tmp_path, golden_text):
    # stdout stays reference-identical; diagnostics go to stderr / JSON
    import json

    exe = os.path.join(ROOT, "wordcount")
    (tmp_path / "test.txt").write_bytes(golden_text)
    env = dict(os.environ, WC_LOG="info")
    out = subprocess.run([exe, "--cpu", "--bench", "--bench-json", "b.json", "--checkpoint", "c", "--checkpoint-every",
                          "20"], cwd=tmp_path, capture_output=True, timeout=60, env=env)
    assert out.returncode == 0 and out.stdout == GOLDEN_OUTPUT
    assert b"wordcount bench: {" in out.stderr and b"[wc info" in out.stderr
    d = json.loads((tmp_path / "b.json").read_text())
    assert d["tokens"] == 9 and d["keys"] == 6 and d["path"] == "cpu" and "device_ms" in d
    quiet = subprocess.run([exe, "--cpu"], cwd=tmp_path, capture_output=True, timeout=60,
                           env=dict(os.environ, WC_LOG="warn"))
    assert quiet.stderr == b""


@pytest.mark.timeout(600)
def test_host_code_under_asan_ubsan(tmp_path, golden_text):
    """host code (CLI, CPU oracle, quirks emulation, checkpoint I/O,
    formatter) built with -fsanitize=address,undefined (`make asan`) runs the CPU
    paths clean; GPU code is not sanitised (no GPU ASan on this pool)."""
    b = subprocess.run(["make", "-C", ROOT, "-j8", "asan"], capture_output=True, timeout=600)
    assert b.returncode == 0, b.stderr[-2000:]
    exe = os.path.join(ROOT, "build", "wordcount_asan")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    (tmp_path / "test.txt").write_bytes(golden_text)
    rng = np.random.default_rng(5)
    alphabet = np.frombuffer(b"abcXYZ,\t  \r\n", dtype=np.uint8)
    (tmp_path / "r.txt").write_bytes(alphabet[rng.integers(0, len(alphabet), 200000)].tobytes())
    for args in (["--cpu"], ["--compat=reference"], ["r.txt", "--cpu", "--no-echo", "--top", "5"],
                 ["r.txt", "--compat=reference", "--no-echo"],
                 ["r.txt", "--cpu", "--no-echo", "--checkpoint", "ck", "--checkpoint-every", "30000"],
                 ["r.txt", "--cpu", "--no-echo", "--checkpoint", "ck", "--resume", "--bench"]):
        r = subprocess.run([exe] + args, cwd=tmp_path, capture_output=True, timeout=120, env=env)
        assert r.returncode == 0, (args, r.stderr[-3000:])
        assert b"ERROR: AddressSanitizer" not in r.stderr and b"runtime error" not in r.stderr, args
    r = subprocess.run([exe, "--cpu"], cwd=tmp_path, capture_output=True, timeout=120, env=env)
    assert r.stdout == GOLDEN_OUTPUT


def test_cli_refuses_more_gpus_than_visible(tmp_path, golden_text):
    """`wordcount --gpus N` with N above the visible GPUs (none in this CPU
    container) fails with a clear message instead of silently running on fewer
    and reporting N; --virtual-ranks is the one-GPU multi-rank form."""
    exe = os.path.join(ROOT, "wordcount")
    (tmp_path / "test.txt").write_bytes(golden_text)
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", ROCR_VISIBLE_DEVICES="")
    out = subprocess.run([exe, "--gpus", "8", "--no-echo"], cwd=tmp_path, capture_output=True, timeout=60, env=env)
    assert out.returncode != 0
    assert b"8 GPUs requested" in out.stderr and b"visible" in out.stderr
    bad = subprocess.run([exe, "--virtual-ranks", "4", "--gpus", "2"], cwd=tmp_path, capture_output=True, timeout=60)
    assert bad.returncode != 0 and b"--virtual-ranks runs on one GPU" in bad.stderr


@pytest.mark.parametrize("piece", [65521, 1 << 20, (4 << 20) + 7, 48 << 20])
def test_parallel_file_reader(tmp_path, piece):
    """FileSource through pread_parallel's persistent reader pool (16 threads,
    4 MiB slices; src/io/source.cpp): every byte of [begin, end) in order, for
    pieces below, at and above the slice size, and a range that starts and ends
    mid-file."""
    import ctypes

    from cuda_mapreduce_amd.ops._lib import check, lib

    rng = np.random.default_rng(piece)
    data = rng.integers(0, 256, (40 << 20) + 12345, dtype=np.uint8)
    path = tmp_path / "f.bin"
    data.tofile(path)
    for begin, end in ((0, len(data)), (777, len(data) - 999)):
        out = np.zeros(end - begin, np.uint8)
        got = ctypes.c_uint64(0)
        check(lib.wc_debug_read_file(str(path).encode(), begin, end, piece,
                                     out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), ctypes.byref(got)))
        assert got.value == end - begin
        assert np.array_equal(out, data[begin:end])


def test_parallel_file_reader_concurrent_callers(tmp_path):
    """Several threads stream through FileSource at once (the CLI's one
    streaming thread per GPU): each caller has its own reader pool
    (src/io/source.cpp, thread_local) and its tasks are claimed through a
    generation-tagged ticket, so no caller runs another's slices, returns early
    or hangs.  ctypes drops the GIL for the native calls: the reads overlap."""
    import ctypes
    import threading

    from cuda_mapreduce_amd.ops._lib import check, lib

    rng = np.random.default_rng(11)
    data = rng.integers(0, 256, (48 << 20) + 4321, dtype=np.uint8)
    path = tmp_path / "f.bin"
    data.tofile(path)
    errors = []

    def reader(k):
        try:
            for rep in range(6):
                begin = (k * 5 + rep) * 1_000_003 % (8 << 20)
                end = len(data) - (k * 7 + rep) * 999_983 % (8 << 20)
                piece = (4 << 20) * (1 + (k + rep) % 3) + k
                out = np.zeros(end - begin, np.uint8)
                got = ctypes.c_uint64(0)
                check(lib.wc_debug_read_file(str(path).encode(), begin, end, piece,
                                             out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), ctypes.byref(got)))
                assert got.value == end - begin, (k, rep, got.value)
                assert np.array_equal(out, data[begin:end]), (k, rep)
        except Exception as ex:  # noqa: BLE001 - surfaced below
            errors.append(repr(ex))

    th = [threading.Thread(target=reader, args=(k,)) for k in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in th), "a reader hung"
    assert not errors, errors
