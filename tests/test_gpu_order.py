"""First-occurrence ordering on the GPU (sort.hip: the three-launch sample sort,
the bitmap ranks and their radix-sort fallbacks), exact against the CPU oracle.

Stats()["order_path"]: 1 = sample sort (the engine uses it up to 400k keys;
the kernel takes 512 bins up to 400k and 2048 up to FO_MAX_KEYS = 1.6M, tested
directly below), 2 = radix sort (WC_FIRST_ORDER=radix, or above 400k keys when
the bitmap would exceed 128 bytes per key), 3 = a sample-sort bin overflowed and
the radix sort redid the order, 4 = the speculative finalize's sample sort
(sized from the previous job's key count) overflowed and the exact-count redo
did not, 5 = bitmap ranks (above 400k keys, or WC_FIRST_ORDER=bitmap), 6 = two
keys shared a bitmap position and the radix sort redid the order.
WC_FO_CAP=512 lowers the most rows a bin may hold, forcing the overflow paths."""
import numpy as np
import pytest

from test_gpu_engine import assert_same

pytestmark = pytest.mark.gpu

ops = pytest.importorskip("cuda_mapreduce_amd.ops")


def _resident(e, n, seed, vocab, zipf_s=0.6):
    e.reset()
    e.synth_device(n, first_segment=1, seed=seed, vocab=vocab, zipf_s=zipf_s)
    e.count_resident(n, global_base=0)
    return e.result()


@pytest.mark.parametrize("vocab,n", [(40, 1 << 20), (3000, 4 << 20), (120_000, 32 << 20), (900_000, 96 << 20)])
def test_sample_order_sizes(vocab, n):
    want = ops.cpu_count(ops.synth_host(n, first_segment=1, seed=vocab, vocab=vocab, zipf_s=0.6, threads=8))
    with ops.Engine(device=0) as e:
        for job in range(2):  # first job: hint cap/4; second: the previous key count
            got = _resident(e, n, vocab, vocab)
            assert e.stats()["order_path"] in ((1, 4, 5) if job == 0 else (1, 5))
            assert_same(got, want)
        assert e.stats()["order_path"] == (1 if len(want) <= 390_000 else 5)  # the engine's sample-sort limit


def test_radix_order_forced(monkeypatch):
    monkeypatch.setenv("WC_FIRST_ORDER", "radix")
    n = 16 << 20
    want = ops.cpu_count(ops.synth_host(n, first_segment=1, seed=3, vocab=60000, zipf_s=0.6))
    with ops.Engine(device=0) as e:
        assert_same(_resident(e, n, 3, 60000), want)
        assert e.stats()["order_path"] == 2


@pytest.mark.parametrize("vocab,n,chunk", [(40, 1 << 20, None), (60000, 16 << 20, None), (200_000, 24 << 20, 4 << 20)])
def test_bitmap_order_forced(vocab, n, chunk, monkeypatch):
    """WC_FIRST_ORDER=bitmap at every size: the speculative finalize (resident
    text) and the synchronous one (streamed chunks); a second job checks the
    bitmap was left cleared."""
    monkeypatch.setenv("WC_FIRST_ORDER", "bitmap")
    text = ops.synth_host(n, seed=vocab, vocab=vocab, zipf_s=0.6)
    want = ops.cpu_count(text)
    kw = {"chunk_bytes": chunk} if chunk else {}
    with ops.Engine(device=0, **kw) as e:
        for _ in range(2):
            e.reset()
            e.count_bytes(text)
            assert_same(e.result(), want)
            assert e.stats()["order_path"] == 5


@pytest.mark.parametrize("vocab", [40, 60000])
def test_bitmap_order_resident(vocab, monkeypatch):
    """WC_FIRST_ORDER=bitmap on resident text: the last pass's reduce sets the
    keys' bits itself (the order skips its bit-set launch); jobs in a row and a
    count_bytes job in between (which sets its own bits) stay exact."""
    monkeypatch.setenv("WC_FIRST_ORDER", "bitmap")
    n = 16 << 20
    want = ops.cpu_count(ops.synth_host(n, first_segment=1, seed=vocab, vocab=vocab, zipf_s=0.6))
    other = ops.synth_host(4 << 20, seed=7, vocab=5000)
    with ops.Engine(device=0) as e:
        for job in range(3):
            assert_same(_resident(e, n, vocab, vocab), want)
            assert e.stats()["order_path"] == 5
            if job == 1:
                e.reset()
                e.count_bytes(other)
                assert_same(e.result(), ops.cpu_count(other))


def test_bitmap_order_merged(monkeypatch):
    """The merged table's order by bitmap ranks (key columns, count on the device)."""
    monkeypatch.setenv("WC_FIRST_ORDER", "bitmap")
    monkeypatch.setenv("WC_MERGE_ROOT_ROWS", "0")
    text = ops.synth_host(24 << 20, seed=13, vocab=200_000, zipf_s=0.5)
    want = ops.cpu_count(text)
    for merge_mode in (0, 1):
        assert_same(ops.loopback_count(text, 3, merge_mode=merge_mode, resident=True, chunk_bytes=8 << 20), want)


def test_bitmap_shared_position_falls_back(monkeypatch):
    """Two texts counted at the same global base: different words share first
    offsets (bitmap positions), so the bitmap's overflow word sends the order to
    the radix sort (order_path 6); counts stay exact and first offsets ordered."""
    monkeypatch.setenv("WC_FIRST_ORDER", "bitmap")
    a = b"alpha beta gamma delta " * 1000
    b = b"one two three four " * 1000
    with ops.Engine(device=0) as e:
        e.count_bytes(a, global_base=0)
        e.count_bytes(b, global_base=0)
        got = e.result()
        assert e.stats()["order_path"] == 6
        assert got.as_dict() == {**ops.cpu_count(a).as_dict(), **ops.cpu_count(b).as_dict()}
        assert np.all(np.diff(got.first_off.astype(np.int64)) >= 0)
        e.reset()  # the bitmap was cleared despite the overflow
        e.count_bytes(a)
        assert_same(e.result(), ops.cpu_count(a))
        assert e.stats()["order_path"] == 5


def test_overflow_falls_back_to_radix(monkeypatch):
    monkeypatch.setenv("WC_FO_CAP", "512")  # bins average ~600 rows here
    n = 32 << 20
    want = ops.cpu_count(ops.synth_host(n, first_segment=1, seed=8, vocab=400_000, zipf_s=0.6, threads=8))
    with ops.Engine(device=0) as e:
        assert_same(_resident(e, n, 8, 400_000), want)
        assert e.stats()["order_path"] == 3
    # bins built from the reducer's exact key histogram are balanced: a smaller cap forces the overflow
    monkeypatch.setenv("WC_FO_CAP", "128")
    text = ops.synth_host(4 << 20, seed=9, vocab=300_000, zipf_s=0.3)
    with ops.Engine(device=0, chunk_bytes=1 << 20) as e:  # streamed chunks: the non-speculative finalize
        e.count_bytes(text)
        assert_same(e.result(), ops.cpu_count(text))
        assert e.stats()["order_path"] == 3


def test_speculative_hint_then_many_keys():
    # job 1 has ~40 keys, job 2 ~300k: the speculative finalize's order is chosen
    # by the previous job's count (the sample sort sizes itself from the table)
    n = 48 << 20
    want = ops.cpu_count(ops.synth_host(n, first_segment=1, seed=5, vocab=300_000, zipf_s=0.4, threads=8))
    with ops.Engine(device=0) as e:
        _resident(e, 1 << 20, 1, 40)
        assert e.stats()["order_path"] == 1
        assert_same(_resident(e, n, 5, 300_000, zipf_s=0.4), want)
        assert e.stats()["order_path"] in (1, 4)
        assert_same(_resident(e, n, 5, 300_000, zipf_s=0.4), want)
        assert e.stats()["order_path"] == 1  # hinted by job 2 now


@pytest.mark.parametrize("cap", [None, "512"])
@pytest.mark.parametrize("merge_mode", [0, 1])
def test_merged_order(cap, merge_mode, monkeypatch):
    """The merged table's order (sort_cols_by_first on key columns, count on the
    device): sample sort, and with WC_FO_CAP=512 its overflow redo by the radix
    sort after the finalize's last wait."""
    if cap:
        monkeypatch.setenv("WC_FO_CAP", cap)
    monkeypatch.setenv("WC_MERGE_ROOT_ROWS", "0")
    text = ops.synth_host(24 << 20, seed=12, vocab=200_000, zipf_s=0.5)
    want = ops.cpu_count(text)
    for all_ranks in (False, True):
        assert_same(ops.loopback_count(text, 3, merge_mode=merge_mode, all_ranks=all_ranks, resident=True,
                                       chunk_bytes=8 << 20), want)


def _first_order(keys, reps=1):
    import ctypes

    from cuda_mapreduce_amd.ops._lib import check, lib

    keys = np.ascontiguousarray(keys, np.uint64)
    n = len(keys)
    srt = np.empty(max(n, 1), np.uint64)
    perm = np.empty(max(n, 1), np.uint32)
    ovf, ms = ctypes.c_int(0), ctypes.c_double(0)
    P64, P32 = ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint32)
    check(lib.wc_debug_first_order(0, keys.ctypes.data_as(P64), n, reps, srt.ctypes.data_as(P64),
                                   perm.ctypes.data_as(P32), ctypes.byref(ovf), ctypes.byref(ms)))
    return srt[:n], perm[:n], ovf.value


@pytest.mark.parametrize("n", [1, 2, 63, 4095, 4097, 100_000, 300_000, 400_000, 400_001, 1_000_000, 1_600_000])
@pytest.mark.parametrize("dist", ["uniform", "crowded", "sorted", "reversed"])
def test_first_order_kernel(n, dist):
    rng = np.random.default_rng(n)
    if dist == "uniform":
        keys = rng.permutation(np.unique(rng.integers(0, 1 << 40, n + n // 8 + 8, dtype=np.uint64))[:n])
    elif dist == "crowded":  # first offsets crowd the start of a text
        keys = rng.permutation(np.unique((rng.random(3 * n) ** 4 * (1 << 34)).astype(np.uint64))[:n])
    elif dist == "sorted":
        keys = np.arange(n, dtype=np.uint64) * 7
    else:
        keys = (np.arange(n, dtype=np.uint64) * 3)[::-1].copy()
    srt, perm, ovf = _first_order(keys)
    assert ovf == 0
    assert np.array_equal(srt, np.sort(keys))
    assert np.array_equal(keys[perm], srt)


def _bitmap_order(keys):
    import ctypes

    from cuda_mapreduce_amd.ops._lib import check, lib

    keys = np.ascontiguousarray(keys, np.uint64)
    n = len(keys)
    srt = np.empty(max(n, 1), np.uint64)
    perm = np.empty(max(n, 1), np.uint32)
    ovf, ms, res = ctypes.c_int(0), ctypes.c_double(0), ctypes.c_uint64(0)
    P64, P32 = ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint32)
    check(lib.wc_debug_order(0, 1, keys.ctypes.data_as(P64), n, 2, srt.ctypes.data_as(P64), perm.ctypes.data_as(P32),
                             ctypes.byref(ovf), ctypes.byref(ms), ctypes.byref(res)))
    return srt[:n], perm[:n], ovf.value, res.value


@pytest.mark.parametrize("n", [1, 2, 511, 512, 513, 131_073, 1_000_000, 3_000_000])
@pytest.mark.parametrize("dist", ["uniform", "crowded", "dense", "reversed"])
def test_bitmap_order_kernel(n, dist):
    """bitmap_order on distinct keys (shift 0, bitmap of max key + 1 bits): the
    sorted keys and the permutation exact, the bitmap all zero after two calls."""
    rng = np.random.default_rng(n + 7)
    if dist == "uniform":
        keys = rng.permutation(np.unique(rng.integers(0, 1 << 30, n + n // 8 + 8, dtype=np.uint64))[:n])
    elif dist == "crowded":
        keys = rng.permutation(np.unique((rng.random(3 * n) ** 4 * (1 << 30)).astype(np.uint64))[:n])
    elif dist == "dense":  # every bit of every line set
        keys = rng.permutation(np.arange(n, dtype=np.uint64))
    else:
        keys = (np.arange(n, dtype=np.uint64) * 3 + 5)[::-1].copy()
    srt, perm, ovf, res = _bitmap_order(keys)
    assert ovf == 0 and res == 0
    assert np.array_equal(srt, np.sort(keys))
    assert np.array_equal(keys[perm], srt)


def test_bitmap_order_kernel_shared_position():
    keys = np.array([5, 900, 5, 70000, 3], np.uint64)
    _, _, ovf, res = _bitmap_order(keys)
    assert ovf == 1 and res == 0


def test_first_order_kernel_overflow_flag(monkeypatch):
    """A sample that misses a dense run of keys: the key column is sampled at
    rows i * n / 4096, so spread keys there and consecutive small keys
    everywhere else put ~96k rows in bin 0 — beyond every LDS capacity: the
    overflow word is raised (and nothing is written out of bounds)."""
    n = 100_000
    sampled = (np.arange(4096, dtype=np.uint64) * n) // 4096
    keys = np.zeros(n, np.uint64)
    keys[sampled] = (np.arange(4096, dtype=np.uint64) + 1) << 20
    rest = np.setdiff1d(np.arange(n, dtype=np.uint64), sampled)
    keys[rest] = np.arange(1, len(rest) + 1, dtype=np.uint64)
    assert len(np.unique(keys)) == n
    _, _, ovf = _first_order(keys)
    assert ovf == 1
    monkeypatch.setenv("WC_FO_CAP", "8192")
    _, _, ovf = _first_order(np.random.default_rng(3).permutation(np.arange(n, dtype=np.uint64)))
    assert ovf == 0
