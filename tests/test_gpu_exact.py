"""Exact word equality for LONG words (>= 16 bytes, hashed keys: keys.hpp) and
engine buffer independence — GPU tests against the CPU oracle.

`k1_hash_bits` (Options) truncates the LONG-word tail hash to a few bits, so
words that share their first 8 bytes and length collide in (k0, k1) by
construction; the map never combines LONG words, the reducer and both merge
protocols compare the word bytes, so the counts must still equal the
byte-keyed CPU oracle exactly."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ops = pytest.importorskip("cuda_mapreduce_amd.ops")


def assert_same(got, want):
    assert got.total == want.total
    assert got.words == want.words
    assert np.array_equal(got.counts, want.counts)
    assert np.array_equal(got.first_off, want.first_off)


def colliding_text(seed, n_words=60000, distinct=300):
    """LONG words sharing one 8-byte prefix and one length (so only the tail
    hash separates them), mixed with short and medium words."""
    rng = np.random.default_rng(seed)
    longs = [b"prefix__" + bytes(rng.integers(97, 123, 12, dtype=np.uint8)) for _ in range(distinct)]
    other = [b"a", b"bb", b"ccccccccc", b"medium_word_15b", b"prefix__xyz"]
    out = []
    for i in range(n_words):
        if rng.random() < 0.6:
            out.append(longs[int(rng.zipf(1.3)) % distinct])
        else:
            out.append(other[int(rng.integers(0, len(other)))])
        out.append(b" " if rng.random() < 0.9 else b"\n")
    return b"".join(out)


@pytest.mark.parametrize("bits", [1, 3])
def test_forced_long_key_collisions_single_gpu(bits):
    text = colliding_text(bits)
    want = ops.cpu_count(text)
    with ops.Engine(device=0, chunk_bytes=1 << 20, k1_hash_bits=bits) as e:
        e.count_bytes(text)
        assert_same(e.result(), want)


@pytest.mark.parametrize("merge_mode", [0, 1])
@pytest.mark.parametrize("ranks", [2, 4])
def test_forced_long_key_collisions_merge(ranks, merge_mode, monkeypatch):
    monkeypatch.setenv("WC_MERGE_ROOT_ROWS", "0")  # the owner exchange, not the root gather
    text = colliding_text(10 + ranks)
    want = ops.cpu_count(text)
    got = ops.loopback_count(text, ranks, merge_mode=merge_mode, k1_hash_bits=2, chunk_bytes=1 << 20)
    assert_same(got, want)


def test_resident_text_survives_streaming():
    """Streamed counts use their own staging buffers: a resident synthetic
    text stays valid around them, in either order (advisor finding)."""
    host = ops.synth_host(3 << 20, first_segment=5, seed=9, vocab=2000)
    with ops.Engine(device=0, chunk_bytes=1 << 22) as e:
        e.count_bytes(host)
        a = e.result()
        e.synth_device(8 << 20, first_segment=0, seed=4, vocab=3000)
        e.reset()
        e.count_bytes(host)
        b = e.result()
        e.reset()
        e.count_resident(8 << 20)
        c = e.result()
    assert_same(a, ops.cpu_count(host))
    assert_same(b, ops.cpu_count(host))
    assert_same(c, ops.cpu_count(ops.synth_host(8 << 20, first_segment=0, seed=4, vocab=3000)))


def test_reset_ignores_stale_slices():
    """reset() zeroes only the bucket occupancy: slices of a previous job stay
    in memory and must never leak into the next one (reduce, compaction,
    split and an empty finalize all treat occupancy-0 buckets as empty)."""
    big = ops.synth_host(64 << 20, seed=11, vocab=200_000)
    small = b"alpha beta alpha gamma\nbeta alpha\n"
    with ops.Engine(device=0, chunk_bytes=16 << 20) as e:
        e.count_bytes(big)
        first = e.result()
        e.reset()
        empty = e.result()  # no pass since the reset
        e.reset()
        e.count_bytes(small)
        tiny = e.result()
        e.reset()
        e.count_bytes(big)  # grows / splits again over stale slices
        again = e.result()
    assert_same(first, ops.cpu_count(big))
    assert empty.total == 0 and len(empty.words) == 0
    assert_same(tiny, ops.cpu_count(small))
    assert_same(again, first)


def test_long_layout_follows_the_pass_before():
    """The LONG-record layout is picked per pass from the LONG token share of
    the pass before (Engine::Impl::long_direct): a fresh engine queues LONG
    records from the 24-byte runs, a LONG-heavy pass switches the next one to
    the top-down layout streamed by long_direct, a LONG-free pass switches back.
    Every job is exact whichever layout ran."""
    heavy = colliding_text(21, n_words=80000, distinct=3000)  # ~60 % LONG tokens
    light = ops.synth_host(2 << 20, seed=2, vocab=5000)  # no word reaches 16 bytes
    want_h, want_l = ops.cpu_count(heavy), ops.cpu_count(light)
    layouts = []
    with ops.Engine(device=0) as e:
        for text, want in ((heavy, want_h), (heavy, want_h), (light, want_l), (light, want_l), (heavy, want_h)):
            e.reset()
            e.count_bytes(text)
            assert_same(e.result(), want)
            st = e.stats()
            layouts.append(st["long_direct"])
            assert st["long_tokens"] > 0 if text is heavy else st["long_tokens"] == 0
    assert layouts == [0, 1, 1, 0, 0]


@pytest.mark.parametrize("order,kernel", [("", "wc_fo_sort"), ("radix", "wc_table_keys"), ("bitmap", "wc_bm_place")])
def test_bounds_guard_names_the_writer(order, kernel, monkeypatch):
    """The finalize's row writers are bounds-guarded (kernels.hpp Bounds,
    profiles/r5_fault_hunt.md): a host key count short of the table's keys —
    the output columns sized too small, the class of the round-4 illegal
    access — ends in a clean error naming the kernel, not a GPU fault, and the
    next engine on the device counts exactly."""
    text = ops.synth_host(4 << 20, seed=3, vocab=20_000)
    monkeypatch.setenv("WC_FAULT_OCC_UNDER", "3000")  # read at engine creation
    monkeypatch.setenv("WC_NO_SPECULATE", "1")  # the host-sized finalize
    if order:
        monkeypatch.setenv("WC_FIRST_ORDER", order)
    with ops.Engine(device=0) as e:
        e.count_bytes(text)
        with pytest.raises(ops.WcError, match="bounds guard: " + kernel):
            e.result()
    monkeypatch.delenv("WC_FAULT_OCC_UNDER")
    with ops.Engine(device=0) as e:
        e.count_bytes(text)
        assert_same(e.result(), ops.cpu_count(text))


@pytest.mark.parametrize("opts", [dict(log2_tab_buckets=1, chunk_bytes=8 << 20),
                                  dict(min_records=16384, records_per_byte=0.001, chunk_bytes=1 << 20)])
def test_speculative_finalize_recovers(opts):
    """count_resident leaves its last pass pending and finalizes behind it; a
    pass that overflows (table split / shuffle-region re-run) must discard that
    speculative result and redo it.  Same table as the fully synchronous path
    (WC_NO_SPECULATE=1 is read at engine creation) and as the oracle."""
    import os
    want = ops.cpu_count(ops.synth_host(24 << 20, seed=5, vocab=50_000))
    with ops.Engine(device=0, **opts) as e:
        e.synth_device(24 << 20, seed=5, vocab=50_000)
        for _ in range(2):  # the second run starts from the grown table / same capacity
            e.reset()
            e.count_resident(24 << 20)
            got = e.result()
            assert_same(got, want)
    os.environ["WC_NO_SPECULATE"] = "1"
    try:
        with ops.Engine(device=0, **opts) as e:
            e.synth_device(24 << 20, seed=5, vocab=50_000)
            e.count_resident(24 << 20)
            assert_same(e.result(), want)
    finally:
        del os.environ["WC_NO_SPECULATE"]


def test_headline_stream_key_for_key():
    """The exact benchmark input (1 GiB, seed 1, Zipf(1.0), 100k words, one
    device chunk) against the generator-walk oracle; and 256 MiB of it against
    the tokenizing CPU oracle, which also checks the walk oracle itself."""
    n = 1 << 30
    with ops.Engine(device=0, chunk_bytes=n) as e:
        e.synth_device(n, first_segment=0, seed=1, vocab=100000, zipf_s=1.0)
        e.count_resident(n)
        got = e.result()
    assert_same(got, ops.cpu_count_synth(n, 0, 1, 100000, 1.0, 0, 16))
    m = 256 << 20
    with ops.Engine(device=0, chunk_bytes=m) as e:
        e.synth_device(m, first_segment=0, seed=1, vocab=100000, zipf_s=1.0)
        e.count_resident(m)
        got = e.result()
    assert_same(got, ops.cpu_count(ops.synth_host_array(m, 0, 1, 100000, 1.0, 16)))


def test_host_pool_replay_matches_oracle():
    """Native page-locked pool (HostPool) replayed chunk by chunk == oracle of the replay."""
    from cuda_mapreduce_amd.utils import compare_results, synthetic_oracle

    pool_b, chunk, total = 64 << 20, 16 << 20, 160 << 20
    pool = ops.HostPool(pool_b, first_segment=0, seed=3, vocab=20000, zipf_s=1.0, threads=8)
    with ops.Engine(device=0, chunk_bytes=chunk) as e:
        e.count_pool(pool, total)
        got = e.result()
    pool.close()
    assert compare_results(got, synthetic_oracle(1, total, 3, 20000, 1.0, pool_bytes=pool_b, chunk=chunk)) == ""


@pytest.mark.parametrize("chunk", [128 << 20, 32 << 20])
def test_long_words_under_load(chunk):
    """30 % of the vocabulary 16..64-byte words (hashed keys, byte-verified in the
    reduce), 1M-word Zipf vocabulary, one pass and four: key for key vs the
    generator-walk oracle."""
    n = 128 << 20
    with ops.Engine(device=0, chunk_bytes=chunk) as e:
        e.synth_device(n, first_segment=0, seed=3, vocab=1_000_000, zipf_s=1.0, long_frac=0.3)
        e.count_resident(n)
        got = e.result()
    want = ops.cpu_count_synth(n, 0, 3, 1_000_000, 1.0, 0, 16, 0.3)
    long_tokens = sum(int(c) for w, c in zip(want.words, want.counts) if len(w) >= 16)
    assert long_tokens > 0.2 * want.total
    assert_same(got, want)


def test_many_new_long_words_per_bucket():
    """More than 2048 distinct new LONG words per table bucket in one pass
    (the round-2 reducer queued at most 2048 per bucket and re-scanned beyond):
    every one is claimed in parallel and byte-verified."""
    n = 192 << 20
    with ops.Engine(device=0, chunk_bytes=n) as e:
        e.synth_device(n, first_segment=0, seed=8, vocab=3_000_000, zipf_s=0.6, long_frac=0.7)
        e.count_resident(n)
        got = e.result()
        buckets = 1 << e.stats()["log2_buckets"]
    want = ops.cpu_count_synth(n, 0, 8, 3_000_000, 0.6, 0, 16, 0.7)
    distinct_long = sum(1 for w in want.words if len(w) >= 16)
    assert distinct_long > 2048 * 256, distinct_long
    assert distinct_long / buckets > 256
    assert_same(got, want)


def test_synth_while_pass_pending():
    """count_resident leaves its last pass pending; regenerating the resident
    text before the result must not let a recovery of that pass (overflowing
    options: table splits / shuffle re-runs) read the new text (advisor)."""
    from cuda_mapreduce_amd.utils import merge_results

    for opts in (dict(log2_tab_buckets=1, chunk_bytes=8 << 20),
                 dict(min_records=16384, records_per_byte=0.001, chunk_bytes=1 << 20)):
        with ops.Engine(device=0, **opts) as e:
            e.synth_device(24 << 20, seed=5, vocab=50_000)
            e.count_resident(24 << 20)
            e.synth_device(24 << 20, seed=6, vocab=70_000)
            e.count_resident(24 << 20, global_base=24 << 20)  # B follows A in one logical stream
            got = e.result()
        want = merge_results([ops.cpu_count_synth(24 << 20, 0, 5, 50_000, 1.0, 0, 16),
                              ops.cpu_count_synth(24 << 20, 0, 6, 70_000, 1.0, 24 << 20, 16)])
        assert_same(got, want)
