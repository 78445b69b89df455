"""Split reduce (src/kernels/reduce.hip): while the table has fewer buckets than
CUs, each bucket is reduced by several blocks over interleaved map-block runs
into partial tables that the last block of the bucket merges.  Every block
count per bucket — one (the classic reduce), two, a non-power-of-two three,
and the clamp at the partial-table area — must give the byte-keyed CPU
oracle's table exactly, for inline and LONG (byte-verified) words, in one pass
and over several passes, and through table overflows that split the table and
re-run buckets mid-pass."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ops = pytest.importorskip("cuda_mapreduce_amd.ops")


def assert_same(got, want):
    assert got.total == want.total
    assert got.words == want.words
    assert np.array_equal(got.counts, want.counts)
    assert np.array_equal(got.first_off, want.first_off)


@pytest.mark.parametrize("red_q", ["1", "2", "3", "16"])
@pytest.mark.parametrize("chunk", [64 << 20, 16 << 20])
def test_split_reduce_blocks_per_bucket(red_q, chunk, monkeypatch):
    monkeypatch.setenv("WC_RED_Q", red_q)  # read when the engine is built
    n = 64 << 20
    want = ops.cpu_count_synth(n, 0, 11, 200_000, 1.0, 0, 16, 0.2)
    # 16 table buckets to start: Q up to the 16 the partial-table area allows, and 200k words
    # overflow it (splits + bucket re-runs inside the first pass)
    with ops.Engine(device=0, chunk_bytes=chunk, log2_tab_buckets=4, log2_rec_buckets=4) as e:
        e.synth_device(n, first_segment=0, seed=11, vocab=200_000, zipf_s=1.0, long_frac=0.2)
        e.count_resident(n)
        got = e.result()
        st = e.stats()
    assert st["table_splits"] >= 1
    assert_same(got, want)
