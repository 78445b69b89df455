"""Words longer than a whole host stream piece (SURVEY §5.7 long-word fallback).

The streaming path cuts host pieces at their last delimiter; a piece with no
delimiter at all is the start of a word longer than the piece.  Its bytes are
gathered up to the next delimiter and counted as a pass of its own
(src/engine/engine.cpp count_source / count_giant).  Every case is compared
exactly (words, first-occurrence order, counts, first offsets, total) with the
CPU oracle.  Engine pieces are 32 KiB here (chunk_bytes), so the giant words are
40 KiB - 300 KiB: at the stream start, in the middle, adjacent, repeated (the
second occurrence is merged with the first by the byte comparison of LONG
words), and running to the end of the input without a trailing delimiter."""
import pytest

pytestmark = pytest.mark.gpu
ops = pytest.importorskip("cuda_mapreduce_amd.ops")

PIECE = 1 << 15


def giant(n, seed):
    return bytes(97 + (i * 7 + seed * 13 + (i >> 5)) % 26 for i in range(n))


def cases():
    g1, g2, g3 = giant(40_000, 1), giant(PIECE * 3 + 17, 2), giant(300_000, 3)
    body = b"the cat sat on the mat\n" * 500
    return {
        "start": g1 + b" " + body,
        "middle": body + g2 + b"\n" + body,
        "adjacent": body + g1 + b" " + g2 + b"  " + g3 + b"\r\n" + body,
        "repeated": g2 + b" " + body + g2 + b" x " + g2,
        "end_no_delimiter": body + b" " + g3,
        "exactly_one_piece": body[: PIECE - 1] + b" " + giant(PIECE, 4) + b" tail",
    }


@pytest.fixture(scope="module")
def eng():
    with ops.Engine(device=0, chunk_bytes=PIECE) as e:
        yield e


@pytest.mark.parametrize("name", list(cases()))
def test_giant_word_matches_cpu_oracle(eng, name):
    text = cases()[name]
    eng.reset()
    eng.count_bytes(text)
    got = eng.result()
    want = ops.cpu_count(text)
    assert got.words == want.words
    assert list(got.counts) == list(want.counts)
    assert list(got.first_off) == list(want.first_off)
    assert got.total == want.total
