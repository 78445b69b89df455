"""GPU property tests (hypothesis): the native engine on arbitrary byte strings
equals the pure-Python definition of the clean semantics, across chunk, unit and
lane boundaries (32 KiB chunks; inputs up to ~100 KiB; long words straddling)."""
import pytest

hypothesis = pytest.importorskip("hypothesis")
from hypothesis import HealthCheck, given, settings, strategies as st  # noqa: E402

from test_tokenizer_props import py_count  # noqa: E402

pytestmark = pytest.mark.gpu
ops = pytest.importorskip("cuda_mapreduce_amd.ops")

_ENG = {}


def engine():
    if "e" not in _ENG:
        _ENG["e"] = ops.Engine(device=0, chunk_bytes=1 << 15)
    return _ENG["e"]


piece = st.one_of(
    st.lists(st.sampled_from(list(b"ab \n\t\x00Z,")), max_size=64).map(bytes),
    st.integers(1, 300).map(lambda n: b"w" * n),          # long words (lane window, halo, units)
    st.integers(1, 40).map(lambda n: b" " * n),           # delimiter runs
    st.sampled_from([b"the", b"of", b"and", b"\r\n", b"abcdefgh", b"abcdefghi"]),
)


@settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(st.lists(piece, max_size=400).map(b"".join), st.integers(0, 3))
def test_engine_matches_python_definition(text, reps):
    text = text * (1 + reps * 40)  # up to ~100 KiB: several chunks
    e = engine()
    e.reset()
    # words longer than a 32 KiB host piece take the giant-word pass (tests/test_gpu_giant.py)
    e.count_bytes(text)
    got = e.result()
    want = py_count(text)
    assert [(w, int(c)) for w, c in zip(got.words, got.counts)] == want
