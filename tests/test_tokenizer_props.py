"""Property tests of the tokenizer semantics (hypothesis): the native CPU oracle
against a pure-Python definition of the clean semantics (delimiters
exactly {' ', '\\r', '\\n'}, empty tokens ignored, exact byte equality, first-
occurrence order, a final word without newline counted) on arbitrary bytes —
TAB, NUL, punctuation and high bytes are word bytes."""
import pytest

hypothesis = pytest.importorskip("hypothesis")
from hypothesis import given, settings, strategies as st  # noqa: E402

ops = pytest.importorskip("cuda_mapreduce_amd.ops")

DELIMS = b" \r\n"


def py_count(text: bytes):
    order, counts = [], {}
    word = bytearray()
    for c in text + b" ":
        if c in DELIMS:
            if word:
                w = bytes(word)
                if w not in counts:
                    order.append(w)
                    counts[w] = 0
                counts[w] += 1
                word.clear()
        else:
            word.append(c)
    return [(w, counts[w]) for w in order]


alphabet = st.sampled_from(list(b"ab \r\n\t\x00,\xffZ"))


@settings(max_examples=300, deadline=None)
@given(st.lists(alphabet, max_size=400).map(bytes))
def test_cpu_oracle_matches_python_definition(text):
    res = ops.cpu_count(text)
    assert [(w, int(c)) for w, c in zip(res.words, res.counts)] == py_count(text)
    assert res.total == sum(c for _, c in py_count(text))


@settings(max_examples=100, deadline=None)
@given(st.lists(st.sampled_from([b"aaaaaaaa", b"aaaaaaaab", b"a" * 17, b"x", b"x\x00", b"\x00"]), max_size=60),
       st.sampled_from([b" ", b"\n", b"\r\n", b"  "]))
def test_long_and_nul_words_are_distinct_keys(words, sep):
    """Words sharing their first 8 bytes, or differing only by NUL padding, stay distinct."""
    text = sep.join(words)
    res = ops.cpu_count(text)
    assert [(w, int(c)) for w, c in zip(res.words, res.counts)] == py_count(text)
