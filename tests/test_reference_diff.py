"""Differential test against the reference program itself.

The reference (/root/reference/main.cu) cannot be compiled for a GPU here, so
the test builds a HOST EMULATION of it at test time, in a temp dir: a shim
`cuda_runtime.h` maps cudaMalloc/Memcpy/Memset/Free to host memory (calloc =
the zero-filled device memory the reference relies on) and
the two `<<< >>>` launch lines are rewritten into loops running every thread of
the grid serially (exact: mapKernel threads write disjoint records and
reduceKernel works on thread 0 only).  Nothing of the reference is copied into
this repository; the test is skipped where the reference is not mounted (e.g.
on the GPU box).

Random inputs are drawn inside the reference's safe envelope (<= 9 lines, <= 20
tokens per line, tokens <= 19 bytes, <= 10 distinct words, trailing LF) and
the emulated reference's stdout is compared byte for byte with
  * `wordcount --compat=reference` (quirks mode: prefix compare, fgets records),
  * `wordcount --cpu` (clean semantics) when no word is a prefix of another
    and the input has single spaces only — where the two semantics coincide.
"""
import os
import re
import shutil
import subprocess

import numpy as np
import pytest

from conftest import ROOT

REF = "/root/reference/main.cu"
EXE = os.path.join(ROOT, "wordcount")

SHIM = r"""
#pragma once
#include <cstdlib>
#include <cstring>
#define __global__
#define __device__
#define __host__
typedef int cudaError_t;
enum cudaMemcpyKind { cudaMemcpyHostToDevice = 1, cudaMemcpyDeviceToHost = 2 };
template <class T> inline cudaError_t cudaMalloc(T** p, size_t n) { *p = (T*)calloc(1, n); return 0; }
inline cudaError_t cudaFree(void* p) { free(p); return 0; }
inline cudaError_t cudaMemcpy(void* d, const void* s, size_t n, cudaMemcpyKind) { memcpy(d, s, n); return 0; }
inline cudaError_t cudaMemset(void* p, int v, size_t n) { memset(p, v, n); return 0; }
struct wc_dim { unsigned x; };
static wc_dim threadIdx, blockIdx, blockDim, gridDim;
#define WC_LAUNCH(kernel, g, b, ...)                                         \
  for (unsigned wc_b = 0; wc_b < (unsigned)(g); ++wc_b)                     \
    for (unsigned wc_t = 0; wc_t < (unsigned)(b); ++wc_t) {                 \
      blockIdx.x = wc_b; threadIdx.x = wc_t; blockDim.x = (b); gridDim.x = (g); \
      kernel(__VA_ARGS__);                                                  \
    }
"""


@pytest.fixture(scope="module")
def ref_exe(tmp_path_factory):
    if not os.path.exists(REF):
        pytest.skip("reference not mounted")
    if shutil.which("g++") is None:
        pytest.skip("no host compiler")
    d = tmp_path_factory.mktemp("refemu")
    src = open(REF, encoding="latin-1").read()
    src, n = re.subn(r"(\w+)\s*<<\s*<\s*(\w+)\s*,\s*(\w+)\s*>>\s*>\s*\((.*?)\);", r"WC_LAUNCH(\1, \2, \3, \4);", src)
    assert n == 2, "expected the two kernel launches of the reference"
    (d / "cuda_runtime.h").write_text(SHIM)
    (d / "main.cpp").write_text(src, encoding="latin-1")
    out = subprocess.run(["g++", "-O1", "-w", "-I", str(d), "-o", str(d / "ref"), str(d / "main.cpp")],
                         capture_output=True, timeout=120)
    if out.returncode != 0:
        pytest.skip("reference emulation did not compile: " + out.stderr.decode()[-300:])
    return str(d / "ref")


def run_in(cwd, argv, text):
    with open(os.path.join(cwd, "test.txt"), "wb") as f:
        f.write(text)
    out = subprocess.run(argv, cwd=cwd, capture_output=True, timeout=60)
    assert out.returncode == 0, out.stderr
    return out.stdout


def envelope_text(rng, vocab, max_lines=9, max_words=6):
    lines = []
    for _ in range(int(rng.integers(1, max_lines + 1))):
        words = [vocab[i] for i in rng.integers(0, len(vocab), int(rng.integers(1, max_words + 1)))]
        lines.append(b" ".join(words) + b"\n")
    return b"".join(lines)


def test_golden_matches_reference(ref_exe, tmp_path, golden_text):
    want = run_in(tmp_path, [ref_exe], golden_text)
    assert run_in(tmp_path, [EXE, "--cpu"], golden_text) == want
    assert run_in(tmp_path, [EXE, "--compat=reference"], golden_text) == want


def test_compat_mode_matches_reference_with_prefix_words(ref_exe, tmp_path):
    """Prefix words ('Go' / 'Good'), TABs and CRLF exercise the reference's quirks."""
    rng = np.random.default_rng(7)
    vocab = [b"Go", b"Good", b"a", b"ab", b"abc", b"b\tc", b"x", b"Hello", b"hello,", b"W"]
    for _ in range(40):
        t = envelope_text(rng, vocab)
        if rng.integers(0, 4) == 0:
            t = t.replace(b"\n", b"\r\n")
        want = run_in(tmp_path, [ref_exe], t)
        assert run_in(tmp_path, [EXE, "--compat=reference"], t) == want, t


def test_clean_mode_matches_reference_inside_envelope(ref_exe, tmp_path):
    rng = np.random.default_rng(11)
    vocab = [b"alpha", b"beta", b"gamma", b"delta", b"eps", b"zeta", b"Eta", b"theta,", b"iota!", b"kappa\t1"]
    for _ in range(40):
        t = envelope_text(rng, vocab)
        want = run_in(tmp_path, [ref_exe], t)
        assert run_in(tmp_path, [EXE, "--cpu"], t) == want, t


def test_compat_mode_echo_stops_at_blank_line(ref_exe, tmp_path):
    """A blank line ends the reference's input (main.cu:185-186): the echo stops there too."""
    rng = np.random.default_rng(23)
    vocab = [b"one", b"two", b"three", b"four", b"Go", b"Good"]
    for _ in range(20):
        head = envelope_text(rng, vocab, max_lines=4)
        tail = envelope_text(rng, vocab, max_lines=4)
        t = head + b"\n" + tail  # the blank line hides `tail` from the reference
        want = run_in(tmp_path, [ref_exe], t)
        got = run_in(tmp_path, [EXE, "--compat=reference"], t)
        assert got == want, t
        assert tail not in got.split(b"-" * 26)[0][len(b"Input Data:\n") + len(head):]
