import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pytest_sessionstart(session):
    # The native library and CLI are git-ignored build products: build them in-tree
    # when a fresh checkout runs the suite (a no-op when `make` / build() already ran).
    import subprocess

    lib = os.path.join(ROOT, "cuda_mapreduce_amd", "lib", "libwc.so")
    exe = os.path.join(ROOT, "wordcount")
    if not (os.path.exists(lib) and os.path.exists(exe)):
        jobs = str(min(16, os.cpu_count() or 8))
        subprocess.run(["make", "-C", ROOT, f"-j{jobs}", "all"], check=True, capture_output=True)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on a GPU box)")


@pytest.fixture(scope="session")
def golden_text():
    with open(os.path.join(ROOT, "tests", "data", "test.txt"), "rb") as f:
        return f.read()


GOLDEN_OUTPUT = (
    b"Input Data:\nHello World EveryOne\nWorld Good News\nGood Morning Hello\n"
    b"--------------------------\nHello\t2\nWorld\t2\nEveryOne\t1\nGood\t2\nNews\t1\nMorning\t1\n"
    b"--------------------------\nTotal Count:9\n"
)
