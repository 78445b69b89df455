import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


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
