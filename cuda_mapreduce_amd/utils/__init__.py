"""Helpers shared by the Python entry points (bench.py, tests)."""
from .validate import compare_results, merge_results, synthetic_oracle  # noqa: F401
