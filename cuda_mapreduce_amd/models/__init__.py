"""Job definitions (the BASELINE.json word-count configurations)."""
from .wordcount import CONFIGS, JobConfig, JobResult, run_job  # noqa: F401
