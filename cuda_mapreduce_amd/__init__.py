"""cuda_mapreduce_amd — MI355X-native GPU MapReduce word count.

Capability parity with zimisoho/cuda-mapreduce (/root/reference/main.cu): count
whitespace-delimited words, report ``word<TAB>count`` in first-occurrence order
and the total.  The compute path is hand-written HIP for gfx950 (CDNA4) in
``src/kernels``; multi-GPU merges use RCCL over xGMI (``src/dist``).

Layout:
  ops/       ctypes binding of the native engine (lib/libwc.so) + CPU paths
  models/    job definitions: the BASELINE word-count configurations
  parallel/  one-process-per-GPU driver: torch.distributed rendezvous, RCCL
             communicator, shard ownership, host (gloo) merge for CPU runs
"""
from .ops import Engine, Result, cpu_count, cpu_count_compat, format_output, synth_host  # noqa: F401

__version__ = "0.1.0"
