"""cuda_mapreduce_amd — MI355X-native GPU MapReduce word count.

Capability parity with zimisoho/cuda-mapreduce (/root/reference/main.cu): count
whitespace-delimited words, report ``word<TAB>count`` in first-occurrence order
and the total.  The compute path is hand-written HIP for gfx950 (CDNA4) in
``src/kernels``; multi-GPU merges use RCCL over xGMI (``src/dist``).

Layout:
  ops/       ctypes binding of the native engine (lib/libwc.so) + CPU paths
  models/    job definitions: the BASELINE word-count configurations
  parallel/  one-process-per-GPU driver: torch-free launcher + file rendezvous
             (launch.py), torch.distributed helpers, RCCL communicator, shard
             ownership, host (gloo) merge for CPU runs
"""
__version__ = "0.1.0"

_OPS = ("Engine", "Result", "cpu_count", "cpu_count_compat", "format_output", "synth_host")


def __getattr__(name):
    # Lazy: importing the package (e.g. parallel.launch in a launcher process that
    # must never touch a GPU) does not load lib/libwc.so and its HIP runtime.
    if name in _OPS:
        from . import ops

        return getattr(ops, name)
    raise AttributeError(f"module {__name__!r} has no attribute {name!r}")
