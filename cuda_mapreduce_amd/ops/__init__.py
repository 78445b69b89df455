"""Native MapReduce ops: the HIP/CDNA4 engine (map / shuffle / reduce kernels), CPU paths."""
from .engine import (  # noqa: F401
    Comm,
    Engine,
    HostPool,
    Result,
    cpu_count,
    cpu_count_synth,
    cpu_count_compat,
    cpu_count_file_checkpointed,
    default_options,
    device_count,
    format_output,
    loopback_count,
    virtual_bench,
    numa_of_pci,
    h2d_bench,
    file_read_bench,
    shard_range,
    shard_range_file,
    synth_host,
    synth_host_array,
)
from ._lib import LIB_PATH, WcError  # noqa: F401
