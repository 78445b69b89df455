"""ctypes binding of the native engine ``lib/libwc.so`` (C ABI: include/wc/wc.h).

The shared library is built in-tree (``make`` / ``__graft_entry__.build()``) and
loaded from ``cuda_mapreduce_amd/lib``.  There is deliberately NO Python
fallback: if the library is missing the import fails loudly, so a GPU run can
never silently pass on an eager re-implementation.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char, c_char_p, c_double, c_int, c_uint32, c_uint64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
# WC_LIB selects another in-tree build of the engine (tuning variants, tools/variants.sh).
LIB_PATH = os.environ.get("WC_LIB") or os.path.join(os.path.dirname(_HERE), "lib", "libwc.so")


class WcError(RuntimeError):
    """Error raised by the native engine (message from wc_last_error)."""


class Options(ctypes.Structure):
    _fields_ = [
        ("device", ctypes.c_int32),
        ("log2_rec_buckets", c_uint32),
        ("log2_tab_buckets", c_uint32),
        ("max_log2_tab_buckets", c_uint32),
        ("map_blocks", c_uint32),
        ("staging_buffers", c_uint32),
        ("chunk_bytes", c_uint64),
        ("arena_bytes", c_uint64),
        ("min_records", c_uint64),
        ("records_per_byte", c_double),
        ("merge_mode", c_uint32),  # 0 shuffle (all-to-all by key owner), 1 dense reduce-scatter
        ("k1_hash_bits", c_uint32),  # tests: LONG-word hash bits kept (0 = all) to force collisions
    ]


def _load() -> ctypes.CDLL:
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"native engine not built: {LIB_PATH} is missing; run `make -j8` in the repo root "
            "or `python -c 'import __graft_entry__ as g; g.build()'`"
        )
    lib = ctypes.CDLL(LIB_PATH)
    P8 = POINTER(ctypes.c_uint8)
    P64 = POINTER(c_uint64)
    sig = {
        "wc_last_error": (c_char_p, []),
        "wc_version": (c_char_p, []),
        "wc_device_count": (c_int, []),
        "wc_debug_radix_sort": (c_int, [c_int, P64, c_uint64, c_int, P64, POINTER(ctypes.c_uint32)]),
        "wc_bench_radix_sort": (c_int, [c_int, P64, c_uint64, c_int, c_int, POINTER(ctypes.c_double)]),
        "wc_debug_first_order": (c_int, [c_int, P64, c_uint64, c_int, P64, POINTER(ctypes.c_uint32),
                                         POINTER(c_int), POINTER(ctypes.c_double)]),
        "wc_debug_read_file": (c_int, [c_char_p, c_uint64, c_uint64, c_uint64, P8, POINTER(c_uint64)]),
        "wc_debug_order": (c_int, [c_int, c_int, P64, c_uint64, c_int, P64, POINTER(ctypes.c_uint32),
                                   POINTER(c_int), POINTER(ctypes.c_double), P64]),
        "wc_default_options": (None, [POINTER(Options)]),
        "wc_engine_create": (c_void_p, [POINTER(Options)]),
        "wc_engine_destroy": (None, [c_void_p]),
        "wc_engine_reset": (c_int, [c_void_p]),
        "wc_engine_set_stage_events": (c_int, [c_void_p, c_int]),
        "wc_job_resident": (c_int, [c_void_p, c_uint64, c_uint64, c_void_p, POINTER(c_uint64)]),
        "wc_count_host": (c_int, [c_void_p, P8, c_uint64, c_uint64]),
        "wc_count_file": (c_int, [c_void_p, c_char_p, c_uint64, c_uint64, c_uint64]),
        "wc_count_file_checkpointed": (c_void_p, [c_void_p, c_char_p, c_uint64, c_uint64, c_int, c_int, c_char_p,
                                                   c_uint64, c_int]),
        "wc_result_merge": (c_int, [c_void_p, c_void_p]),
        "wc_count_replay": (c_int, [c_void_p, P8, c_uint64, c_uint64, c_uint64]),
        "wc_count_pinned_replay": (c_int, [c_void_p, P8, c_uint64, c_uint64, c_uint64]),
        "wc_synth_device": (c_int, [c_void_p, c_uint64, c_uint64, c_uint64, c_uint32, c_double, c_double]),
        "wc_count_resident": (c_int, [c_void_p, c_uint64, c_uint64]),
        "wc_finalize_device": (c_int, [c_void_p, c_void_p, P64]),
        "wc_engine_result": (c_void_p, [c_void_p, c_void_p, c_int]),
        "wc_engine_stats_json": (c_int, [c_void_p, c_char_p, c_int]),
        "wc_engine_sync": (c_int, [c_void_p]),
        "wc_result_size": (c_uint64, [c_void_p]),
        "wc_result_total": (c_uint64, [c_void_p]),
        "wc_result_bytes": (c_uint64, [c_void_p]),
        "wc_result_export": (None, [c_void_p, P64, P64, P64, POINTER(c_char)]),
        "wc_result_free": (None, [c_void_p]),
        "wc_format": (c_int, [c_void_p, P8, c_uint64, c_int, c_int, c_uint64, POINTER(c_void_p), P64]),
        "wc_free": (None, [c_void_p]),
        "wc_cpu_count": (c_void_p, [P8, c_uint64, c_uint64]),
        "wc_key_owner": (c_uint32, [P8, c_uint64, c_uint32]),
        "wc_debug_comm_counters": (None, [P64, P64]),
        "wc_debug_loopback_async": (c_int, [c_int, POINTER(c_int), POINTER(c_int), POINTER(c_int)]),
        "wc_cpu_count_compat": (c_void_p, [P8, c_uint64]),
        "wc_synth_host": (c_int, [P8, c_uint64, c_uint64, c_uint64, c_uint32, c_double]),
        "wc_synth_host_mt": (c_int, [P8, c_uint64, c_uint64, c_uint64, c_uint32, c_double, c_double, c_int]),
        "wc_cpu_count_synth": (c_void_p, [c_uint64, c_uint64, c_uint64, c_uint32, c_double, c_double, c_uint64, c_int]),
        "wc_pool_create": (c_void_p, [c_uint64, c_uint64, c_uint64, c_uint32, c_double, c_double, c_int, c_int]),
        "wc_pool_numa_node": (c_int, [c_void_p]),
        "wc_numa_of_pci": (c_int, [c_char_p, c_char_p, POINTER(c_int), POINTER(c_int), c_int]),
        "wc_h2d_bench": (c_int, [c_int, c_int, c_uint64, c_int, POINTER(c_double), POINTER(c_int)]),
        "wc_file_read_bench": (c_int, [c_char_p, c_uint64, c_int, POINTER(c_double), P64]),
        "wc_pool_destroy": (None, [c_void_p]),
        "wc_pool_build_seconds": (c_double, [c_void_p]),
        "wc_count_pool": (c_int, [c_void_p, c_void_p, c_uint64, c_uint64]),
        "wc_shard_range_mem": (c_int, [P8, c_uint64, c_int, c_int, P64, P64]),
        "wc_shard_range_file": (c_int, [c_char_p, c_int, c_int, P64, P64]),
        "wc_rccl_unique_id": (c_int, [POINTER(c_char)]),
        "wc_comm_rccl_create": (c_void_p, [POINTER(c_char), c_int, c_int, c_int]),
        "wc_comm_destroy": (None, [c_void_p]),
        "wc_comm_barrier": (c_int, [c_void_p]),
        "wc_comm_allgather_host": (c_int, [c_void_p, c_void_p, c_uint64, c_void_p]),
        "wc_loopback_count": (c_void_p, [P8, c_uint64, c_int, POINTER(c_int), POINTER(Options), c_int, c_int, P8,
                                         c_uint64]),
        "wc_virtual_bench": (c_void_p, [POINTER(Options), c_int, c_int, c_uint64, c_uint64, c_uint32, c_double, c_double,
                                        c_int, c_int, POINTER(c_double)]),
    }
    for name, (res, args) in sig.items():
        if not hasattr(lib, name):
            continue  # an older A/B variant build (WC_LIB) without this entry point: calling it raises
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def last_error() -> str:
    msg = lib.wc_last_error()
    return msg.decode(errors="replace") if msg else "unknown error"


def check(rc: int) -> None:
    if rc != 0:
        raise WcError(last_error())


def check_ptr(p):
    if not p:
        raise WcError(last_error())
    return p
