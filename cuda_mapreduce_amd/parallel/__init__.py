"""Data parallelism across GPUs: torch-free launcher / rendezvous (launch.py),
torch.distributed helpers (dist.py), native RCCL merge."""
_DIST = ("CommFault", "DistEnv", "DistributedWordCount", "comm_timeout_s", "host_merge", "init_from_env", "rccl_comm",
         "gather_merge")


def __getattr__(name):
    # Lazy: `parallel.launch` must be importable without loading the native engine.
    if name in _DIST:
        from . import dist

        return getattr(dist, name)
    raise AttributeError(f"module {__name__!r} has no attribute {name!r}")
