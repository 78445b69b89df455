"""Data parallelism across GPUs: torch.distributed rendezvous + native RCCL merge."""
from .dist import (CommFault, DistEnv, DistributedWordCount, comm_timeout_s, host_merge, init_from_env,  # noqa: F401
                   rccl_comm)
