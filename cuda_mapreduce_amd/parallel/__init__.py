"""Data parallelism across GPUs: torch.distributed rendezvous + native RCCL merge."""
from .dist import DistEnv, DistributedWordCount, host_merge, init_from_env, rccl_comm  # noqa: F401
