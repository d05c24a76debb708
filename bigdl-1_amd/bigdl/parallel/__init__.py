"""Multi-GPU execution: one process per GPU, RCCL (``torch.distributed`` backend "nccl") over xGMI."""
from .comm import is_dist, world, rank, bf16_truncate, broadcast_module, barrier, allreduce_scalar
from .distri_optimizer import DistriOptimizer, ParallelOptimizer
