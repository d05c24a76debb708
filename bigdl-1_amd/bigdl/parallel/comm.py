"""Communication primitives over RCCL (xGMI) / gloo.

The reference's parameter exchange is a Spark BlockManager all-reduce built from bf16-truncated
shards (``DL/parameters/AllReduceParameter.scala:138-328``, ``FP16CompressedTensor.scala:43-277``).
Here the same algorithm — reduce-scatter, shard-local update, all-gather — maps one-to-one onto
RCCL collectives issued per gradient bucket.  Helpers:

* :func:`bf16_truncate` — the reference wire format (top 16 bits of the fp32, no rounding;
  golden value 1.111111 → 1.109375, ``TS/parameters/FP16ParameterSpec.scala:50-66``).
* :func:`broadcast_module` — rank-0 initial weights + buffers to every rank (X1 / X14).
* :func:`barrier` / :func:`allreduce_scalar` — control-plane helpers (X7).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def is_dist() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def world() -> int:
    return dist.get_world_size() if is_dist() else 1


def rank() -> int:
    return dist.get_rank() if is_dist() else 0


def bf16_truncate(x: torch.Tensor) -> torch.Tensor:
    """fp32 → bf16 by dropping the low 16 bits (reference compat mode, no rounding)."""
    i = x.float().contiguous().view(torch.int32)
    return (i >> 16).to(torch.int16).view(torch.bfloat16)


def bf16_expand(x: torch.Tensor) -> torch.Tensor:
    return x.float()


def broadcast_module(module, src: int = 0):
    if not is_dist():
        return
    p = module.parameters()
    arena = module.flat_parameters()
    from ..ops import fp32x3
    if arena is not None:
        dist.broadcast(arena.weight, src)
        fp32x3.mark_dirty(arena.weight)  # a collective writes behind torch's version counters
    elif p is not None:
        for w in p[0]:
            dist.broadcast(w.data, src)
            fp32x3.mark_dirty(w)
    ex = module.getExtraParameter()
    if ex:
        for b in ex:
            dist.broadcast(b, src)


def barrier():
    if is_dist():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def allreduce_scalar(t: torch.Tensor, average: bool = True) -> torch.Tensor:
    if not is_dist():
        return t
    t = t.clone()
    dist.all_reduce(t)
    if average:
        t /= dist.get_world_size()
    return t


def allreduce_max(v: float) -> float:
    if not is_dist():
        return v
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([v], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
