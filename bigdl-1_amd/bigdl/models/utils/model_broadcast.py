"""``ModelBroadcast`` (``DL/models/utils/ModelBroadcast.scala:51-277``): make every rank hold the
same model.  The reference Spark-broadcasts the weight-stripped graph plus the weights and clones
replicas that share them; here each rank builds the model (same code) and rank 0's parameters
and buffers are broadcast with RCCL (one collective per tensor group), so the replicas are
bit-identical (X1 of the collective inventory)."""
from __future__ import annotations


class ModelBroadcast:
    def __init__(self, apply_protobuf: bool = False):
        self.applyProtoBuffer = apply_protobuf
        self._model = None

    def broadcast(self, sc, model, src: int = 0):
        from ...parallel import comm
        comm.broadcast_module(model, src)
        self._model = model
        return self

    def value(self, init_gradient: bool = False, share_weight: bool = True):
        m = self._model if share_weight else self._model.cloneModule()
        if init_gradient:
            m.zeroGradParameters()
        return m


class CachedModels:
    """Per-process cache of model replicas keyed by a broadcast id (``ModelBroadcast.scala:301-349``):
    the reference keeps executor-side clones so repeated ``value()`` calls share weights and a
    finished job can drop them.  ``add`` registers a replica under ``uuid``; ``delete_key`` /
    ``delete_all(current)`` release replicas (their parameter storage goes back to the caching
    allocator)."""

    _cache = {}

    @classmethod
    def add(cls, uuid: str, model) -> None:
        cls._cache.setdefault(uuid, []).append(model)

    @classmethod
    def get(cls, uuid: str):
        return list(cls._cache.get(uuid, []))

    @classmethod
    def delete_key(cls, uuid: str) -> None:
        cls._cache.pop(uuid, None)

    @classmethod
    def delete_all(cls, current: str = None) -> None:
        for k in list(cls._cache):
            if k != current:
                del cls._cache[k]

    deleteKey = delete_key
    deleteAll = delete_all
