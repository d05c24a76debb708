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
