"""Batch inference and serving.

* ``LocalPredictor`` (``DL/optim/LocalPredictor.scala:33-197``): ``predict``, ``predict_class``,
  ``predict_image`` over arrays of Samples / MiniBatch datasets / ImageFrames.
* ``Predictor`` (``DL/optim/Predictor.scala:35-257``): the distributed form — every rank predicts
  its shard of the dataset (the reference's RDD partitions) and results are returned per rank or
  gathered to rank 0.
* ``PredictionService`` (``DL/optim/PredictionService.scala:56-354``): thread-safe serving with a
  pool of ``num_threads`` weight-sharing model instances.  On a GPU each instance runs on its own
  HIP stream, so up to ``num_threads`` requests are in flight on the device at once; requests and
  replies can be raw bytes in the reference's ``AttrValue`` protobuf encoding.

Batching uses the device the model lives on; inputs are moved there asynchronously (pinned host
buffers), and the model runs in eval mode under ``torch.no_grad``.
"""
from __future__ import annotations

import queue
import threading
from typing import List, Optional, Sequence

import numpy as np
import torch

from ..dataset import MiniBatch, Sample, SampleToMiniBatch
from ..utils.engine import Engine
from ..utils.table import Table


def _model_device(model) -> torch.device:
    p = model.parameters()
    if p is not None and p[0]:
        return p[0][0].device
    for b in (model.getExtraParameter() or []):
        return b.device
    return Engine.device()


def _split_batch(out, n: int) -> List:
    """``Predictor.splitBatch``: one activity per sample (views of the batch output)."""
    if isinstance(out, torch.Tensor):
        return [out[i] for i in range(n)]
    if isinstance(out, Table):
        parts = [_split_batch(v, n) for v in out.values()]
        keys = list(out.keys())
        res = []
        for i in range(n):
            t = Table()
            for k, p in zip(keys, parts):
                t[k] = p[i]
            res.append(t)
        return res
    raise TypeError(f"unsupported activity {type(out)}")


def _to_host(a):
    if isinstance(a, torch.Tensor):
        a = a.detach()
        if a.dtype in (torch.bfloat16, torch.float16):
            a = a.float()
        return a.cpu()
    if isinstance(a, Table):
        t = Table()
        for k, v in a.items():
            t[k] = _to_host(v)
        return t
    return a


def _batches(data, batch_size: int):
    """Samples / ndarrays / MiniBatches / datasets → MiniBatch iterator."""
    from ..dataset import AbstractDataSet
    if isinstance(data, AbstractDataSet):
        yield from data.data(train=False)
        return
    if isinstance(data, MiniBatch):
        yield data
        return
    if isinstance(data, (np.ndarray, torch.Tensor)):
        data = [Sample(d) for d in data]
    data = list(data)
    if data and isinstance(data[0], MiniBatch):
        yield from data
        return
    yield from SampleToMiniBatch(batch_size if batch_size > 0 else max(1, len(data)))(iter(data))


class LocalPredictor:
    """``compiled`` (default ``bigdl.predict.compiled`` = on): on a GPU the model is lowered through
    the IR once (``ConversionUtils.convert``: BN folded, conv+sum+ReLU epilogues — the reference's
    LocalPredictor converts every model, ``LocalPredictor.scala:66``), each distinct batch shape is
    planned once and its forward captured into a HIP graph (``nn/compiled.py``); later batches of
    that shape are a copy-in plus one graph replay.  The lowered graph holds folded weights taken at
    the first prediction: :meth:`refresh` drops it after the model's weights change."""

    def __init__(self, model, feature_padding=None, batch_size: int = -1, compiled: Optional[bool] = None):
        self.model = model
        self.batch_size = batch_size if batch_size > 0 else 4 * max(1, Engine.core_number())
        self.feature_padding = feature_padding
        self.compiled = compiled
        self._graphs = {}

    @staticmethod
    def create(model, batch_size=-1, feature_padding=None):
        return LocalPredictor(model, feature_padding, batch_size)

    def refresh(self):
        """Forget the lowered / captured forms (after the model's weights changed)."""
        self._graphs = {}
        self.__dict__.pop("_lowered", None)

    def _run(self, m, x, eager: bool = False):
        from ..utils import config
        use = self.compiled if self.compiled is not None else bool(config.get_property("bigdl.predict.compiled"))
        if eager or not (use and isinstance(x, torch.Tensor) and x.is_cuda):
            return m.forward(x)
        key = (tuple(x.shape), x.dtype)
        c = self._graphs.get(key)
        if c is None:
            from ..nn.compiled import compile as compile_module, _lower
            low = self.__dict__.get("_lowered")
            if low is None:  # one IR lowering per predictor, shared by every batch shape
                low = self.__dict__["_lowered"] = _lower(m, None)
            c = self._graphs[key] = compile_module(low, x, lower=False)
        return c(x)

    def _forward_all(self, data, eager: bool = False):
        m = self.model
        dev = _model_device(m)
        was_training = m.isTraining()
        m.evaluate()
        if dev.type == "cuda":
            from ..nn.fusion import fuse
            fuse(m)  # conv+ReLU epilogues, zero-copy concats (idempotent)
        outs = []
        try:
            with torch.no_grad():
                for b in _batches(data, self.batch_size):
                    b = b.to(dev, dtype=Engine.compute_dtype() if dev.type == "cuda" else None)
                    out = self._run(m, b.getInput(), eager)
                    outs.extend(_split_batch(_to_host(out), b.size()))
        finally:
            if was_training:
                m.training()
        return outs

    def predict(self, data) -> List:
        """One output Activity per input sample."""
        return self._forward_all(data)

    def predict_class(self, data) -> np.ndarray:
        """1-based arg-max class per sample (``LocalPredictor.predictClass``)."""
        outs = self._forward_all(data)
        return np.array([int(torch.argmax(o.reshape(-1)).item()) + 1 for o in outs], dtype=np.int64)

    predictClass = predict_class

    def predict_image(self, image_frame, output_layer: Optional[str] = None, share_buffer: bool = False,
                      predict_key: str = "predict"):
        """Run the model over an ImageFrame's ``sample`` entries and store each output under
        ``predict_key`` (``LocalPredictor.predictImage``)."""
        feats = image_frame.to_local().array if hasattr(image_frame, "to_local") else list(image_frame)
        samples = [f.get_sample() for f in feats]
        # an intermediate layer's output exists only on the unlowered model: run it eagerly then
        outs = self._forward_all(samples, eager=output_layer is not None)
        if output_layer is not None:
            layer = self.model.flattened_modules()
            target = [l for l in layer if l.get_name() == output_layer]
            if target:
                outs = _split_batch(_to_host(target[0].output), len(samples)) if len(samples) else []
        for f, o in zip(feats, outs):
            f[predict_key] = o if share_buffer else (o.clone() if isinstance(o, torch.Tensor) else o)
        return image_frame

    predictImage = predict_image

    def shutdown(self):
        pass


class Predictor(LocalPredictor):
    """Distributed predictor: each rank predicts its shard; ``gather=True`` collects to rank 0
    (the reference returns an RDD that stays partitioned)."""

    def __init__(self, model, feature_padding=None, batch_per_partition: int = 4, batch_size: int = -1):
        super().__init__(model, feature_padding, batch_size)
        self.batch_per_partition = batch_per_partition

    def predict(self, data, batch_size: int = -1, share_buffer: bool = False, gather: bool = False):
        if batch_size > 0:
            self.batch_size = batch_size
        outs = super().predict(data)
        if gather and Engine.is_distributed():
            import torch.distributed as dist
            allv = [None] * Engine.world_size()
            dist.all_gather_object(allv, outs)
            outs = [o for part in allv for o in part]
        return outs

    def predict_class(self, data, batch_size: int = -1, gather: bool = False):
        outs = self.predict(data, batch_size, gather=gather)
        return np.array([int(torch.argmax(o.reshape(-1)).item()) + 1 for o in outs], dtype=np.int64)

    predictClass = predict_class


# ------------------------------------------------------------------------------------------------- serving
def _error_activity(stage: str, e: BaseException):
    return f"ERROR during {stage}: {type(e).__name__}: {e}"


def _tensor_pb(t):
    from ..serialization import bigdl_pb as pb
    tp = pb.BigDLTensor()
    DT = pb.DataType
    if isinstance(t, str):
        tp.datatype = DT["STRING"]
        tp.isScalar = True
        tp.storage.datatype = DT["STRING"]
        tp.storage.string_data.append(t)
        tp.nElements = 1
        tp.offset = 1
        return tp
    if isinstance(t, (bool, int, float)):
        t = torch.tensor(t)
    t = t.detach().cpu().contiguous()
    if t.dtype in (torch.bfloat16, torch.float16):
        t = t.float()
    dmap = {torch.float32: ("FLOAT", "float_data"), torch.float64: ("DOUBLE", "double_data"),
            torch.int64: ("INT64", "long_data"), torch.int32: ("INT32", "int_data"), torch.bool: ("BOOL", "bool_data")}
    name, field = dmap.get(t.dtype, ("FLOAT", "float_data"))
    if t.dtype not in dmap:
        t = t.float()
    tp.datatype = DT[name]
    tp.size.extend(list(t.shape))
    tp.stride.extend(list(t.stride()))
    tp.dimension = t.dim()
    tp.nElements = t.numel()
    tp.isScalar = t.dim() == 0
    tp.offset = 1
    tp.storage.datatype = DT[name]
    getattr(tp.storage, field).extend(t.reshape(-1).numpy().tolist())
    return tp


def _tensor_from(tp):
    from ..serialization import bigdl_pb as pb
    DT = pb.DataType
    sp = tp.storage
    if tp.datatype == DT["STRING"]:
        return sp.string_data[0] if len(sp.string_data) == 1 else list(sp.string_data)
    for field, dt in (("float_data", torch.float32), ("double_data", torch.float64), ("long_data", torch.int64),
                      ("int_data", torch.int32), ("bool_data", torch.bool)):
        vals = getattr(sp, field)
        if len(vals):
            flat = torch.tensor(list(vals), dtype=dt)
            break
    else:
        flat = torch.empty(0)
    if tp.isScalar:
        return flat.reshape(())
    return flat[tp.offset - 1:tp.offset - 1 + tp.nElements].reshape(list(tp.size))


def serialize_activity(activity) -> bytes:
    """``PredictionService.serializeActivity``: a Tensor → ``AttrValue{tensorValue}``; a Table →
    ``AttrValue{arrayValue = [isKeyPrimitive, keys…, values…]}``."""
    from ..serialization import bigdl_pb as pb
    av = pb.AttrValue()
    if isinstance(activity, Table):
        keys = list(activity.keys())
        prim = not isinstance(keys[0], torch.Tensor)
        ts = [torch.tensor(prim)] + [torch.tensor(k) if prim and not isinstance(k, str) else k for k in keys] + \
             [activity[k] for k in keys]
        av.dataType = pb.DataType["ARRAY_VALUE"]
        av.arrayValue.datatype = pb.DataType["TENSOR"]
        av.arrayValue.size = len(ts)
        for t in ts:
            av.arrayValue.tensor.add().CopyFrom(_tensor_pb(t))
    else:
        av.dataType = pb.DataType["TENSOR"]
        av.tensorValue.CopyFrom(_tensor_pb(activity))
    return av.SerializeToString()


def deserialize_activity(data: bytes):
    from ..serialization import bigdl_pb as pb
    av = pb.AttrValue()
    av.ParseFromString(data)
    if av.dataType == pb.DataType["ARRAY_VALUE"]:
        ts = [_tensor_from(t) for t in av.arrayValue.tensor]
        n = (len(ts) - 1) // 2
        prim = bool(ts[0])
        keys = ts[1:n + 1]
        if prim:
            keys = [k if isinstance(k, str) else k.item() for k in keys]
        t = Table()
        for k, v in zip(keys, ts[n + 1:]):
            t[k] = v
        return t
    if av.dataType == pb.DataType["TENSOR"]:
        return _tensor_from(av.tensorValue)
    raise ValueError(f"Unsupported DataType({av.dataType})")


class PredictionService:
    """Thread-safe prediction with a pool of ``num_threads`` weight-sharing instances.

    Each instance is a shallow clone (parameters shared, activations private) in eval mode and —
    on a GPU — owns a dedicated HIP stream, so concurrent requests overlap on the device."""

    def __init__(self, model, num_threads: int = 4, compiled: Optional[bool] = None):
        from ..utils import config
        self.model = model.evaluate() if hasattr(model, "evaluate") else model
        self.num_threads = num_threads
        self._dev = _model_device(model)
        self._q: "queue.Queue" = queue.Queue()
        use = compiled if compiled is not None else bool(config.get_property("bigdl.predict.compiled"))
        self._compiled = use and self._dev.type == "cuda"
        for _ in range(num_threads):
            inst = _shallow_clone(model)
            if self._compiled:
                # each replica is IR-lowered (BN folded, fused epilogues) and captures its own HIP
                # graph per request shape, replayed on its own stream
                from ..nn.compiled import _lower
                inst = _lower(inst, None)
            stream = torch.cuda.Stream(device=self._dev) if self._dev.type == "cuda" else None
            self._q.put((_ServeInstance(inst, self._compiled), stream))

    @staticmethod
    def create(model, num_threads: int = 4):
        return PredictionService(model, num_threads)

    def predict(self, request):
        if isinstance(request, (bytes, bytearray)):
            try:
                act = deserialize_activity(bytes(request))
            except Exception as e:  # noqa: BLE001 - reference returns the error as a tensor
                out = _error_activity("DeSerialize Input", e)
            else:
                out = self._predict_activity(act)
            try:
                return serialize_activity(out)
            except Exception as e:  # noqa: BLE001
                return serialize_activity(_error_activity("Serialize Output", e))
        return self._predict_activity(request)

    def _predict_activity(self, request):
        inst, stream = self._q.get()
        try:
            try:
                with torch.no_grad():
                    if stream is not None:
                        with torch.cuda.stream(stream):
                            x = _move(request, self._dev)
                            out = inst.forward(x)
                            out = _to_host(out)
                    else:
                        out = _to_host(inst.forward(request))
            except Exception as e:  # noqa: BLE001
                return _error_activity("running forward", e)
            try:
                return _clone(out)
            except Exception as e:  # noqa: BLE001
                return _error_activity("Clone Result", e)
        finally:
            self._q.put((inst, stream))


class _ServeInstance:
    """One serving replica: its module plus, when compiled, a HIP graph per request shape."""

    def __init__(self, module, compiled: bool):
        self.module, self.compiled, self.graphs = module, compiled, {}

    def forward(self, x):
        if not (self.compiled and isinstance(x, torch.Tensor) and x.is_cuda):
            return self.module.forward(x)
        key = (tuple(x.shape), x.dtype)
        c = self.graphs.get(key)
        if c is None:
            from ..nn.compiled import compile as compile_module
            c = self.graphs[key] = compile_module(self.module, x, lower=False)
        return c(x)


def _move(a, dev):
    if isinstance(a, torch.Tensor):
        a = a.to(dev, non_blocking=True)
        if dev.type == "cuda" and a.is_floating_point():
            a = a.to(Engine.compute_dtype())
        return a
    if isinstance(a, np.ndarray):
        return _move(torch.from_numpy(a), dev)
    if isinstance(a, Table):
        t = Table()
        for k, v in a.items():
            t[k] = _move(v, dev)
        return t
    return a


def _clone(a):
    if isinstance(a, torch.Tensor):
        return a.clone()
    if isinstance(a, Table):
        t = Table()
        for k, v in a.items():
            t[_clone(k) if isinstance(k, torch.Tensor) else k] = _clone(v)
        return t
    return a


def _shallow_clone(model):
    """Clone module structure, sharing parameter/buffer storage (``model.clone(false)``)."""
    import copy
    memo = {}
    for m in model.flattened_modules():
        for n in m._tensors_attrs():
            t = getattr(m, n, None)
            if isinstance(t, torch.Tensor):
                memo[id(t)] = t
        if m._arena is not None:
            memo[id(m._arena)] = m._arena
    c = copy.deepcopy(model, memo)
    c.evaluate()
    return c
