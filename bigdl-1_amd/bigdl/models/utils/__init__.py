"""Model utilities (``DL/models/utils``): ``ModelBroadcast``, the optimizer perf harnesses and the
ImageNet / COCO sequence-file generators."""
from .model_broadcast import ModelBroadcast, CachedModels  # noqa: F401
