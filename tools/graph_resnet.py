#!/usr/bin/env python
"""ResNet-50 training step: eager vs the whole step captured into one HIP graph (A/B)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bigdl-1_amd"))


def main():
    import torch
    from bigdl.utils import config
    config.set_property("bigdl.compute.dtype", "bf16")
    from bigdl.utils.engine import Engine
    Engine.init()
    from bigdl.models.resnet import ResNet, DatasetType, model_init
    from bigdl.nn import CrossEntropyCriterion
    from bigdl.optim import SGD
    from bigdl.optim.optimizer import LocalOptimizer
    from bigdl.dataset import MiniBatch
    dev = Engine.device()
    model = ResNet(1000, depth=50, dataset=DatasetType.ImageNet)
    model_init(model)
    sgd = SGD(learningrate=0.1, weightdecay=1e-4, momentum=0.9, dampening=0.0, nesterov=True)
    g = torch.Generator().manual_seed(0)
    bs = []
    for _ in range(2):
        x = torch.randn(256, 3, 224, 224, generator=g).to(dev).bfloat16().contiguous(memory_format=torch.channels_last)
        y = (torch.randint(0, 1000, (256,), generator=g) + 1).float().to(dev)
        bs.append(MiniBatch(x, y))
    opt = LocalOptimizer(model, [bs[0]], CrossEntropyCriterion(), sgd, batch_size=256)
    opt.prepare()
    mode = os.environ.get("MODE", "graph")
    if mode == "graph":
        config.set_property("bigdl.graph.capture", True)
    step = opt._step
    for i in range(5):
        step(bs[i % 2])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 30
    for i in range(n):
        loss = step(bs[i % 2])
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / n * 1e3
    print(json.dumps({"mode": mode, "ms_per_step": round(ms, 3), "captured": getattr(opt, "_graphed", None) is not None,
                      "loss": float(loss)}))


if __name__ == "__main__":
    main()
