#!/usr/bin/env python
"""A/B the training trajectory of the native-kernel path against the torch reference path.

Builds the same seeded ResNet (default ResNet-50, batch 32) twice on cuda:0 — once with the HIP
kernels (``bigdl.native.enable=1``) and once routed to ``bigdl/ops/reference.py`` — trains K steps
on one fixed synthetic batch and prints both loss curves.  bf16 compute makes the curves drift
apart slowly; a kernel race or wrong gradient shows as an early, large divergence.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(_HERE, "..", "bigdl-1_amd"))


def run(native: bool, args):
    import torch
    from bigdl.utils import config
    config.set_property("bigdl.compute.dtype", args.dtype)
    config.set_property("bigdl.native.enable", native)
    from bigdl.utils.engine import Engine
    Engine.init(device="cuda:0")
    from bigdl.models.resnet import ResNet, DatasetType, model_init
    from bigdl.nn import CrossEntropyCriterion
    from bigdl.optim import SGD
    from bigdl.optim.optimizer import LocalOptimizer
    from bigdl.dataset import MiniBatch
    from bigdl.utils.random import RNG
    RNG.setSeed(7)
    torch.manual_seed(7)
    model = model_init(ResNet(1000, depth=args.depth, dataset=DatasetType.ImageNet))
    g = torch.Generator().manual_seed(11)
    x = torch.randn(args.batch, 3, 224, 224, generator=g).cuda().to(Engine.compute_dtype()).contiguous(
        memory_format=torch.channels_last)
    y = (torch.randint(0, 1000, (args.batch,), generator=g) + 1).float().cuda()
    opt = LocalOptimizer(model, [MiniBatch(x, y)], CrossEntropyCriterion(),
                         SGD(learningrate=args.lr, momentum=0.9, dampening=0.0, nesterov=True, weightdecay=1e-4),
                         batch_size=args.batch)
    opt.prepare()
    losses = []
    for _ in range(args.steps):
        losses.append(float(opt.train_step(MiniBatch(x, y))))
    torch.cuda.synchronize()
    return losses


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--dtype", default="bf16")
    args = ap.parse_args()
    a = run(True, args)
    b = run(False, args)
    print(json.dumps({"native": [round(v, 4) for v in a], "reference": [round(v, 4) for v in b]}))
    for i, (u, v) in enumerate(zip(a, b)):
        print(f"step {i:3d} native {u:9.4f} reference {v:9.4f} diff {u - v:+.4f}")


if __name__ == "__main__":
    main()
