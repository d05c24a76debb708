"""Optimizer perf harnesses (``DL/models/utils/{Local,Distri}OptimizerPerf.scala``): time a model's
training iterations on synthetic data.

    python -m bigdl.models.utils.perf --model resnet50 --batch 256 --iteration 20 [--graph]
    python -m bigdl.launch --nproc 8 -m bigdl.models.utils.perf --model inception_v1 ...

Models: lenet5, vgg16 (CIFAR), resnet50, inception_v1, inception_v2, alexnet-free (the reference's
list minus AlexNet, which has no builder in the reference's model zoo either).  Prints the
reference's per-iteration log line and a final throughput line.
"""
from __future__ import annotations

import argparse
import os
import sys
import time


def build(name: str):
    from .. import lenet, vgg, resnet, inception
    if name == "lenet5":
        return lenet.LeNet5(10), (1, 28, 28), 10
    if name == "vgg16":
        return vgg.VggForCifar10(10), (3, 32, 32), 10
    if name == "resnet50":
        m = resnet.model_init(resnet.ResNet(1000, depth=50, dataset=resnet.DatasetType.ImageNet))
        return m, (3, 224, 224), 1000
    if name == "inception_v1":
        return inception.Inception_v1_NoAuxClassifier(1000), (3, 224, 224), 1000
    if name == "inception_v2":
        return inception.Inception_v2_NoAuxClassifier(1000), (3, 224, 224), 1000
    raise ValueError(f"unknown model {name}")


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="perf")
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", "-b", type=int, default=128)
    ap.add_argument("--iteration", "-i", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--graph", action="store_true")
    a = ap.parse_args(argv)
    import torch
    from ...utils import config
    config.set_property("bigdl.compute.dtype", a.dtype)
    from ...utils.engine import Engine
    world = int(os.environ.get("WORLD_SIZE", "1"))
    Engine.init(dist=world > 1)
    dev = Engine.device()
    from ...nn import ClassNLLCriterion, CrossEntropyCriterion
    from ...optim import SGD
    from ...optim.optimizer import LocalOptimizer
    from ...dataset import MiniBatch
    model, shape, classes = build(a.model)
    dt = Engine.compute_dtype() if dev.type == "cuda" else torch.float32
    x = torch.randn(a.batch, *shape).to(dev).to(dt)
    if x.dim() == 4 and dev.type == "cuda":
        x = x.contiguous(memory_format=torch.channels_last)
    y = (torch.randint(0, classes, (a.batch,)) + 1).float().to(dev)
    crit = ClassNLLCriterion() if a.model in ("lenet5", "vgg16") else CrossEntropyCriterion()
    b = MiniBatch(x, y)
    if world > 1:
        from ...parallel import DistriOptimizer
        opt = DistriOptimizer(model, [b], crit, SGD(learningrate=0.01), batch_size=a.batch)
    else:
        opt = LocalOptimizer(model, [b], crit, SGD(learningrate=0.01), batch_size=a.batch)
    opt.prepare()
    step = opt.train_step
    if a.graph and world == 1 and dev.type == "cuda":
        from ...optim.graph_step import graphed_train_step
        step = lambda bb: graphed_train_step(opt, bb)  # noqa: E731
    for _ in range(a.warmup):
        step(b)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    total = 0.0
    for i in range(a.iteration):
        t0 = time.perf_counter()
        loss = step(b)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        dt_s = time.perf_counter() - t0
        total += dt_s
        if Engine.rank() == 0:
            print(f"[Iteration {i + 1}] Trained {a.batch * world} records in {dt_s:.4f} seconds. "
                  f"Throughput is {a.batch * world / dt_s:.1f} records/second. Loss is {float(loss):.4f}.")
    if Engine.rank() == 0:
        print(f"{a.model}: average throughput {a.batch * world * a.iteration / total:.1f} records/second")
    Engine.shutdown()
    return 0


LocalOptimizerPerf = DistriOptimizerPerf = main

if __name__ == "__main__":
    sys.exit(main())
