#!/usr/bin/env python
"""Compiled ResNet-50 inference at one batch size, ITERS timed calls (a rocprofv3 target: the last
ITERS × ms window of the trace is the steady state).  Prints {"batch", "ms"}."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bigdl-1_amd"))


def main():
    import torch
    from bigdl.utils.engine import Engine
    from bigdl.models.resnet import ResNet, DatasetType
    from bigdl.nn.compiled import compile as compile_module
    Engine.init(device="cuda:0")
    bs = int(os.environ.get("BS", "256"))
    it = int(os.environ.get("ITERS", "20"))
    m = ResNet(1000, depth=50, dataset=DatasetType.ImageNet).to(device="cuda")
    m.evaluate()
    x = torch.randn(bs, 3, 224, 224, device="cuda")
    c = compile_module(m, x)
    for _ in range(5):
        c(x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(it):
        c(x)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / it * 1e3
    print(json.dumps({"batch": bs, "ms": round(ms, 3), "captured": c.captured, "lowered": c.lowered}), flush=True)


if __name__ == "__main__":
    main()
