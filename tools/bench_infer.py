#!/usr/bin/env python
"""Inference latency: eager forward vs the compiled (planned + HIP-graph) forward of ResNet-50
at serving batch sizes (bf16, 224², random init)."""
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
    from bigdl.nn.fusion import fuse
    Engine.init(device="cuda:0")
    m = ResNet(1000, depth=50, dataset=DatasetType.ImageNet).to(device="cuda")
    m.evaluate()
    fuse(m)
    for bs in [int(v) for v in os.environ.get("BATCHES", "1,8,32,256").split(",")]:
        x = torch.randn(bs, 3, 224, 224, device="cuda")

        def eager():
            with torch.no_grad():
                return m.forward(x)
        for _ in range(3):
            eager()
        torch.cuda.synchronize()
        it = 20
        t0 = time.perf_counter()
        for _ in range(it):
            eager()
        torch.cuda.synchronize()
        te = (time.perf_counter() - t0) / it * 1e3
        c = compile_module(m, x)
        for _ in range(3):
            c(x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(it):
            c(x)
        torch.cuda.synchronize()
        tc = (time.perf_counter() - t0) / it * 1e3
        for _ in range(3):
            eager()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(it):
            eager()  # the same eager forward, now with the compile phase's pinned conv tiles
        torch.cuda.synchronize()
        tt = (time.perf_counter() - t0) / it * 1e3
        ref = eager().float()
        err = float((c(x).float() - ref).abs().max())
        print(json.dumps({"batch": bs, "eager_ms": round(te, 3), "compiled_ms": round(tc, 3), "captured": c.captured,
                          "speedup": round(te / tc, 2),
                          "eager_tuned_ms": round(tt, 3), "tiles_pinned": len(c.tiles), "img_per_s_compiled": round(bs / tc * 1e3, 1),
                          "lowered": c.lowered, "max_abs_diff": err, "arena_MiB": round(c.plan.arena_bytes / 2 ** 20, 1),
                          "total_MiB": round(c.plan.total_bytes / 2 ** 20, 1)}), flush=True)


if __name__ == "__main__":
    main()
