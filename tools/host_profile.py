"""Host-side cost of one ResNet-50 training step: cProfile over N steps at a small batch (the GPU
finishes first, so the step time is the host's), plus the host enqueue time per step at the bench
batch (time for train_step() to return, GPU running behind).

    python tools/host_profile.py [--batch 16] [--steps 10] [--big 256] [--top 40]"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bigdl-1_amd"))
import torch  # noqa: E402


def build(B):
    from bigdl.dataset import MiniBatch
    from bigdl.models.resnet import DatasetType, ResNet, model_init
    from bigdl.nn import CrossEntropyCriterion
    from bigdl.optim import SGD
    from bigdl.optim.optimizer import LocalOptimizer
    model = model_init(ResNet(1000, depth=50, dataset=DatasetType.ImageNet))
    x = torch.randn(B, 3, 224, 224, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = (torch.randint(0, 1000, (B,), device="cuda") + 1).float()
    opt = LocalOptimizer(model, [MiniBatch(x, y)], CrossEntropyCriterion(),
                         SGD(learningrate=0.1, momentum=0.9, dampening=0.0, nesterov=True, weightdecay=1e-4),
                         batch_size=B)
    opt.prepare()
    return opt, MiniBatch(x, y)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--big", type=int, default=256)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    from bigdl.utils import config
    config.set_property("bigdl.compute.dtype", "bf16")
    from bigdl.utils.engine import Engine
    Engine.init()
    opt, mb = build(a.batch)
    for _ in range(5):
        opt.train_step(mb)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        opt.train_step(mb)
    torch.cuda.synchronize()
    print(f"batch {a.batch}: {(time.perf_counter() - t0) / a.steps * 1e3:.2f} ms/step (host-bound)", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.steps):
        opt.train_step(mb)
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(a.top)
    print(s.getvalue()[:12000], flush=True)
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(a.top)
    print(s.getvalue()[:12000], flush=True)
    del opt, mb
    torch.cuda.empty_cache()
    if a.big:
        opt, mb = build(a.big)
        for _ in range(5):
            opt.train_step(mb)
        torch.cuda.synchronize()
        enq = []
        t0 = time.perf_counter()
        for _ in range(a.steps):
            t1 = time.perf_counter()
            opt.train_step(mb)
            enq.append(time.perf_counter() - t1)
        torch.cuda.synchronize()
        tot = (time.perf_counter() - t0) / a.steps
        print(f"batch {a.big}: {tot * 1e3:.2f} ms/step; train_step() returns after "
              f"{sum(enq) / len(enq) * 1e3:.2f} ms (min {min(enq) * 1e3:.2f}, max {max(enq) * 1e3:.2f})", flush=True)


if __name__ == "__main__":
    main()
