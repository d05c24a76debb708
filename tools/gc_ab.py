"""A/B of Python garbage-collector settings on the ResNet-50 bs-256 step: default, gc.freeze()
after warm-up, gc disabled in the timed loop.  Host stalls (a gen-2 collection walks every live
object) show up as idle gaps on the GPU when the host is less than a stall ahead of it."""
import gc
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402
from host_profile import build  # noqa: E402


def run(opt, mb, steps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        opt.train_step(mb)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    from bigdl.utils import config
    config.set_property("bigdl.compute.dtype", "bf16")
    from bigdl.utils.engine import Engine
    Engine.init()
    opt, mb = build(int(os.environ.get("B", "256")))
    for _ in range(5):
        opt.train_step(mb)
    steps = int(os.environ.get("STEPS", "20"))
    print("gc counts", gc.get_count(), "thresholds", gc.get_threshold(), "objects", len(gc.get_objects()), flush=True)
    for rep in range(2):
        print(f"default      {run(opt, mb, steps):.3f} ms/step", flush=True)
        gc.freeze()
        print(f"freeze       {run(opt, mb, steps):.3f} ms/step", flush=True)
        gc.unfreeze()
        gc.disable()
        print(f"disabled     {run(opt, mb, steps):.3f} ms/step", flush=True)
        gc.enable()
        t0 = time.perf_counter()
        n = gc.collect()
        print(f"full collect {1e3 * (time.perf_counter() - t0):.2f} ms ({n} freed)", flush=True)


if __name__ == "__main__":
    main()
