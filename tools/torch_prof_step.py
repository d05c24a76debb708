"""Attribute the non-HIP-kernel work of one ResNet-50 training step (copies, fills, torch
elementwise) to its Python call sites with torch.profiler (CPU-side op stacks)."""
import os
import sys
import collections

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bigdl-1_amd"))
import torch
from bigdl.utils import config
DT = os.environ.get("DTYPE", "bf16")
config.set_property("bigdl.compute.dtype", DT)
from bigdl.utils.engine import Engine
Engine.init()
from bigdl.models.resnet import ResNet, DatasetType, model_init
from bigdl.nn import CrossEntropyCriterion
from bigdl.optim import SGD
from bigdl.optim.optimizer import LocalOptimizer
from bigdl.dataset import MiniBatch

B = int(os.environ.get("B", "64"))
model = model_init(ResNet(1000, depth=50, dataset=DatasetType.ImageNet))
x = torch.randn(B, 3, 224, 224, device="cuda").to(torch.bfloat16 if DT == "bf16" else torch.float32).contiguous(memory_format=torch.channels_last)
y = (torch.randint(0, 1000, (B,), device="cuda") + 1).float()
opt = LocalOptimizer(model, [MiniBatch(x, y)], CrossEntropyCriterion(),
                     SGD(learningrate=0.1, momentum=0.9, dampening=0.0, nesterov=True, weightdecay=1e-4), batch_size=B)
opt.prepare()
for _ in range(3):
    opt.train_step(MiniBatch(x, y))
torch.cuda.synchronize()
from torch.profiler import profile, ProfilerActivity
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    opt.train_step(MiniBatch(x, y))
    torch.cuda.synchronize()
cnt = collections.Counter()
for ev in prof.events():
    if ev.name in ("aten::copy_", "aten::fill_", "aten::zero_", "aten::flip", "aten::index", "aten::clone",
                   "aten::contiguous", "aten::cat", "aten::mul", "aten::add", "aten::sum", "aten::to", "aten::_to_copy",
                   "aten::zeros", "aten::empty_strided", "aten::index_select", "aten::gather"):
        if os.environ.get("DEVICE_ONLY") and getattr(ev, "device_time_total", 0) <= 0:
            continue
        frames = [f for f in (ev.stack or []) if "bigdl" in f][:3]
        cnt[(ev.name, " <- ".join(frames))] += 1
for (name, st), c in cnt.most_common(40):
    print(f"{c:5d} {name:22s} {st}")


if os.environ.get("DISPATCH"):
    # the Python call sites of the aten ops that launch torch kernels on the device
    import traceback
    from torch.utils._python_dispatch import TorchDispatchMode
    WATCH = ("zero_", "fill_", "copy_", "_to_copy", "zeros", "flip", "index", "add", "sum", "mul", "clone", "cat")

    class Watch(TorchDispatchMode):
        def __init__(self):
            super().__init__()
            self.sites = collections.Counter()

        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            out = func(*args, **(kwargs or {}))
            name = func.__name__.split(".")[0].rstrip("_")
            if name in WATCH:
                dev = [a.device.type for a in list(args) + list((kwargs or {}).values()) if isinstance(a, torch.Tensor)]
                if isinstance(out, torch.Tensor):
                    dev.append(out.device.type)
                if "cuda" in dev:
                    fr = [f"{os.path.basename(f.filename)}:{f.lineno}" for f in traceback.extract_stack()[:-1]
                          if "bigdl" in f.filename][-3:]
                    self.sites[(func.__name__, " <- ".join(reversed(fr)))] += 1
            return out
    w = Watch()
    with w:
        opt.train_step(MiniBatch(x, y))
    torch.cuda.synchronize()
    print("dispatch sites (one step):")
    for (name, st), c in w.sites.most_common(40):
        print(f"{c:5d} {name:28s} {st}")
