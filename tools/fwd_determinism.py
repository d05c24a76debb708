import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bigdl-1_amd"))
import torch
from bigdl.models.resnet import ResNet, DatasetType, model_init
from bigdl.nn.fusion import fuse
from bigdl.utils import config
from bigdl.utils.engine import Engine
from bigdl.utils.random import RNG
"""Training-mode forward determinism of the fused ResNet-50 (same input, repeated forwards); argv:
key=value config overrides (e.g. bigdl.bn.shiftedStats=false)."""
config.set_property("bigdl.compute.dtype", "bf16")
for kv in sys.argv[1:]:
    k, v = kv.split("=", 1)
    config.set_property(k, v.lower() in ("1", "true", "yes") if v.lower() in ("1", "0", "true", "false", "yes", "no") else v)
Engine.init(device="cuda:0")
RNG.setSeed(5)
m = model_init(ResNet(10, depth=50, dataset=DatasetType.ImageNet, image_size=64))
m.cuda(); m.training(); fuse(m); m.getParameters(); m.flat_parameters().enable_shadow(torch.bfloat16)
g = torch.Generator().manual_seed(0)
x = torch.randn(8, 3, 64, 64, generator=g).cuda().bfloat16().contiguous(memory_format=torch.channels_last)
ys = [m.forward(x).float().cpu() for _ in range(3)]
print("fwd-fwd diffs", [(ys[i+1]-ys[i]).abs().max().item() for i in range(2)])
gy = torch.randn(ys[0].shape, generator=g).cuda().bfloat16()
m.backward(x, gy); y4 = m.forward(x).float().cpu()
print("after bwd", (y4-ys[2]).abs().max().item())
m.evaluate(); e1 = m.forward(x).float().cpu(); e2 = m.forward(x).float().cpu(); print("eval diff", (e1-e2).abs().max().item())

# first layer whose training-mode output differs between two forwards, and its BN statistics
m.training()
mods = [mm for mm in m.flattened_modules() if isinstance(getattr(mm, "output", None), torch.Tensor)
        and not getattr(mm, "modules", None)]
m.forward(x)
outs = [mm.output.float().clone() for mm in mods]
rms = [getattr(mm, "runningMean", None) for mm in mods]
rms = [r.clone() if isinstance(r, torch.Tensor) else None for r in rms]
m.forward(x)
for i, mm in enumerate(mods):
    d = (mm.output.float() - outs[i]).abs().max().item()
    if d > 0:
        print("first differing:", i, type(mm).__name__, "maxdiff", d, "out absmax", outs[i].abs().max().item())
        if hasattr(mm, "saveMean"):
            xin = mods[i - 1].output.float() if i > 0 else None
            print("  saveMean[:4]", mm.saveMean[:4].tolist(), "saveStd[:4]", mm.saveStd[:4].tolist())
            if xin is not None and xin.dim() == 4:
                mu = xin.mean((0, 2, 3)); sd = xin.var((0, 2, 3), unbiased=False)
                print("  input mean[:4]", mu[:4].tolist(), "invstd[:4]", torch.rsqrt(sd[:4] + 1e-5).tolist())
                print("  prev running mean[:4]", rms[i][:4].tolist() if rms[i] is not None else None)
        break
