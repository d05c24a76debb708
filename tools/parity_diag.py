"""Per-parameter gradient agreement of the fused bf16 GPU ResNet-50 step vs the fp32 host oracle
(the diagnostic behind tests/test_train_parity.py).  Prints one line per parameter:
index, owning module, shape, cosine, relative norm error.

    python tools/parity_diag.py [--fusion 0|1] [--batch 4]
"""
import argparse
import copy
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bigdl-1_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fusion", type=int, default=1)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--only-bad", type=int, default=0)
    ap.add_argument("--native", type=int, default=1)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--depth", type=int, default=50)
    args = ap.parse_args()
    import torch
    from bigdl.utils import config
    from bigdl.utils.engine import Engine
    config.set_property("bigdl.compute.dtype", args.dtype)
    config.set_property("bigdl.fusion", bool(args.fusion))
    config.set_property("bigdl.native.enable", bool(args.native))
    Engine.init(device="cuda:0")
    from bigdl.models.resnet import ResNet, DatasetType, model_init
    from bigdl.nn import CrossEntropyCriterion
    from bigdl.nn.fusion import fuse, mark_input_no_grad
    from bigdl.utils.random import RNG
    RNG.setSeed(7)
    torch.manual_seed(7)
    cpu = model_init(ResNet(100, depth=args.depth, dataset=DatasetType.ImageNet))
    gpu = copy.deepcopy(cpu)
    g = torch.Generator().manual_seed(3)
    x = torch.randn(args.batch, 3, 224, 224, generator=g)
    y = (torch.randint(0, 100, (args.batch,), generator=g) + 1).float()
    cc, cg = CrossEntropyCriterion(), CrossEntropyCriterion()
    cpu.training()
    cpu.zeroGradParameters()
    oc = cpu.forward(x)
    lc = float(cc.forward(oc, y))
    cpu.backward(x, cc.backward(oc, y))
    gpu.cuda()
    gpu.training()
    fuse(gpu)
    mark_input_no_grad(gpu)
    gpu.getParameters()
    if args.dtype == "bf16":
        gpu.flat_parameters().enable_shadow(torch.bfloat16)
    gpu.zeroGradParameters()
    xg = x.cuda().to(Engine.compute_dtype()).contiguous(memory_format=torch.channels_last)
    og = gpu.forward(xg)
    lg = float(cg.forward(og, y.cuda()))
    gpu.backward(xg, cg.backward(og, y.cuda()))
    torch.cuda.synchronize()
    print(f"loss fp32 host {lc:.5f}  {args.dtype} device {lg:.5f}  native={args.native} fusion={args.fusion}")
    owners = [f"{type(m).__name__}[{m.get_name()}].{n}" for (m, n, _g) in cpu._param_entries()]
    gc, gg = cpu.parameters()[1], gpu.parameters()[1]
    coss = []
    for i, (a, b) in enumerate(zip(gg, gc)):
        if owners[i].endswith(".bias") and "Convolution" in owners[i]:
            continue  # a conv bias feeding a BN has zero true gradient: cosine is noise
        aa, bb = a.float().cpu().double().reshape(-1), b.double().reshape(-1)
        coss.append(float((aa @ bb) / (aa.norm() * bb.norm()).clamp_min(1e-30)))
    cs = sorted(coss)
    print(f"gradient cosine: min {cs[0]:.4f}  p10 {cs[len(cs) // 10]:.4f}  median {cs[len(cs) // 2]:.4f}  "
          f"over {len(cs)} tensors")
    for i, (a, b) in enumerate(zip(gg, gc)):
        a = a.float().cpu().double().reshape(-1)
        b = b.double().reshape(-1)
        cos = float((a @ b) / (a.norm() * b.norm()).clamp_min(1e-30))
        rel = float((a - b).norm() / b.norm().clamp_min(1e-30))
        if args.only_bad and (cos > 0.99 or owners[i].endswith(".bias") and "Convolution" in owners[i]):
            continue
        own = owners[i] if i < len(owners) else "?"
        print(f"{i:4d} {own:40s} {str(tuple(gc[i].shape)):22s} cos {cos:+.4f} relerr {rel:.3e}")


if __name__ == "__main__":
    main()
