"""Does a training run on the fused native bf16 path learn like the fp32 reference?  ResNet-50
memorises one fixed batch (synthetic images, random labels) with SGD; prints the loss curve of the
device bf16 run and of the fp32 host run (reference ops) from the same initial weights.

    python tools/memorize_check.py [--steps 25] [--lr 0.01] [--batch 16] [--host 1]
"""
import argparse
import copy
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bigdl-1_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=25)
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--host", type=int, default=1)
    args = ap.parse_args()
    import torch
    from bigdl.utils import config
    config.set_property("bigdl.compute.dtype", "bf16")
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
    model = model_init(ResNet(10, depth=args.depth, dataset=DatasetType.ImageNet))
    host_model = copy.deepcopy(model)
    g = torch.Generator().manual_seed(11)
    x = torch.randn(args.batch, 3, 224, 224, generator=g)
    y = (torch.randint(0, 10, (args.batch,), generator=g) + 1).float()
    sgd = lambda: SGD(learningrate=args.lr, momentum=0.9, dampening=0.0)  # noqa: E731
    b = MiniBatch(x.cuda().to(torch.bfloat16).contiguous(memory_format=torch.channels_last), y.cuda())
    opt = LocalOptimizer(model, [b], CrossEntropyCriterion(), sgd(), batch_size=args.batch)
    opt.prepare()
    dev_curve = [round(float(opt.train_step(b)), 4) for _ in range(args.steps)]
    print(json.dumps({"run": "device bf16 native", "loss": dev_curve}), flush=True)
    if args.host:
        Engine.set_device("cpu")
        Engine.set_compute_dtype("fp32")
        hb = MiniBatch(x, y)
        hopt = LocalOptimizer(host_model, [hb], CrossEntropyCriterion(), sgd(), batch_size=args.batch)
        hopt.device = torch.device("cpu")
        hopt.compute_dtype = torch.float32
        hopt.prepare()
        host_curve = [round(float(hopt.train_step(hb)), 4) for _ in range(args.steps)]
        print(json.dumps({"run": "host fp32 reference", "loss": host_curve}), flush=True)


if __name__ == "__main__":
    main()
