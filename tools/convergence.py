"""ResNet-50 training curves, bf16 vs fp32 compute, on a learnable synthetic 224² task: every class
is a random 7×7×3 pattern upsampled to 224² (a spatial template, not a flat colour), each image its
class template plus Gaussian noise drawn on the GPU from a per-step seed — the same stream of
batches for both dtypes.  Same init (RNG seed), same SGD as bench.py (lr 0.1 with a linear warm-up,
momentum 0.9 Nesterov, weight decay 1e-4, L2 1e-4 on the classifier).  Prints one JSON line per
logged step and a final held-out accuracy (fresh noise, evaluation mode).

    python tools/convergence.py --dtype fp32 --steps 600 --batch 128
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bigdl-1_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--steps", type=int, default=600)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--classes", type=int, default=100)
    ap.add_argument("--noise", type=float, default=1.0)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--log-every", type=int, default=20)
    ap.add_argument("--model", default="resnet50", help="resnet50 (224²) | vgg_cifar (VggForCifar10, 32²)")
    ap.add_argument("--check-bn", type=int, default=0,
                    help="after every step compare each BN's saved batch statistics with fp64 statistics of its input")
    args = ap.parse_args()
    from bigdl.utils import config
    config.set_property("bigdl.compute.dtype", args.dtype)
    from bigdl.utils.engine import Engine
    Engine.init()
    from bigdl.models.resnet import ResNet, DatasetType, model_init
    from bigdl.nn import CrossEntropyCriterion
    from bigdl.optim import SGD
    from bigdl.optim.optimizer import LocalOptimizer
    from bigdl.dataset import MiniBatch
    from bigdl.utils.random import RNG
    dev = torch.device("cuda")
    dt = Engine.compute_dtype()
    RNG.setSeed(42)
    S = 224
    if args.model == "vgg_cifar":
        from bigdl.models.vgg import VggForCifar10
        model = VggForCifar10(args.classes)
        S = 32
    else:
        model = model_init(ResNet(args.classes, depth=50, dataset=DatasetType.ImageNet))
    crit = CrossEntropyCriterion()
    sgd = SGD(learningrate=args.lr, learningrate_decay=0.0, weightdecay=1e-4, momentum=0.9, dampening=0.0,
              nesterov=True)
    g0 = torch.Generator(device="cpu").manual_seed(7)
    templates = torch.nn.functional.interpolate(torch.randn(args.classes, 3, 7, 7, generator=g0), size=(S, S),
                                                mode="nearest").to(dev)

    def batch(step, salt=0):
        g = torch.Generator(device=dev).manual_seed(1000003 * salt + step)
        lab = torch.randint(0, args.classes, (args.batch,), generator=g, device=dev)
        x = templates[lab] + args.noise * torch.randn(args.batch, 3, S, S, generator=g, device=dev)
        return MiniBatch(x.to(dt).contiguous(memory_format=torch.channels_last), (lab + 1).float())

    first = batch(0)
    opt = LocalOptimizer(model, [first], crit, sgd, batch_size=args.batch)
    opt.prepare()
    t0 = time.perf_counter()
    for step in range(args.steps):
        sgd.learningRate = args.lr * min(1.0, (step + 1) / max(args.warmup, 1))
        loss = opt.train_step(batch(step))
        if args.check_bn:
            from bigdl.nn import SpatialBatchNormalization
            worst = (0.0, 0.0, "")
            for i, bn in enumerate(m for m in model.flattened_modules() if isinstance(m, SpatialBatchNormalization)):
                x = bn.__dict__.get("_last_input")
                if x is None or bn.saveStd is None:
                    continue
                xd = x.double().permute(0, 2, 3, 1).reshape(-1, x.shape[1])
                mu, var = xd.mean(0), xd.var(0, unbiased=False)
                inv = torch.rsqrt(var + bn.eps)
                e_inv = float(((bn.saveStd.double() - inv).abs() / inv).max())
                e_mu = float(((bn.saveMean.double() - mu).abs() / var.sqrt().clamp_min(1e-12)).max())
                if e_inv > worst[0]:
                    worst = (e_inv, e_mu, f"bn{i} C{x.shape[1]} |mu|/sd {float((mu.abs() / var.sqrt().clamp_min(1e-12)).max()):.1f}")
            if worst[0] > 1e-3 or step % args.log_every == 0:
                print(json.dumps({"step": step, "bn_worst_rel_invstd_err": worst[0], "mean_err_sd": worst[1],
                                  "where": worst[2]}), flush=True)
        if step % args.log_every == 0 or step == args.steps - 1:
            print(json.dumps({"dtype": args.dtype, "step": step, "loss": round(float(loss), 5),
                              "lr": round(sgd.learningRate, 5), "t": round(time.perf_counter() - t0, 2)}),
                  flush=True)
    model.evaluate()
    correct = total = 0
    with torch.no_grad():
        for i in range(8):
            b = batch(i, salt=1)
            out = model.forward(b.getInput()).float()
            correct += int((out.argmax(1) + 1 == b.getTarget().to(out.device)).sum())
            total += b.size()
    print(json.dumps({"dtype": args.dtype, "final": True, "steps": args.steps, "heldout_acc": correct / total,
                      "train_s": round(time.perf_counter() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
