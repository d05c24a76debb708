"""int8 accuracy on a TRAINED network (no pretrained weights exist here, so the network is trained
first): ResNet-50 learns the synthetic 224² task of tools/convergence.py (bf16 native, N steps), then
is calibrated (calcScales on held-in images, the bigdl.int8.calibration rule) and quantised
(static int8 chains through residual blocks, int8 FC head), and top-1 accuracy of the float (fp32)
and int8 models is measured on held-out images — the reference's int8 claim is a top-1 change on
trained ImageNet models (docs/docs/whitepaper.md: −0.04 % on VGG16).

    python tools/int8_trained.py --steps 1500 --classes 1000 --noise 3
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bigdl-1_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=1500)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--classes", type=int, default=1000)
    ap.add_argument("--noise", type=float, default=3.0)
    ap.add_argument("--calib", type=int, default=2, help="calibration batches")
    ap.add_argument("--eval", type=int, default=16, help="held-out batches")
    args = ap.parse_args()
    from bigdl.utils import config
    config.set_property("bigdl.compute.dtype", "bf16")
    from bigdl.utils.engine import Engine
    Engine.init()
    from bigdl.models.resnet import ResNet, DatasetType, model_init
    from bigdl.nn import CrossEntropyCriterion
    from bigdl.optim import SGD
    from bigdl.optim.optimizer import LocalOptimizer
    from bigdl.dataset import MiniBatch
    from bigdl.utils.random import RNG
    dev = torch.device("cuda")
    RNG.setSeed(42)
    model = model_init(ResNet(args.classes, depth=50, dataset=DatasetType.ImageNet))
    g0 = torch.Generator(device="cpu").manual_seed(7)
    templates = torch.nn.functional.interpolate(torch.randn(args.classes, 3, 7, 7, generator=g0), size=(224, 224),
                                                mode="nearest").to(dev)

    def batch(step, salt=0, dt=torch.bfloat16):
        g = torch.Generator(device=dev).manual_seed(1000003 * salt + step)
        lab = torch.randint(0, args.classes, (args.batch,), generator=g, device=dev)
        x = templates[lab] + args.noise * torch.randn(args.batch, 3, 224, 224, generator=g, device=dev)
        return x.to(dt).contiguous(memory_format=torch.channels_last), lab

    sgd = SGD(learningrate=0.1, learningrate_decay=0.0, weightdecay=1e-4, momentum=0.9, dampening=0.0, nesterov=True)
    x0, l0 = batch(0)
    opt = LocalOptimizer(model, [MiniBatch(x0, (l0 + 1).float())], CrossEntropyCriterion(), sgd,
                         batch_size=args.batch)
    opt.prepare()
    for step in range(args.steps):
        sgd.learningRate = 0.1 * min(1.0, (step + 1) / 100)
        x, lab = batch(step)
        loss = opt.train_step(MiniBatch(x, (lab + 1).float()))
        if step % 250 == 0 or step == args.steps - 1:
            print(json.dumps({"step": step, "loss": round(float(loss), 4)}), flush=True)
    torch.cuda.synchronize()

    def accuracy(m, dt):
        m.evaluate()
        correct, logits = 0, []
        with torch.no_grad():
            for i in range(args.eval):
                x, lab = batch(i, salt=2, dt=dt)
                out = m.forward(x).float()
                logits.append(out.cpu())
                correct += int((out.argmax(1) == lab).sum())
        return correct / (args.eval * args.batch), torch.cat(logits)

    # float reference in fp32 compute (a clone: the trained weights, fp32 kernels)
    config.set_property("bigdl.compute.dtype", "fp32")
    Engine.init()
    fm = model.cloneModule().to(dev)
    acc_f, lf = accuracy(fm, torch.float32)
    # calibration + quantisation (as tools/bench_configs.py --config int8)
    config.set_property("bigdl.compute.dtype", "bf16")
    Engine.init()
    cal = model.cloneModule().to(dev)
    cal.evaluate()
    xc = torch.cat([batch(i, salt=3)[0] for i in range(args.calib)])
    with torch.no_grad():
        cal.forward(xc)
    cal.calcScales(xc)
    q = cal.quantize().to(dev)
    acc_q, lq = accuracy(q, torch.bfloat16)
    bm = model.cloneModule().to(dev)
    acc_b, lb = accuracy(bm, torch.bfloat16)
    agree = float((lq.argmax(1) == lf.argmax(1)).float().mean())
    cf, cq = lf - lf.mean(1, keepdim=True), lq - lq.mean(1, keepdim=True)
    cos = float((cf.double().flatten() @ cq.double().flatten()) / (cf.double().norm() * cq.double().norm()))
    print(json.dumps({"final": True, "steps": args.steps, "classes": args.classes, "noise": args.noise,
                      "top1_fp32": round(acc_f, 4), "top1_bf16": round(acc_b, 4), "top1_int8": round(acc_q, 4),
                      "top1_change_int8_vs_fp32": round(acc_q - acc_f, 4), "top1_agreement": round(agree, 4),
                      "logit_cosine": round(cos, 5), "calibration": str(config.get_property("bigdl.int8.calibration")),
                      "calib_images": args.calib * args.batch, "eval_images": args.eval * args.batch}), flush=True)


if __name__ == "__main__":
    main()
