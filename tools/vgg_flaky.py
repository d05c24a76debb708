"""Repeat the VGG-CIFAR learning check (tests/test_gpu_learning.py) a few times per BN-statistics
mode and report eval accuracy and running-statistics health (NaN / non-positive variance)."""
import json
import sys
import os
import torch
_R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(_R, "tests"), os.path.join(_R, "bigdl-1_amd")]
import test_gpu_learning as T  # noqa: E402
from bigdl.utils import config  # noqa: E402

for rep in (32, 0):
    config.set_property("bigdl.bn.statReplicas", rep)
    for it in range(3):
        T._setup()
        from bigdl.models.vgg import VggForCifar10
        from bigdl.nn import ClassNLLCriterion
        from bigdl.optim import SGD
        torch.manual_seed(0)
        x, y = T._images(512)
        batches = [(x[i:i + 64], y[i:i + 64]) for i in range(0, 512, 64)]
        model = VggForCifar10(10).to(device="cuda")
        losses, mbs = T._train(model, ClassNLLCriterion(), SGD(learningrate=0.02, momentum=0.9, dampening=0.0),
                               batches, 20)
        acc = T._accuracy(model, mbs)
        bad = []

        def walk(m, path="m"):
            rv, rm = getattr(m, "runningVar", None), getattr(m, "runningMean", None)
            if isinstance(rv, torch.Tensor) and (not torch.isfinite(rv).all() or (rv <= 0).any()):
                bad.append(path + ".runningVar")
            if isinstance(rm, torch.Tensor) and not torch.isfinite(rm).all():
                bad.append(path + ".runningMean")
            for i, c in enumerate(m.children()):
                walk(c, f"{path}.{i}")
        walk(model)
        print(json.dumps({"replicas": rep, "it": it, "loss_first": sum(losses[:4]) / 4, "loss_last": sum(losses[-4:]) / 4,
                          "acc": acc, "bad_running_stats": bad[:6]}), flush=True)
