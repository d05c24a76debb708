"""Kernel sequence of one fp32 ResNet-50 forward / backward with and without bigdl.fp32.bnPrologue."""
import sys
sys.path.insert(0, "tests")
sys.path.insert(0, "bigdl-1_amd")
import torch
import test_fp32_bn_prologue as T

for pro in (True, False):
    l, g, names = T._resnet_grads(pro)
    short = [n.split("(")[0].replace("void ", "")[:60] for n in names]
    print("=== prologue", pro, "loss", l, "kernels", len(short))
    for i, n in enumerate(short[:140]):
        print(i, n)
