"""SyncBN at world 1 (multi-rank kernels rehearsed) vs local BN on a fused ResNet-50 (bf16, 64² input):
loss and per-parameter gradient cosines between pairs of runs — local vs local (the atomics noise
floor), local vs SyncBN without / with the projection-shortcut deferral, SyncBN without vs with it."""
import copy
import os
import socket
import sys

import torch

sys.path.insert(0, "bigdl-1_amd")


def main():
    import torch.distributed as dist
    from bigdl.models.resnet import ResNet, DatasetType, model_init
    from bigdl.nn import CrossEntropyCriterion
    from bigdl.nn.fusion import fuse
    from bigdl.utils import config
    from bigdl.utils.engine import Engine
    from bigdl.utils.random import RNG
    config.set_property("bigdl.compute.dtype", "bf16")
    config.set_property("bigdl.bn.syncOneRankLocal", False)
    Engine.init(device="cuda:0")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(s.getsockname()[1]))
    s.close()
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    HW = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    tail_gamma = float(sys.argv[3]) if len(sys.argv) > 3 else 0.2
    RNG.setSeed(5)
    base = model_init(ResNet(10, depth=50, dataset=DatasetType.ImageNet, image_size=HW))
    with torch.no_grad():
        for mod in base.flattened_modules():
            if type(mod).__name__ == "SpatialBatchNormalization" and float(mod.weight.abs().max()) == 0.0:
                mod.weight.fill_(tail_gamma)
    g = torch.Generator().manual_seed(1)
    x = torch.randn(N, 3, HW, HW, generator=g).cuda()
    y = (torch.randint(0, 10, (N,), generator=g) + 1).float().cuda()
    crit = CrossEntropyCriterion()

    def run(sync, defer):
        m = copy.deepcopy(base)
        m.cuda()
        m.training()
        for mod in m.flattened_modules():
            if type(mod).__name__ == "SpatialBatchNormalization" and sync:
                mod.setParallism(1)
                mod.set_sync_group(None, True, force=True)
        fuse(m)
        if not defer:
            for mod in m.flattened_modules():
                if type(mod).__name__ == "SpatialBatchNormalization":
                    mod._defer_ok = False
        m.getParameters()
        m.flat_parameters().enable_shadow(Engine.compute_dtype())
        for _ in range(2):
            m.zeroGradParameters()
            out = m.forward(x)
            loss = float(crit.forward(out, y))
            m.backward(x, crit.backward(out, y))
            torch.cuda.synchronize()
        names = [f"{type(mm).__name__}.{n}" for (mm, n, _g) in m._param_entries()]
        return loss, out.float().clone(), [(nm, p.detach().float().clone()) for nm, p in zip(names, m.parameters()[1])]

    runs = {"local": run(False, True), "local2": run(False, True), "local_nodefer": run(False, False),
            "sync_nodefer": run(True, False), "sync": run(True, True)}

    def cmp(a, b):
        la, oa, ga = runs[a]
        lb, ob, gb = runs[b]
        cs = []
        for (nm, u), (_n, v) in zip(ga, gb):
            if float(v.norm()) == 0 or (nm.endswith(".bias") and "Convolution" in nm):
                continue
            cs.append((float(u.reshape(-1) @ v.reshape(-1) / (u.norm() * v.norm()).clamp_min(1e-30)), nm))
        cs.sort()
        oc = float(oa.reshape(-1) @ ob.reshape(-1) / (oa.norm() * ob.norm()))
        print(f"{a:14s} vs {b:14s} loss {la:.5f} {lb:.5f} out cos {oc:.6f} grad cos min {cs[0][0]:.4f} ({cs[0][1]}) "
              f"p10 {cs[len(cs) // 10][0]:.4f} median {cs[len(cs) // 2][0]:.5f}", flush=True)

    cmp("local", "local2")
    cmp("local", "local_nodefer")
    cmp("local_nodefer", "sync_nodefer")
    cmp("sync_nodefer", "sync")
    cmp("local", "sync")


if __name__ == "__main__":
    main()
