#!/usr/bin/env python
"""Headline benchmark: ResNet-50, ImageNet shape (3×224×224, 1000 classes), synchronous SGD,
bf16 compute with fp32 master weights, synthetic data / random-init weights.

    python bench.py --gpus N --steps K --warmup W            (N=1)
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One process per GPU; N>1 runs the DistriOptimizer (bucketed RCCL reduce-scatter → sharded fused
SGD → all-gather, overlapped with backward).  Weak scaling: per-GPU batch fixed (default 256),
global batch = 256·N.  The timed region is exactly K full training steps (forward, criterion,
backward, gradient sync, optimizer update) bracketed by barrier + device synchronize; the MAX
elapsed over ranks is reported.  Rank 0 prints one JSON line.

The model, criterion and optimizer are built exactly as the reference's ImageNet ResNet-50
training (``DL/models/resnet/{ResNet,TrainImageNet,Utils}.scala``): convs with bias and
L2Regularizer(1e-4), BN eps 1e-3, SGD(lr 0.1, momentum 0.9, dampening 0, nesterov, wd 1e-4).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(_HERE, "bigdl-1_amd"))

METRIC = "images/sec (whole node) ResNet-50 ImageNet-shape sync-SGD at 1/2/4/8 MI355X"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--model", default="resnet50", choices=["resnet50"])
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--comm-dtype", default=os.environ.get("BIGDL_COMM_DTYPE", "fp32"))
    ap.add_argument("--force-distri", action="store_true",
                    help="use the DistriOptimizer (RCCL path) even at world size 1 (path validation)")
    args = ap.parse_args()

    import torch
    from bigdl.utils import config
    config.set_property("bigdl.compute.dtype", args.dtype)
    config.set_property("bigdl.comm.dtype", args.comm_dtype)
    from bigdl.utils.engine import Engine
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.force_distri and "RANK" not in os.environ:
        # a single rank outside torchrun: env:// rendezvous with itself on 127.0.0.1
        import socket
        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
        sk.close()
        os.environ.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    Engine.init(dist=world > 1 or args.force_distri)
    dev = Engine.device()
    rank = Engine.rank()

    from bigdl.models.resnet import ResNet, DatasetType, model_init
    from bigdl.nn import CrossEntropyCriterion
    from bigdl.optim import SGD
    from bigdl.optim.optimizer import LocalOptimizer
    from bigdl.dataset import MiniBatch
    from bigdl.utils.random import RNG

    RNG.setSeed(42)
    model = ResNet(1000, depth=50, dataset=DatasetType.ImageNet)
    model_init(model)
    crit = CrossEntropyCriterion()
    sgd = SGD(learningrate=0.1, learningrate_decay=0.0, weightdecay=1e-4, momentum=0.9, dampening=0.0,
              nesterov=True)
    B = args.batch
    g = torch.Generator(device="cpu").manual_seed(1234 + rank)
    # two distinct preallocated batches, alternated every step: no step can reuse work cached from
    # the previous step's input (a real loader hands over a fresh tensor each iteration)
    batches = []
    for _ in range(2):
        x = torch.randn(B, 3, 224, 224, generator=g).to(dev).to(Engine.compute_dtype()).contiguous(
            memory_format=torch.channels_last)
        y = (torch.randint(0, 1000, (B,), generator=g) + 1).float().to(dev)
        batches.append(MiniBatch(x, y))
    batch = batches[0]

    if world > 1 or args.force_distri:
        from bigdl.parallel import DistriOptimizer
        opt = DistriOptimizer(model, [batch], crit, sgd, batch_size=B)
    else:
        opt = LocalOptimizer(model, [batch], crit, sgd, batch_size=B)
    opt.prepare()

    from bigdl.parallel import comm
    for i in range(args.warmup):
        opt.train_step(batches[i % 2])
    if hasattr(opt, "_wait_all_gathers"):
        opt._wait_all_gathers()
    comm.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    loss = None
    for i in range(args.steps):
        loss = opt.train_step(batches[i % 2])
    if hasattr(opt, "_wait_all_gathers"):
        opt._wait_all_gathers()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    comm.barrier()
    elapsed = time.perf_counter() - t0
    elapsed = comm.allreduce_max(elapsed)
    final_loss = float(loss) if loss is not None else float("nan")

    ms = elapsed / args.steps * 1e3
    imgs = B * world * args.steps / elapsed
    if rank == 0:
        from bigdl.ops import native_status
        ns = native_status()
        print(json.dumps({
            "metric": METRIC, "value": round(imgs, 2), "unit": "images/sec", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.dtype, "data": "synthetic",
            "config": {"model": "ResNet-50", "global_batch": B * world, "per_gpu_batch": B, "seq_len": None,
                       "image_size": 224, "classes": 1000, "parallelism": f"dp{world}",
                       "optimizer": "SGD(lr=0.1,m=0.9,nesterov,wd=1e-4)+L2Reg(1e-4)",
                       "comm_dtype": args.comm_dtype},
            "final_loss": final_loss, "native_kernels": ns.get("loaded", False),
        }), flush=True)
    Engine.shutdown()


if __name__ == "__main__":
    main()
