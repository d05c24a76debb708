#!/usr/bin/env python
"""Headline benchmark: ResNet-50, ImageNet shape (3×224×224, 1000 classes), synchronous SGD,
bf16 compute with fp32 master weights, synthetic data / random-init weights.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One process per GPU.  ``--gpus N`` with N > 1 outside a launcher (no ``WORLD_SIZE`` in the
environment) re-launches this script under ``torch.distributed.run`` with N ranks BEFORE anything
touches the GPU and exits with the launcher's code; inside a launcher it asserts
``WORLD_SIZE == N``.  N > 1 runs the DistriOptimizer (bucketed RCCL reduce-scatter → sharded fused
SGD → all-gather, overlapped with backward; the reference's ``DistriOptimizerPerf``,
``DL/models/utils/DistriOptimizerPerf.scala:32-146``).  Weak scaling: per-GPU batch fixed (default
256), global batch = 256·N.  The timed region is exactly K full training steps (forward, criterion,
backward, gradient sync, optimizer update) bracketed by barrier + device synchronize; the MAX
elapsed over ranks is reported.  Rank 0 prints one JSON line.  After the timed region a few extra
steps run with per-phase HIP-event timers to report the mean "aggregate gradient" (reduce-scatter
wait), "compute weight" (shard update) and "send weights" (all-gather wait) times — outside the
timed region, so the timers cannot perturb the headline number.

The model, criterion and optimizer are built exactly as the reference's ImageNet ResNet-50
training (``DL/models/resnet/{ResNet,TrainImageNet,Utils}.scala``): convs with bias and
L2Regularizer(1e-4), BN eps 1e-3, SGD(lr 0.1, momentum 0.9, dampening 0, nesterov, wd 1e-4).

The same invocation then times the identical config at the reference's precision — fp32 compute
(bf16x3 operand splits on the matrix cores, fp32 accumulation; ``--fp32-steps``, default 10 on GPU)
— and reports it as ``"fp32": {"value", "ms_per_step", ...}`` next to the bf16 headline ``value``.

``--device cpu`` (gloo, fp32) with ``--batch`` / ``--image-size`` exists to exercise the
multi-rank launch path on a host without GPUs (tests/test_bench_launch.py).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(_HERE, "bigdl-1_amd"))

METRIC = "images/sec (whole node) ResNet-50 ImageNet-shape sync-SGD at 1/2/4/8 MI355X"
PHASES = ("forward", "backward", "aggregate gradient", "compute weight", "send weights")


def _parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--model", default="resnet50", choices=["resnet50"])
    ap.add_argument("--dtype", default=None, help="compute dtype (default bf16 on GPU, fp32 on CPU)")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"])
    ap.add_argument("--comm-dtype", default=os.environ.get("BIGDL_COMM_DTYPE"),
                    help="gradient wire format (fp32 | bf16 | bf16_truncate); default bf16_truncate for "
                         "N > 1 — the reference's FP16CompressedTensor bit format "
                         "(DL/parameters/FP16CompressedTensor.scala:271-277) — and fp32 at N = 1")
    ap.add_argument("--phase-steps", type=int, default=3,
                    help="extra untimed steps with per-phase timers (0 = off)")
    ap.add_argument("--syncbn", action="store_true",
                    help="cross-rank SyncBN in every BN (setParallism), the reference's TrainImageNet option")
    ap.add_argument("--force-distri", action="store_true",
                    help="use the DistriOptimizer (RCCL path) even at world size 1 (path validation)")
    ap.add_argument("--fp32-steps", type=int, default=None,
                    help="also time this many steps of the same config in fp32 compute (the reference's "
                         "precision; bf16x3 on the matrix cores) after the bf16 headline, reported as "
                         "\"fp32\" in the JSON line (default 5 on GPU, 0 on CPU; 0 = off)")
    ap.add_argument("--fp32-warmup", type=int, default=2)
    return ap.parse_args(argv)


def _free_port() -> int:
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    return port


def _relaunch(args) -> int:
    """Start ``args.gpus`` rank processes of this script under torch.distributed.run (the parent
    has imported nothing that touches the GPU) and return the launcher's exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)]
    cmd += sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL
    env.setdefault("OMP_NUM_THREADS", "4")
    return subprocess.call(cmd, env=env)


def _build(args, dev, rank):
    import torch
    from bigdl.models.resnet import ResNet, DatasetType, model_init
    from bigdl.nn import CrossEntropyCriterion
    from bigdl.optim import SGD
    from bigdl.dataset import MiniBatch
    from bigdl.utils.engine import Engine
    from bigdl.utils.random import RNG

    RNG.setSeed(42)
    model = ResNet(1000, depth=50, dataset=DatasetType.ImageNet, image_size=args.image_size)
    model_init(model)
    if args.syncbn:
        from bigdl.nn import SpatialBatchNormalization
        for m in model.flattened_modules():
            if isinstance(m, SpatialBatchNormalization):
                m.setParallism(2)
                if int(os.environ.get("WORLD_SIZE", "1")) == 1:
                    # one rank: still run the cross-rank kernels (local sums -> finalize from sums),
                    # the 1-rank collective being the identity
                    m.set_sync_group(None, True, force=True)
    crit = CrossEntropyCriterion()
    sgd = SGD(learningrate=0.1, learningrate_decay=0.0, weightdecay=1e-4, momentum=0.9, dampening=0.0,
              nesterov=True)
    B, S = args.batch, args.image_size
    g = torch.Generator(device="cpu").manual_seed(1234 + rank)
    # two distinct preallocated batches, alternated every step: no step can reuse work cached from
    # the previous step's input (a real loader hands over a fresh tensor each iteration)
    batches = []
    for _ in range(2):
        x = torch.randn(B, 3, S, S, generator=g).to(dev).to(Engine.compute_dtype())
        if dev.type == "cuda":
            x = x.contiguous(memory_format=torch.channels_last)
        y = (torch.randint(0, 1000, (B,), generator=g) + 1).float().to(dev)
        batches.append(MiniBatch(x, y))
    return model, crit, sgd, batches


def _timed(args, dev, rank, distri, warmup, steps):
    """Build the model / optimizer at the current compute dtype, run ``warmup`` untimed steps (the
    first is the training compile phase), then time exactly ``steps`` steps bracketed by barrier +
    device synchronize; returns (optimizer, batches, max elapsed over ranks, final loss, sync)."""
    import torch
    from bigdl.optim.optimizer import LocalOptimizer
    from bigdl.parallel import comm
    model, crit, sgd, batches = _build(args, dev, rank)
    B = args.batch
    if distri:
        from bigdl.parallel import DistriOptimizer
        opt = DistriOptimizer(model, [batches[0]], crit, sgd, batch_size=B)
    else:
        opt = LocalOptimizer(model, [batches[0]], crit, sgd, batch_size=B)
    opt.prepare()

    def sync():
        if hasattr(opt, "_wait_all_gathers"):
            opt._wait_all_gathers()
        if dev.type == "cuda":
            torch.cuda.synchronize()

    for i in range(warmup):
        opt.train_step(batches[i % 2])
    sync()
    comm.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    loss = None
    for i in range(steps):
        loss = opt.train_step(batches[i % 2])
    sync()
    comm.barrier()
    elapsed = comm.allreduce_max(time.perf_counter() - t0)
    return opt, batches, elapsed, (float(loss) if loss is not None else float("nan")), sync


def main(argv=None):
    args = _parse(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if args.gpus > 1 and env_world is None:
        sys.exit(_relaunch(args))
    world = int(env_world or "1")
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")

    import torch
    from bigdl.utils import config
    if args.comm_dtype is None:
        args.comm_dtype = "bf16_truncate" if (world > 1 or args.force_distri) else "fp32"
    dtype = args.dtype or ("bf16" if args.device == "cuda" else "fp32")
    config.set_property("bigdl.compute.dtype", dtype)
    config.set_property("bigdl.comm.dtype", args.comm_dtype)
    from bigdl.utils.engine import Engine
    if args.force_distri and "RANK" not in os.environ:
        # a single rank outside torchrun: env:// rendezvous with itself on 127.0.0.1
        os.environ.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
                          MASTER_PORT=str(_free_port()))
    distri = world > 1 or args.force_distri
    if args.device == "cpu":
        Engine.init(device="cpu", dist=distri, backend="gloo")
    else:
        Engine.init(dist=distri)
    dev = Engine.device()
    rank = Engine.rank()

    from bigdl.parallel import comm
    B = args.batch
    opt, batches, elapsed, final_loss, sync = _timed(args, dev, rank, distri, args.warmup, args.steps)

    # per-phase means over a few extra (untimed) steps: HIP-event timers on the step stream
    phases = {}
    if args.phase_steps > 0:
        tr = opt.tracer
        tr.enabled = True
        tr.device = dev.type == "cuda"
        tr.host_timers = True
        tr.last_phases = {}
        acc = {}
        for i in range(args.phase_steps):
            opt.train_step(batches[i % 2])
            sync()
            tr.flush()
            for k, v in tr.last_phases.items():
                acc[k] = acc.get(k, 0.0) + v
        for k in PHASES:
            v = comm.allreduce_max(acc.get(k, 0.0) / args.phase_steps)
            if k in acc or v > 0:
                phases[k] = round(v * 1e3, 3)
        tr.enabled = False

    ms = elapsed / args.steps * 1e3
    imgs = B * world * args.steps / elapsed

    # the same config at the reference's precision (fp32 compute: bf16x3 splits on the matrix cores,
    # tests/test_fp32x3.py), timed the same way after the bf16 headline
    fp32 = None
    n32 = args.fp32_steps if args.fp32_steps is not None else (10 if dev.type == "cuda" else 0)
    driver = type(opt).__name__
    if n32 > 0 and dtype != "fp32":
        del opt, batches
        if dev.type == "cuda":
            torch.cuda.empty_cache()
        config.set_property("bigdl.compute.dtype", "fp32")
        Engine.set_compute_dtype("fp32")
        o32, b32, el32, loss32, _ = _timed(args, dev, rank, distri, args.fp32_warmup, n32)
        fp32 = {"value": round(B * world * n32 / el32, 2), "ms_per_step": round(el32 / n32 * 1e3, 3), "steps": n32,
                "warmup": args.fp32_warmup, "dtype": "fp32", "final_loss": loss32}
        del o32, b32
    if rank == 0:
        from bigdl.ops import native_status
        ns = native_status()
        print(json.dumps({
            "metric": METRIC, "value": round(imgs, 2), "unit": "images/sec", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": dtype, "data": "synthetic",
            "config": {"model": "ResNet-50", "global_batch": B * world, "per_gpu_batch": B, "seq_len": None,
                       "image_size": args.image_size, "classes": 1000, "parallelism": f"dp{world}",
                       "optimizer": "SGD(lr=0.1,m=0.9,nesterov,wd=1e-4)+L2Reg(1e-4)",
                       "comm_dtype": args.comm_dtype, "device": dev.type, "syncbn": bool(args.syncbn),
                       "driver": driver},
            "phase_ms_max_over_ranks": phases,
            "final_loss": final_loss, "native_kernels": ns.get("loaded", False),
            "fp32": fp32,
        }), flush=True)
    Engine.shutdown()


if __name__ == "__main__":
    main()
