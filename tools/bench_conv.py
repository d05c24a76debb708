#!/usr/bin/env python
"""Per-shape throughput of the native conv kernels (fwd / dgrad / wgrad) on the ResNet-50 layer
shapes at batch B, next to MIOpen (torch.nn.functional.conv2d / its autograd) on the same tensors.

Prints one line per unique shape with TFLOP/s and writes a JSON summary.  Timing: HIP events,
median of R repetitions after warmup; every variant runs in the same process on the same data.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(_HERE, "..", "bigdl-1_amd"))

# (C, K, R, stride, H) for ResNet-50 v1 (stride on the 3x3), with multiplicity per forward pass
RESNET50 = [
    (3, 64, 7, 2, 224, 1),
    (64, 64, 1, 1, 56, 1), (64, 64, 3, 1, 56, 3), (64, 256, 1, 1, 56, 4), (256, 64, 1, 1, 56, 2),
    (256, 128, 1, 1, 56, 1), (128, 128, 3, 2, 56, 1), (128, 512, 1, 1, 28, 4), (256, 512, 1, 2, 56, 1),
    (512, 128, 1, 1, 28, 3), (128, 128, 3, 1, 28, 3),
    (512, 256, 1, 1, 28, 1), (256, 256, 3, 2, 28, 1), (256, 1024, 1, 1, 14, 6), (512, 1024, 1, 2, 28, 1),
    (1024, 256, 1, 1, 14, 5), (256, 256, 3, 1, 14, 5),
    (1024, 512, 1, 1, 14, 1), (512, 512, 3, 2, 14, 1), (512, 2048, 1, 1, 7, 3), (1024, 2048, 1, 2, 14, 1),
    (2048, 512, 1, 1, 7, 2), (512, 512, 3, 1, 7, 2),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--out", default="gpurun_out/bench_conv.json")
    ap.add_argument("--no-miopen", action="store_true")
    ap.add_argument("--wgrad-sweep", default="", help="comma list of wgrad target block counts to A/B")
    args = ap.parse_args()
    import torch
    import torch.nn.functional as F
    from bigdl.ops import native_ops as NO

    dev = "cuda"
    bf = torch.bfloat16

    def timeit(fn):
        for _ in range(3):
            fn()
        ts = []
        for _ in range(args.reps):
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b))
        ts.sort()
        return ts[len(ts) // 2]

    rows = []
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0, "mi_fwd": 0.0, "mi_bwd": 0.0}
    for (C, K, R, s, H, mult) in RESNET50:
        B = args.batch
        pad = R // 2
        x = torch.randn(B, C, H, H, device=dev).to(bf).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(K, C, R, R, device=dev) * (2.0 / (C * R * R)) ** 0.5).to(bf)
        y = NO.conv2d_forward(x, w, None, (s, s), (pad, pad))
        P = y.shape[2]
        flops = 2.0 * B * P * P * K * C * R * R
        gy = torch.randn_like(y)
        gw = torch.zeros(K, C, R, R, device=dev, dtype=torch.float32)
        t_f = timeit(lambda: NO.conv2d_forward(x, w, None, (s, s), (pad, pad)))
        t_d = timeit(lambda: NO.conv2d_backward(gy, x, w, (s, s), (pad, pad), need_input=True)) if C != 3 else 0.0
        t_w = timeit(lambda: NO.conv2d_backward(gy, x, w, (s, s), (pad, pad), need_input=False, gw_acc=gw))
        sweep = {}
        for tb in [int(v) for v in args.wgrad_sweep.split(",") if v]:
            old = NO._WGRAD_TARGET_BLOCKS[0]
            NO._WGRAD_TARGET_BLOCKS[0] = tb
            sweep[tb] = timeit(lambda: NO.conv2d_backward(gy, x, w, (s, s), (pad, pad), need_input=False, gw_acc=gw))
            NO._WGRAD_TARGET_BLOCKS[0] = old
            tot.setdefault(f"wgrad@{tb}", 0.0)
            tot[f"wgrad@{tb}"] += sweep[tb] * mult
        row = {"C": C, "K": K, "R": R, "s": s, "H": H, "P": P, "mult": mult, "gflop": flops / 1e9,
               "fwd_ms": t_f, "dgrad_ms": t_d, "wgrad_ms": t_w,
               "fwd_tf": flops / t_f / 1e9, "dgrad_tf": flops / t_d / 1e9 if t_d else None,
               "wgrad_tf": flops / t_w / 1e9, "wgrad_sweep_ms": sweep}
        if not args.no_miopen:
            xr = x.detach().clone().requires_grad_(True)
            wr = w.detach().clone().requires_grad_(True)
            t_mf = timeit(lambda: F.conv2d(x, w, None, s, pad))
            yr = F.conv2d(xr, wr, None, s, pad)

            def mi_bwd():
                torch.autograd.grad(yr, (xr, wr), gy, retain_graph=True)
            t_mb = timeit(mi_bwd)
            row.update({"miopen_fwd_ms": t_mf, "miopen_bwd_ms": t_mb, "miopen_fwd_tf": flops / t_mf / 1e9})
            tot["mi_fwd"] += t_mf * mult
            tot["mi_bwd"] += t_mb * mult
        tot["fwd"] += t_f * mult
        tot["dgrad"] += t_d * mult
        tot["wgrad"] += t_w * mult
        rows.append(row)
        print(f"C{C:5d} K{K:5d} R{R} s{s} H{H:3d} x{mult}  fwd {t_f:7.3f}ms {row['fwd_tf']:7.1f}TF  "
              f"dgrad {t_d:7.3f}ms {row['dgrad_tf'] or 0:7.1f}TF  wgrad {t_w:7.3f}ms {row['wgrad_tf']:7.1f}TF"
              + (f"  | miopen fwd {row['miopen_fwd_ms']:7.3f}ms bwd {row['miopen_bwd_ms']:7.3f}ms"
                 if "miopen_fwd_ms" in row else "") + (f"  sweep {sweep}" if sweep else ""), flush=True)
    print("per-step totals (ms, weighted by multiplicity):", json.dumps({k: round(v, 3) for k, v in tot.items()}))
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    with open(args.out, "w") as f:
        json.dump({"batch": args.batch, "rows": rows, "totals_ms": tot}, f, indent=1)


if __name__ == "__main__":
    main()
