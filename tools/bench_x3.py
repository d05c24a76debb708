#!/usr/bin/env python
"""Per-shape timing of the fp32 direct-operand conv kernels (csrc/conv_x3.hip fwd / stride-1 dgrad,
conv_wgrad.hip F32) on the ResNet-50 geometries at batch B, for every conv_x3 tile.  Prints µs, the
bf16-MFMA-equivalent TF/s (3 × the fp32 FLOPs) and the compulsory HBM GB/s (fp32 in + out).
HIP-event median of R repetitions."""
from __future__ import annotations

import argparse
import json
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(_HERE, "..", "bigdl-1_amd"))
sys.path.insert(0, _HERE)
from bench_conv import RESNET50  # noqa: E402

TILES = [(256, 128), (256, 64), (128, 128), (256, 128 | 256), (256, 64 | 256), (128, 128 | 256), (128, 128 | 512), (128, 128 | 768), (128, 64 | 768)]  # bn | 256: 8x1 / 4x1 waves; | 512: 2-deep ring (2-3 blocks/CU)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--out", default="gpurun_out/bench_x3.jsonl")
    ap.add_argument("--only", default="", help="C,K,R,stride,H filter (e.g. 64,256,1,1,56)")
    args = ap.parse_args()
    import torch
    from bigdl.ops import fp32x3 as F3
    dev = "cuda"
    cl = torch.channels_last

    def timeit(fn):
        for _ in range(2):
            fn()
        ts = []
        for _ in range(args.reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b))
        ts.sort()
        return ts[len(ts) // 2] * 1e3

    out = open(args.out, "w")
    tot = {}
    for (C, K, R, st, H, mult) in RESNET50:
        if C % 32 or (args.only and args.only != f"{C},{K},{R},{st},{H}"):
            continue
        N = args.batch
        pad = R // 2
        P = (H + 2 * pad - R) // st + 1
        x = torch.randn(N, C, H, H, device=dev).contiguous(memory_format=cl)
        w = torch.randn(K, C, R, R, device=dev) * 0.05
        gy = torch.randn(N, K, P, P, device=dev).contiguous(memory_format=cl)
        y = torch.empty(N, K, P, P, device=dev).contiguous(memory_format=cl)
        w2 = F3._w_fwd(w)
        flops = 2.0 * N * P * P * K * C * R * R * 3
        rows = {"C": C, "K": K, "R": R, "s": st, "H": H, "mult": mult}
        for (bm, bn) in TILES:
            us = timeit(lambda: F3._x3(x, w2, y, N, H, H, C, K, R, R, P, P, (st, st), (pad, pad), (1, 1),
                                       tile=(bm, bn)))
            rows[f"fwd_{bm}x{bn}"] = us
        byts = 4.0 * N * (H * H * C + P * P * K)
        if st == 1:
            wt = F3.chunk_split(w.flip(2, 3).permute(1, 2, 3, 0).reshape(C, -1))
            gi = torch.empty(N, C, H, H, device=dev).contiguous(memory_format=cl)
            pd = R - 1 - pad
            for (bm, bn) in TILES:
                us = timeit(lambda: F3._x3(gy, wt, gi, N, P, P, K, C, R, R, H, H, (1, 1), (pd, pd), (1, 1),
                                           tile=(bm, bn)))
                rows[f"dgrad_{bm}x{bn}"] = us
        gw = torch.zeros(K, R, R, C, device=dev).permute(0, 3, 1, 2)
        rows["wgrad"] = timeit(lambda: F3._direct_wgrad(x, gy, gw, 1.0, (st, st), (pad, pad), (1, 1)))
        best_f = min(v for k_, v in rows.items() if k_.startswith("fwd_"))
        best_d = min((v for k_, v in rows.items() if k_.startswith("dgrad_")), default=0.0)
        rows["fwd_tf"] = flops / best_f / 1e6
        rows["fwd_gbs"] = byts / best_f / 1e3
        rows["wgrad_tf"] = flops / rows["wgrad"] / 1e6
        for k_, v in (("fwd", best_f), ("dgrad", best_d), ("wgrad", rows["wgrad"])):
            tot[k_] = tot.get(k_, 0.0) + v * mult
        print(f"C{C:5d} K{K:5d} R{R} s{st} H{H:4d} x{mult}  fwd " +
              " ".join(f"{rows[f'fwd_{a}x{b}']:7.1f}" for a, b in TILES) +
              (("  dgrad " + " ".join(f"{rows[f'dgrad_{a}x{b}']:7.1f}" for a, b in TILES)) if st == 1 else " " * 55) +
              f"  wgrad {rows['wgrad']:8.1f}  | fwd {rows['fwd_tf']:6.0f} TF/s {rows['fwd_gbs']:6.0f} GB/s"
              f"  wgrad {rows['wgrad_tf']:6.0f} TF/s", flush=True)

        out.write(json.dumps(rows) + "\n")
    print("per forward pass (best tile, x multiplicity), us:", {k: round(v, 1) for k, v in tot.items()})


if __name__ == "__main__":
    main()
