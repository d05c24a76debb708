#!/usr/bin/env python
"""Run one conv shape (fwd / dgrad / wgrad) N times — a target for rocprofv3 --pmc."""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bigdl-1_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="256,256,3,1,14")  # C,K,R,stride,H
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--op", default="fwd", choices=["fwd", "fwdstats", "dgrad", "wgrad"])
    ap.add_argument("--f32", action="store_true", help="fp32 operands (bf16x3 direct kernels, conv_x3.hip)")
    a = ap.parse_args()
    import torch
    from bigdl.ops import native_ops as NO
    C, K, R, s, H = [int(v) for v in a.shape.split(",")]
    pad = R // 2
    dt = torch.float32 if a.f32 else torch.bfloat16
    x = torch.randn(a.batch, C, H, H, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, R, R, device="cuda") * 0.05).to(dt)
    y = NO.conv2d_forward(x, w, None, (s, s), (pad, pad))
    gy = torch.randn_like(y)
    gw = torch.zeros(K, R, R, C, device="cuda").permute(0, 3, 1, 2)
    for _ in range(a.iters):
        if a.op == "fwd":
            NO.conv2d_forward(x, w, None, (s, s), (pad, pad))
        elif a.op == "fwdstats":
            NO.conv2d_forward_stats(x, w, None, (s, s), (pad, pad))
        elif a.op == "dgrad":
            NO.conv2d_backward(gy, x, w, (s, s), (pad, pad), need_input=True)
        else:
            NO.conv2d_backward(gy, x, w, (s, s), (pad, pad), need_input=False, gw_acc=gw)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
