"""One fp32 direct-operand conv kernel (csrc/conv_x3.hip fwd / stride-1 dgrad, conv_wgrad.hip F32) on one
ResNet-50 geometry, repeated — the program a rocprofv3 --pmc pass wraps (tools/pmc_x3.sh).
    python tools/x3_one.py C,K,R,stride,H {fwd|dgrad|wgrad} [iters] [bm,bn]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bigdl-1_amd"))
from bigdl.ops import fp32x3 as F3  # noqa: E402


def main():
    C, K, R, st, H = (int(v) for v in sys.argv[1].split(","))
    op = sys.argv[2]
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    tile = tuple(int(v) for v in sys.argv[4].split(",")) if len(sys.argv) > 4 else None
    N, dev, cl = 256, "cuda", torch.channels_last
    pad = R // 2
    P = (H + 2 * pad - R) // st + 1
    x = torch.randn(N, C, H, H, device=dev).contiguous(memory_format=cl)
    w = torch.randn(K, C, R, R, device=dev) * 0.05
    gy = torch.randn(N, K, P, P, device=dev).contiguous(memory_format=cl)
    if op == "fwd":
        y = torch.empty(N, K, P, P, device=dev).contiguous(memory_format=cl)
        w2 = F3._w_fwd(w)
        f = lambda: F3._x3(x, w2, y, N, H, H, C, K, R, R, P, P, (st, st), (pad, pad), (1, 1), tile=tile)  # noqa: E731
    elif op == "dgrad":
        wt = F3.chunk_split(w.flip(2, 3).permute(1, 2, 3, 0).reshape(C, -1))
        gi = torch.empty(N, C, H, H, device=dev).contiguous(memory_format=cl)
        pd = R - 1 - pad
        f = lambda: F3._x3(gy, wt, gi, N, P, P, K, C, R, R, H, H, (1, 1), (pd, pd), (1, 1), tile=tile)  # noqa: E731
    else:
        gw = torch.zeros(K, R, R, C, device=dev).permute(0, 3, 1, 2)
        f = lambda: F3._direct_wgrad(x, gy, gw, 1.0, (st, st), (pad, pad), (1, 1))  # noqa: E731
    for _ in range(iters):
        f()
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
