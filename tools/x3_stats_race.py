"""Repeat the fp32 conv-epilogue BN statistics (csrc/conv_x3.hip stats epilogue) on one geometry and
compare Σ(y − K), Σ(y − K)² with fp64 sums of the same output, every iteration: an intermittent
mismatch is a race in the epilogue.    python tools/x3_stats_race.py C,K,R,stride,H [iters] [batch]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bigdl-1_amd"))
from bigdl.ops import fp32x3 as F3  # noqa: E402
from bigdl.utils import config  # noqa: E402


def main():
    C, K, R, st, H = (int(v) for v in sys.argv[1].split(","))
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    N = int(sys.argv[3]) if len(sys.argv) > 3 else 128
    config.set_property("bigdl.compute.dtype", "fp32")
    torch.manual_seed(0)
    dev = "cuda"
    x = torch.randn(N, C, H, H, device=dev).contiguous(memory_format=torch.channels_last)
    w = torch.randn(K, C, R, R, device=dev) * (2.0 / (C * R * R)) ** 0.5
    shift = torch.randn(K, device=dev) * 0.1
    rep = 32
    buf = torch.zeros(2 * rep * K, device=dev)
    bad = 0
    worst = 0.0
    for it in range(iters):
        buf.zero_()
        r = F3.conv_forward_stats(x, w, (st, st), (R // 2, R // 2), (1, 1), (buf, rep), shift)
        assert r is not NotImplemented
        y = r[0]
        torch.cuda.synchronize()
        yd = y.double().permute(0, 2, 3, 1).reshape(-1, K) - shift.double()
        s1, s2 = yd.sum(0), (yd * yd).sum(0)
        b = buf.double().reshape(2, rep, K).sum(1)
        e1 = float(((b[0] - s1).abs() / s2.sqrt()).max())
        e2 = float(((b[1] - s2).abs() / s2).max())
        worst = max(worst, e2)
        if e2 > 1e-4 or e1 > 1e-4:
            bad += 1
            if bad <= 5:
                print(f"iter {it}: sum err {e1:.3g} (in sd·sqrt(M) units) sumsq rel err {e2:.3g}", flush=True)
    print(f"{sys.argv[1]} N{N}: {bad} / {iters} iterations with a statistics mismatch; worst sumsq rel err {worst:.3g}",
          flush=True)


if __name__ == "__main__":
    main()
