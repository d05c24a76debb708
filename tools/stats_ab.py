"""Cost of the BN-statistics conv epilogue: for a few ResNet-50 (bs 256) shapes, time the plain
forward conv against the forward with shifted Σ/Σ² partials (what training runs) and print which
kernels each launches (run under ``rocprofv3 --kernel-trace --stats`` for the names)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bigdl-1_amd"))

SHAPES = [(64, 64, 1, 1, 56), (64, 256, 1, 1, 56), (256, 64, 1, 1, 56), (64, 64, 3, 1, 56),
          (128, 128, 3, 1, 28), (256, 256, 3, 1, 14), (1024, 256, 1, 1, 14)]


def timeit(fn, n=20):
    import torch
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / n * 1e3


def main():
    import torch
    from bigdl.ops import native_ops as NO
    bs = int(os.environ.get("BS", "256"))
    for C, K, R, s, H in SHAPES:
        pd = R // 2
        x = torch.randn(bs, C, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        w = (torch.randn(K, C, R, R, device="cuda") * 0.05).bfloat16()
        shift = torch.zeros(K, device="cuda")
        row = {"C": C, "K": K, "R": R, "s": s, "H": H}
        row["fwd"] = round(timeit(lambda: NO.conv2d_forward(x, w, None, (s, s), (pd, pd))), 1)
        row["stats"] = round(timeit(lambda: NO.conv2d_forward_stats(x, w, None, (s, s), (pd, pd))), 1)
        row["stats_shift"] = round(timeit(lambda: NO.conv2d_forward_stats(x, w, None, (s, s), (pd, pd),
                                                                          shift=shift)), 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
