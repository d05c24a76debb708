"""hipBLASLt (torch.matmul, bf16) on the ResNet-50 1×1-conv GEMM shapes at batch 256: forward
[M,C]·[C,K], dgrad [M,K]·[K,C], wgrad [K,M]·[M,C] — to compare with the implicit-GEMM kernels
(tools/bench_conv.py)."""
import torch

B = 256
SHAPES = [(64, 64, 56), (64, 256, 56), (256, 64, 56), (256, 128, 56), (128, 512, 28), (512, 128, 28),
          (512, 256, 28), (256, 1024, 14), (1024, 256, 14), (1024, 512, 14), (512, 2048, 7), (2048, 512, 7)]


def t(fn, reps=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


for C, K, H in SHAPES:
    M = B * H * H
    x = torch.randn(M, C, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(K, C, device="cuda", dtype=torch.bfloat16)
    gy = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    fl = 2.0 * M * C * K
    f = t(lambda: x @ w.t())
    d = t(lambda: gy @ w)
    g = t(lambda: gy.t() @ x)
    print(f"C {C:5d} K {K:5d} H {H:3d}  fwd {f:.3f}ms {fl / f / 1e9:7.1f}TF  dgrad {d:.3f}ms {fl / d / 1e9:7.1f}TF  "
          f"wgrad {g:.3f}ms {fl / g / 1e9:7.1f}TF", flush=True)
