#!/usr/bin/env python
"""Pointwise (1×1) conv shapes of ResNet-50 (bs 256): native fwd / fwd+stats / dgrad vs the
hipBLASLt GEMM of the same product and a copy of the same bytes (memory roofline reference)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bigdl-1_amd"))

SHAPES = [  # C, K, stride, H (input), multiplicity per step
    (64, 64, 1, 56, 1), (64, 256, 1, 56, 4), (256, 64, 1, 56, 2), (256, 128, 1, 56, 1),
    (128, 512, 1, 28, 4), (512, 128, 1, 28, 3), (512, 256, 1, 28, 1), (256, 512, 2, 56, 1),
    (256, 1024, 1, 14, 6), (1024, 256, 1, 14, 5), (1024, 512, 1, 14, 1), (512, 1024, 2, 28, 1),
    (512, 2048, 1, 7, 3), (2048, 512, 1, 7, 2), (1024, 2048, 2, 14, 1),
]
SHAPES3 = [  # 3×3 convs (pad 1): C, K, stride, H (input), multiplicity
    (64, 64, 1, 56, 3), (128, 128, 2, 56, 1), (128, 128, 1, 28, 3), (256, 256, 2, 28, 1),
    (256, 256, 1, 14, 5), (512, 512, 2, 14, 1), (512, 512, 1, 7, 2),
]


def timeit(fn, iters=20):
    import torch
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # µs


def main():
    cfgs = os.environ.get("CFGS")
    if cfgs:  # one run per tile pin set, e.g. CFGS="-;BIGDL_CONV_BN=64;BIGDL_CONV_BK=64"
        for c in cfgs.split(";"):
            for k in ("BIGDL_CONV_BN", "BIGDL_CONV_BK", "BIGDL_CONV_BM"):
                os.environ.pop(k, None)
            for kv in c.split(","):
                if "=" in kv:
                    k, v = kv.split("=")
                    os.environ[k] = v
            print(json.dumps({"config": c}), flush=True)
            run()
        return
    run()


def run():
    import torch
    from bigdl.ops import native_ops as NO
    bs = int(os.environ.get("BS", "256"))
    tot = {"fwd": 0.0, "fwdstats": 0.0, "dgrad": 0.0, "mm": 0.0, "copy": 0.0}
    tot["wgrad"] = 0.0
    tot["vendor_fwd"] = tot["vendor_dgrad"] = tot["vendor_wgrad"] = 0.0
    only3 = os.environ.get("ONLY3") == "1"
    for C, K, s, H, mult, R in ([] if only3 else [v + (1,) for v in SHAPES]) + [v + (3,) for v in SHAPES3]:
        pd = R // 2
        x = torch.randn(bs, C, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        w = (torch.randn(K, C, R, R, device="cuda") * 0.05).bfloat16()
        y = NO.conv2d_forward(x, w, None, (s, s), (pd, pd))
        gy = torch.randn_like(y)
        P = y.shape[2]
        M = bs * P * P
        t = {}
        gw = torch.zeros(K, C, R, R, device="cuda")
        t["fwd"] = timeit(lambda: NO.conv2d_forward(x, w, None, (s, s), (pd, pd)))
        t["fwdstats"] = timeit(lambda: NO.conv2d_forward_stats(x, w, None, (s, s), (pd, pd)))
        t["dgrad"] = timeit(lambda: NO.conv2d_backward(gy, x, w, (s, s), (pd, pd), need_input=True))
        t["wgrad"] = timeit(lambda: NO.conv2d_backward(gy, x, w, (s, s), (pd, pd), need_input=False, gw_acc=gw))
        if s == 1 and R == 1:
            a2 = x.permute(0, 2, 3, 1).reshape(M, C)
            w2 = w.view(K, C)
            t["mm"] = timeit(lambda: torch.mm(a2, w2.t()))
        else:
            t["mm"] = 0.0
        if os.environ.get("VENDOR_CONV") == "1":
            # the vendor library's conv of the same shape (torch → MIOpen, NHWC bf16), forward / data
            # gradient / weight gradient.  For a tuned baseline run with MIOPEN_FIND_MODE=NORMAL (the
            # find step benchmarks every MIOpen solver on the shape) and VENDOR_BENCH=1
            # (torch.backends.cudnn.benchmark: the fastest algorithm is chosen per shape, cached)
            torch.backends.cudnn.benchmark = os.environ.get("VENDOR_BENCH") == "1"
            wcl = w.contiguous(memory_format=torch.channels_last)
            t["vendor_fwd"] = timeit(lambda: torch.nn.functional.conv2d(x, wcl, None, s, pd))
            t["vendor_dgrad"] = timeit(lambda: torch.nn.grad.conv2d_input(x.shape, wcl, gy, s, pd))
            t["vendor_wgrad"] = timeit(lambda: torch.nn.grad.conv2d_weight(x, w.shape, gy, s, pd))
        else:
            t["vendor_fwd"] = t["vendor_dgrad"] = t["vendor_wgrad"] = 0.0
        src = torch.empty(M * K + x.numel(), dtype=torch.bfloat16, device="cuda")
        dst = torch.empty_like(src)
        t["copy"] = timeit(lambda: dst.copy_(src)) / 2  # read+write of (in + out) ≈ 2× the conv's bytes
        flops = 2.0 * M * C * K * R * R
        byts = 2.0 * (x.numel() + M * K)
        row = {"C": C, "K": K, "R": R, "s": s, "H": H, "mult": mult, **{k: round(v, 1) for k, v in t.items()},
               "fwd_TF": round(flops / t["fwd"] / 1e6, 1), "dgrad_TF": round(flops / t["dgrad"] / 1e6, 1),
               "wgrad_TF": round(flops / t["wgrad"] / 1e6, 1), "fwd_TBs": round(byts / t["fwd"] / 1e6, 2)}
        print(json.dumps(row), flush=True)
        for k in tot:
            tot[k] += t[k] * mult
    print(json.dumps({"per_step_ms": {k: round(v / 1e3, 3) for k, v in tot.items()}}))


if __name__ == "__main__":
    main()
