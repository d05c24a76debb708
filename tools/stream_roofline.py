"""Streaming-memory roofline on the MI355X and the BatchNorm apply passes against it.

Sweeps the hand-written 16-B streaming copy / read probes (ops/csrc/roofline.hip) over grid size
and loads-in-flight per thread, then times the native BN forward apply (read y, write a) and
backward apply (read g, x, write gx) at the ResNet-50 bs-256 shapes, reporting each as GB/s of
bytes moved and as a fraction of the best copy rate.  One JSON line per measurement.

    python tools/stream_roofline.py [--mb 512]"""
import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bigdl-1_amd"))
import torch  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=512)
    ap.add_argument("--bn-only", action="store_true", help="skip the probe sweep (best copy rate = --best)")
    ap.add_argument("--best", type=float, default=6003.5)
    a = ap.parse_args()
    from bigdl.ops import native as N
    from bigdl.ops.native import ptr
    lib = N.lib()
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    nbytes = a.mb << 20
    src = torch.empty(nbytes // 2, dtype=torch.bfloat16, device="cuda").normal_()
    dst = torch.empty_like(src)
    best = a.best if a.bn_only else 0.0
    for mode, name, mult in (() if a.bn_only else ((0, "copy", 2), (1, "read", 1))):
        for blocks in (1024, 2048, 4096, 8192, 16384):
            for unroll in (1, 2, 4, 8):
                ms = timed(lambda: lib.bigdl_stream_probe(mode, ptr(src), ptr(dst), C.c_longlong(nbytes), blocks,
                                                          unroll, s))
                gbs = mult * nbytes / ms / 1e6
                if mode == 0:
                    best = max(best, gbs)
                print(json.dumps({"probe": name, "blocks": blocks, "unroll": unroll, "ms": round(ms, 4),
                                  "GB/s": round(gbs, 1)}), flush=True)
    if not a.bn_only:
        ms = timed(lambda: dst.copy_(src))
        print(json.dumps({"probe": "torch copy_", "ms": round(ms, 4), "GB/s": round(2 * nbytes / ms / 1e6, 1)}),
              flush=True)
        print(json.dumps({"best_copy_GB/s": round(best, 1)}), flush=True)
    print(json.dumps({"env": {k: os.environ.get(k) for k in ("BIGDL_BN_UNROLL", "BIGDL_BN_APPLY_BLOCKS")}}), flush=True)
    del src, dst
    # BN apply passes at ResNet-50 bs-256 shapes (M = N·H·W rows, C channels)
    from bigdl.ops import native_ops as NO
    for M, Cc in ((802816, 64), (802816, 256), (200704, 512), (50176, 1024), (12544, 2048)):
        x = torch.randn(M, Cc, device="cuda").bfloat16()
        gy = torch.randn(M, Cc, device="cuda").bfloat16()
        gamma = torch.rand(Cc, device="cuda") + 0.5
        beta = torch.randn(Cc, device="cuda")
        rm, rv = torch.zeros(Cc, device="cuda"), torch.ones(Cc, device="cuda")
        sums = torch.cat([x.float().sum(0), (x.float() ** 2).sum(0)]).contiguous()
        ms = timed(lambda: NO.bn_forward_from_sums(x, sums, M, None, gamma, beta, rm, rv, 0.0, 1e-5, relu=True))
        by = 2 * M * Cc * 2
        print(json.dumps({"pass": "bn_fwd_apply+relu", "M": M, "C": Cc, "ms": round(ms, 4),
                          "GB/s": round(by / ms / 1e6, 1), "of_copy": round(by / ms / 1e6 / best, 3)}), flush=True)
        mean, invstd = x.float().mean(0), torch.rsqrt(x.float().var(0) + 1e-5)
        loc = torch.cat([gy.float().sum(0), (gy.float() * (x.float() - mean)).sum(0)]).contiguous()
        ms = timed(lambda: NO.bn_backward_from_sums(gy, x, gamma, mean, invstd, loc, loc, M))
        by = 3 * M * Cc * 2
        print(json.dumps({"pass": "bn_bwd_apply", "M": M, "C": Cc, "ms": round(ms, 4),
                          "GB/s": round(by / ms / 1e6, 1), "of_copy": round(by / ms / 1e6 / best, 3)}), flush=True)
        del x, gy


if __name__ == "__main__":
    main()
