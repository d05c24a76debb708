"""fp32 BatchNorm apply pass in isolation (csrc/batchnorm.hip k_bn32_apply) on every ResNet-50 shape at
batch 256: forward (BN + ReLU, via bigdl_bn32_fwd_infer: 8 B/elem) and backward (gx = A·g + B·x + C,
via bigdl_bn32_bwd_partials: 12 B/elem), µs and TB/s per shape and the per-step total weighted by how
often the shape occurs.  Knobs: BIGDL_BN32_UNROLL, BIGDL_BN32_BLOCKS (read once per process)."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bigdl-1_amd"))
import torch
from bigdl.ops import native as N
from bigdl.ops.native import ptr

# (pixels per image, C, forward applies per step, backward applies per step)
SHAPES = [(112 * 112, 64, 1, 1), (56 * 56, 64, 6, 6), (56 * 56, 256, 4, 3), (28 * 28, 128, 8, 8),
          (28 * 28, 512, 5, 4), (14 * 14, 256, 12, 12), (14 * 14, 1024, 7, 6), (7 * 7, 512, 6, 6),
          (7 * 7, 2048, 4, 3)]


def main():
    lib = N.lib()
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    res, tot_f, tot_b = [], 0.0, 0.0
    for pix, c, nf, nb in SHAPES:
        M = 256 * pix
        x = torch.randn(M * c, device="cuda")
        y = torch.empty_like(x)
        g = torch.randn_like(x)
        gamma, beta = torch.rand(c, device="cuda") + 0.5, torch.randn(c, device="cuda")
        rm, rv = torch.zeros(c, device="cuda"), torch.ones(c, device="cuda")
        coef = torch.empty(3 * c, device="cuda")
        ggam, gbet = torch.zeros(c, device="cuda"), torch.zeros(c, device="cuda")
        part = torch.zeros(2 * c, device="cuda")
        mean, inv = torch.zeros(c, device="cuda"), torch.ones(c, device="cuda")

        def fwd():
            lib.bigdl_bn32_fwd_infer(ptr(x), ptr(y), C.c_longlong(M), C.c_int(c), ptr(gamma), ptr(beta), ptr(rm),
                                     ptr(rv), ptr(None), C.c_float(1e-5), ptr(coef), C.c_int(1), s)

        def bwd():
            lib.bigdl_bn32_bwd_partials(ptr(g), ptr(x), ptr(y), C.c_longlong(M), C.c_int(c), ptr(gamma), ptr(mean),
                                        ptr(inv), ptr(ggam), ptr(gbet), C.c_float(1.0), ptr(None), C.c_float(1.0),
                                        ptr(part), C.c_int(1), ptr(coef), ptr(None), s)
        out = {"pix": pix, "C": c}
        for name, fn, bpe in (("fwd", fwd, 8), ("bwd", bwd, 12)):
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / 20 * 1e3
            out[name + "_us"] = round(us, 1)
            out[name + "_TBs"] = round(bpe * M * c / us / 1e6, 2)
        tot_f += nf * out["fwd_us"]
        tot_b += nb * out["bwd_us"]
        res.append(out)
        del x, y, g
    for r in res:
        print(json.dumps(r))
    print(json.dumps({"unroll": os.environ.get("BIGDL_BN32_UNROLL", "4"), "blocks": os.environ.get("BIGDL_BN32_BLOCKS", "default"),
                      "fwd_ms_per_step": round(tot_f / 1e3, 3), "bwd_ms_per_step": round(tot_b / 1e3, 3)}))


if __name__ == "__main__":
    main()
