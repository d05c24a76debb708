"""Short-reduction int8 convs (the 1×1 convs of ResNet-50 over ≤ 256 input channels, KT ≤ 2 k-tiles)
under each short-K tile variant of ops/csrc/conv_i8.hip (bigdl_conv_i8_set_shortk: 0 = 128×128 2-deep
ring, 2 blocks/CU; 1 = 64×128 2-deep ring, 3 blocks/CU; 2 = 64×128, no ring for one k-tile, 5 blocks/CU),
batch 256, unsigned int8 in/out as in the calibrated chain, with and without the int8 residual of a
block tail.  Prints µs per launch and the HBM rate of the launch's compulsory bytes; checks that every
variant writes the same codes."""
import sys

import torch

sys.path.insert(0, "bigdl-1_amd")
from bigdl.ops import native_ops as NO  # noqa: E402
from bigdl.ops import reference as R  # noqa: E402

SHAPES = [  # (C, K, H, residual)
    (64, 64, 56, False), (64, 256, 56, True), (64, 256, 56, False), (256, 64, 56, False), (256, 128, 56, False),
    (128, 512, 28, True), (256, 1024, 14, True), (128, 128, 28, False),
]


def u8_act(shape, scale):
    N, C, H, W = shape
    t = NO._i8_act(N, C, H, W, "cuda", True)
    t.copy_(torch.randint(-128, 128, (N, C, H, W), device="cuda", dtype=torch.int8))
    t.untyped_storage()[t.numel():].fill_(0x80)
    return NO._tag(t, scale, True)


def main():
    torch.manual_seed(0)
    lib = NO._lib()
    N = 256
    shapes, variants = SHAPES, (0, 1, 2)
    if len(sys.argv) > 1:  # one shape / variant (PMC passes): C,K,H,res variant
        c, k, h, r = (int(v) for v in sys.argv[1].split(","))
        shapes, variants = [(c, k, h, bool(r))], (int(sys.argv[2]) if len(sys.argv) > 2 else 0,)
    for (C, K, H, res) in shapes:
        w = torch.randn(K, C, 1, 1)
        q, ws = R.quant_rows(w.reshape(K, -1))
        wq, ldw = NO.conv_i8_weight(q.cuda(), K, C, 1, 1)
        ws = ws.cuda().float()
        bias = torch.randn(K, device="cuda") * 0.1
        x = u8_act((N, C, H, H), 0.02)
        r = u8_act((N, K, H, H), 0.03) if res else None
        ub = NO.conv_i8_u8_bias(wq, ldw, K, 1, 1, C, 0.02, ws, bias)
        f = lambda: NO.conv2d_i8_forward_static(x, wq, ldw, ws, bias, K, 1, 1, (1, 1), (0, 0), (1, 1), (H, H),  # noqa: E731
                                                relu=True, out_scale=0.04, out_u8=True, u8_bias=ub, residual=r)
        byt = N * H * H * (C + K + (K if res else 0))
        outs, line = [], []
        for v in variants:
            lib.bigdl_conv_i8_set_shortk(v)
            y = f()
            torch.cuda.synchronize()
            outs.append(y.clone())
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            best = 1e9
            for _ in range(3):
                e0.record()
                for _ in range(10):
                    f()
                e1.record()
                torch.cuda.synchronize()
                best = min(best, e0.elapsed_time(e1) / 10 * 1e3)
            line.append(f"v{v} {best:7.1f} us {byt / best / 1e6:5.2f} TB/s")
        lib.bigdl_conv_i8_set_shortk(0)
        same = all(bool(torch.equal(outs[0], o)) for o in outs[1:])
        print(f"C {C:4d} K {K:4d} H {H:3d} res {int(res)} | " + " | ".join(line) + f" | same {same}", flush=True)


if __name__ == "__main__":
    main()
