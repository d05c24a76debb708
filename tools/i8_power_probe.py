"""Does the int8 conv's speed depend on the activation codes?  Times one VGG16 conv (conv3_2 shape,
bs128) of ops/csrc/conv_i8.hip on int8 inputs filled with 0, with -128, with random codes, and on
unsigned-offset inputs (the correction path) — same kernel, same grid, only the data differ."""
import sys
import torch
sys.path.insert(0, "bigdl-1_amd")
from bigdl.ops import native_ops as NO
from bigdl.ops import reference as R

torch.manual_seed(0)
N, C, H, W, K = 128, 256, 56, 56, 256
w = torch.randn(K, C, 3, 3)
q, ws = R.quant_rows(w.reshape(K, -1))
wq, ldw = NO.conv_i8_weight(q.cuda(), K, C, 3, 3)
ws = ws.cuda().float()
bias = torch.zeros(K, device="cuda")


def run(x, u8, label, reps=20):
    x._qscale = 0.01
    x._qzero = 0
    if u8:
        t = NO._i8_act(*x.shape, x.device, True)
        t.copy_(x)
        t.untyped_storage()[x.numel():].fill_(-128 & 0xFF)
        x = NO._tag(t, 0.01, True)
    tabs = NO.conv_i8_u8_bias(wq, ldw, K, 3, 3, C, 0.01, ws, bias) if u8 else None
    f = lambda: NO.conv2d_i8_forward_static(x, wq, ldw, ws, bias, K, 3, 3, (1, 1), (1, 1), (1, 1), (H, W),
                                            relu=True, out_scale=0.05, u8_bias=tabs)
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    print(f"{label:28s} {e0.elapsed_time(e1) / reps * 1e3:8.1f} us", flush=True)


shape = (N, C, H, W)
mk = lambda t: t.to(torch.int8).contiguous(memory_format=torch.channels_last)
zeros = mk(torch.zeros(shape, device="cuda"))
m128 = mk(torch.full(shape, -128.0, device="cuda"))
rnd = mk(torch.randint(-128, 128, shape, device="cuda"))
relu_like = mk((torch.randn(shape, device="cuda").clamp_min(0) * 40).clamp(max=127))
for rep in range(2):
    run(zeros, False, "signed, all 0")
    run(m128, False, "signed, all -128")
    run(rnd, False, "signed, random")
    run(relu_like, False, "signed, relu-like")
    run(mk(relu_like.float() * 2 - 128), True, "u8-offset, relu-like")
    run(zeros, True, "u8-offset path, all 0")
