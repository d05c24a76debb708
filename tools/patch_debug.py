"""Locate the pixels / channels where the halo-patch conv disagrees with the reference."""
import sys
import torch
sys.path.insert(0, "bigdl-1_amd")
from bigdl.ops import native_ops as NO

torch.manual_seed(0)
for (n, h, w) in [(2, 56, 56), (1, 14, 14)]:
    x = torch.randn(n, 64, h, w, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    w4 = (torch.randn(64, 64, 3, 3, device="cuda") * 0.05).bfloat16().contiguous(memory_format=torch.channels_last)
    for trial in range(2):
        y = NO.conv2d_forward(x, w4, None, (1, 1), (1, 1))
        ref = torch.nn.functional.conv2d(x.float(), w4.float(), None, 1, 1)
        bad = ((y.float() - ref).abs() > 0.05)
        idx = bad.nonzero()
        print((n, h, w), "trial", trial, "bad elements", int(bad.sum()), flush=True)
        if idx.numel():
            pix = torch.unique(idx[:, [0, 2, 3]], dim=0)
            chans = torch.unique(idx[:, 1])
            print(" pixels", pix.shape[0], pix[:20].tolist(), flush=True)
            print(" channels", chans.tolist()[:64], flush=True)
            m = pix[:, 0] * h * w + pix[:, 1] * w + pix[:, 2]
            print(" m", m[:40].tolist(), " m%128", (m % 128)[:40].tolist(), flush=True)
