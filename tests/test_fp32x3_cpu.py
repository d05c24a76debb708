"""CPU checks of the bf16x3 fp32 scheme (ops/fp32x3.py) and of the compile-phase tile pinning
(ops/native_ops._tiled_launch): the algebra the GPU path relies on — one GEMM over the
[hi | hi | lo]·[hi | lo | hi] concatenation equals the three-product sum and is fp32-class
accurate — and the pin / reset protocol around a conv launch."""
import torch

from bigdl.ops import fp32x3 as F3


def _split_ref(t):
    hi = t.bfloat16()
    lo = (t - hi.float()).bfloat16()
    return hi, lo


def test_bf16x3_concatenated_gemm_is_fp32_class():
    g = torch.Generator().manual_seed(0)
    a = torch.randn(64, 300, generator=g)
    b = torch.randn(48, 300, generator=g)
    ah, al = _split_ref(a)
    bh, bl = _split_ref(b)
    # part codes as the kernels use them: A = [hi | hi | lo] (HHL), B = [hi | lo | hi] (HLH)
    assert F3.HHL == 0b100 and F3.HLH == 0b010
    a3 = torch.cat([ah, ah, al], 1).double()
    b3 = torch.cat([bh, bl, bh], 1).double()
    got = a3 @ b3.t()
    three = ah.double() @ bh.double().t() + ah.double() @ bl.double().t() + al.double() @ bh.double().t()
    torch.testing.assert_close(got, three, rtol=1e-12, atol=1e-12)
    ref = a.double() @ b.double().t()
    rel = float((got - ref).norm() / ref.norm())
    bf = float((ah.double() @ bh.double().t() - ref).norm() / ref.norm())
    assert rel < 2e-5 and bf > 100 * rel, (rel, bf)


def test_tiled_launch_passes_the_pinned_tile():
    from bigdl.ops import native_ops as NO
    key = ("geom",)
    got = []
    NO._TILE["table"].pop(key, None)
    NO._tiled_launch(key, got.append)
    assert got == [(0, 0, 0)]  # heuristic
    NO._TILE["table"][key] = (64, 64, 128)
    rec = NO._TILE["record"] = []
    try:
        NO._tiled_launch(key, got.append)
    finally:
        NO._TILE["record"] = None
        NO._TILE["table"].pop(key, None)
    assert got == [(0, 0, 0), (64, 64, 128)]
    assert len(rec) == 1 and rec[0][0] == key
