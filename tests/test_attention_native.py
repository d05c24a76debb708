"""Fused attention kernels (ops/csrc/attention.hip) against the fp32 reference op
(``ops/reference.py::attention_forward/backward`` — the math of ``Attention.scala:30-111``):
forward O and LSE, backward dQ/dK/dV, with Q/K/V read as column slices of one fused
[B·L][3·H] projection buffer, an additive padding bias, the in-kernel causal mask, cross
attention (Lq ≠ Lk, neither a multiple of the 64-row tile) and attention dropout (the kernel's
counter-hash mask reproduced on the host)."""
import math

import pytest
import torch

from bigdl.ops import reference as R

pytestmark = pytest.mark.gpu
dev = "cuda"


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


def _case(B, Hh, D, Lq, Lk, bias_kind, causal, keep, seed=123):
    from bigdl.ops import native_ops as NO
    g = torch.Generator().manual_seed(7)
    H = Hh * D
    xq = torch.randn(B * Lq, 3 * H, generator=g).to(torch.bfloat16)
    xk = torch.randn(B * Lk, 3 * H, generator=g).to(torch.bfloat16)
    q, k, v = xq[:, :H], xk[:, H:2 * H], xk[:, 2 * H:]
    bias = None
    if bias_kind == "pad":
        pad = torch.zeros(B, 1, 1, Lk)
        pad[0, ..., Lk - 7:] = -1e9
        bias = pad
    elif bias_kind == "full":
        bias = torch.randn(B, Hh, Lq, Lk, generator=g)
    scale = D ** -0.5
    o_ref, lse_ref = R.attention_forward(q, k, v, B, Hh, Lq, Lk, D, scale, bias, causal, keep, seed)
    gq, gk = xq.to(dev), xk.to(dev)
    qd, kd, vd = gq[:, :H], gk[:, H:2 * H], gk[:, 2 * H:]
    bd = bias.to(dev) if bias is not None else None
    o, lse = NO.attention_forward(qd, kd, vd, B, Hh, Lq, Lk, D, scale, bd, causal, keep, seed)
    torch.cuda.synchronize()
    assert _rel(o.cpu(), o_ref) < 1.5e-2, _rel(o.cpu(), o_ref)
    assert float((lse.cpu() - lse_ref).abs().max()) < 2e-2
    dout = torch.randn(B * Lq, H, generator=g).to(torch.bfloat16)
    dq_r, dk_r, dv_r = R.attention_backward(dout, q, k, v, o_ref, lse_ref, B, Hh, Lq, Lk, D, scale, bias, causal,
                                            keep, seed)
    dqkv = torch.empty(B * Lk if Lq == Lk else 0, 3 * H, dtype=torch.bfloat16, device=dev)
    if Lq == Lk:  # results straight into one fused gradient buffer
        dq, dk, dv = NO.attention_backward(dout.to(dev), qd, kd, vd, o, lse, B, Hh, Lq, Lk, D, scale, bd, causal,
                                           keep, seed, dq=dqkv[:, :H], dk=dqkv[:, H:2 * H], dv=dqkv[:, 2 * H:])
    else:
        dq, dk, dv = NO.attention_backward(dout.to(dev), qd, kd, vd, o, lse, B, Hh, Lq, Lk, D, scale, bd, causal,
                                           keep, seed)
    torch.cuda.synchronize()
    for name, a, b in (("dq", dq, dq_r), ("dk", dk, dk_r), ("dv", dv, dv_r)):
        assert _rel(a.cpu(), b) < 3e-2, (name, _rel(a.cpu(), b))


@pytest.mark.parametrize("D", [32, 64, 96, 128])
def test_self_attention_no_bias(D):
    _case(2, 4, D, 100, 100, None, False, 1.0)


@pytest.mark.parametrize("D", [32, 64, 96, 128])
def test_causal_mask(D):
    _case(2, 3, D, 130, 130, None, True, 1.0)


def test_padding_bias_cross_attention():
    _case(3, 2, 64, 70, 130, "pad", False, 1.0)


def test_full_bias_d128():
    _case(2, 2, 128, 64, 96, "full", False, 1.0)


@pytest.mark.parametrize("causal", [False, True])
def test_dropout_matches_host_mask(causal):
    _case(2, 4, 64, 96, 96, None, causal, 0.8, seed=987)


def test_lse_is_log2_sum_exp():
    from bigdl.ops import native_ops as NO
    B, Hh, D, L = 1, 2, 64, 64
    q = torch.randn(B * L, Hh * D, device=dev).to(torch.bfloat16)
    o, lse = NO.attention_forward(q, q, q, B, Hh, L, L, D, 1.0 / math.sqrt(D))
    s = R._attn_probs(q.cpu(), q.cpu(), B, Hh, L, L, D, 1.0 / math.sqrt(D), None, False)
    torch.testing.assert_close(lse.cpu(), torch.logsumexp(s, -1) / math.log(2.0), rtol=0, atol=2e-2)
