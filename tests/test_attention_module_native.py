"""Attention / FeedForwardNetwork / Transformer on their native device path (fused QKV GEMM →
attention.hip → output GEMM; GEMM+bias+ReLU FFN) against the same modules' fp32 host path
(the torch composition of ``Attention.scala:30-111`` / ``FeedForwardNetwork.scala``): outputs,
input gradients and every parameter gradient."""
import copy

import pytest
import torch

from bigdl.utils.table import T

pytestmark = pytest.mark.gpu
dev = "cuda"


def _cos(a, b):
    a, b = a.double().reshape(-1), b.double().reshape(-1)
    return float((a @ b) / (a.norm() * b.norm()).clamp_min(1e-30))


def _gpu(m):
    from bigdl.utils import config
    from bigdl.utils.engine import Engine
    config.set_property("bigdl.compute.dtype", "bf16")
    Engine.init(device="cuda:0")
    g = copy.deepcopy(m)
    g.cuda()
    g.training()
    g.getParameters()
    g.flat_parameters().enable_shadow(Engine.compute_dtype())
    g.zeroGradParameters()
    return g


def _round_params(m):
    with torch.no_grad():
        for w in m.parameters()[0]:
            w.copy_(w.to(torch.bfloat16).float())


@pytest.mark.parametrize("mode", ["self", "self_causal", "cross_pad"])
def test_attention_module_matches_host(mode):
    from bigdl.nn.layers.attention import Attention, lower_triangle_bias
    from bigdl.utils.random import RNG
    RNG.setSeed(1)
    B, L, Lk, H, nh = 2, 80, 72, 256, 4
    m = Attention(H, nh, 1.0)
    _round_params(m)
    m.training()
    g = torch.Generator().manual_seed(3)
    x = torch.randn(B, L, H, generator=g).to(torch.bfloat16).float()
    if mode == "cross_pad":
        y = torch.randn(B, Lk, H, generator=g).to(torch.bfloat16).float()
        bias = torch.zeros(B, 1, 1, Lk)
        bias[1, ..., -9:] = -1e9
    else:
        y = x
        bias = lower_triangle_bias(L) if mode == "self_causal" else None
    gm = _gpu(m)
    inp = T(x, y, bias) if bias is not None else T(x, y)
    gy = torch.randn(B, L, H, generator=g)
    m.zeroGradParameters()
    out = m.forward(inp)
    gi = m.backward(inp, gy)
    xd = x.to(dev)
    yd = xd if mode != "cross_pad" else y.to(dev)
    bd = None
    if bias is not None:
        bd = lower_triangle_bias(L, device=dev) if mode == "self_causal" else bias.to(dev)
    dinp = T(xd, yd, bd) if bd is not None else T(xd, yd)
    outd = gm.forward(dinp)
    assert getattr(gm, "_nat", None) is not None, "native path not taken"
    gid = gm.backward(dinp, gy.to(dev))
    torch.cuda.synchronize()
    assert _cos(outd.float().cpu(), out) > 0.999
    assert _cos(gid[1].float().cpu(), gi[1]) > 0.995
    if mode == "cross_pad":
        assert _cos(gid[2].float().cpu(), gi[2]) > 0.995
    for a, b in zip(gm.parameters()[1], m.parameters()[1]):
        assert _cos(a.float().cpu(), b) > 0.995


def test_ffn_module_matches_host():
    from bigdl.nn.layers.attention import FeedForwardNetwork
    from bigdl.utils.random import RNG
    RNG.setSeed(2)
    m = FeedForwardNetwork(256, 1024, 1.0)
    _round_params(m)
    m.training()
    g = torch.Generator().manual_seed(4)
    x = torch.randn(3, 40, 256, generator=g).to(torch.bfloat16).float()
    gy = torch.randn(3, 40, 256, generator=g)
    gm = _gpu(m)
    m.zeroGradParameters()
    out = m.forward(x)
    gi = m.backward(x, gy)
    outd = gm.forward(x.to(dev))
    assert getattr(gm, "_nat", None) is not None
    gid = gm.backward(x.to(dev), gy.to(dev))
    torch.cuda.synchronize()
    assert _cos(outd.float().cpu(), out) > 0.999
    assert _cos(gid.float().cpu(), gi) > 0.995
    for a, b in zip(gm.parameters()[1], m.parameters()[1]):
        assert _cos(a.float().cpu(), b) > 0.995


def test_transformer_lm_step_matches_host():
    """Two-layer LanguageModel Transformer: the whole step's parameter gradients (embedding,
    LayerNorms, attention, FFN) through the native attention path vs the host graph."""
    from bigdl.nn.layers.attention import Transformer
    from bigdl.utils.random import RNG
    RNG.setSeed(5)
    m = Transformer(vocab_size=500, hidden_size=128, num_heads=2, filter_size=512, num_hidden_layers=2,
                    embedding_dropout=1.0, attention_dropout=1.0, ffn_dropout=1.0)
    _round_params(m)
    m.training()
    g = torch.Generator().manual_seed(6)
    ids = torch.randint(1, 500, (2, 48), generator=g).float()
    gm = _gpu(m)
    m.zeroGradParameters()
    out = m.forward(ids)
    gy = torch.randn(out.shape, generator=g)
    m.backward(ids, gy)
    outd = gm.forward(ids.to(dev))
    gm.backward(ids.to(dev), gy.to(dev))
    torch.cuda.synchronize()
    assert _cos(outd.float().cpu(), out) > 0.995
    cs = sorted(_cos(a.float().cpu(), b) for a, b in zip(gm.parameters()[1], m.parameters()[1])
                if float(b.norm()) > 1e-8)
    assert cs[len(cs) // 2] > 0.99 and cs[0] > 0.95, cs[:5]


def test_attention_dropout_statistics():
    """keep = 0.9: the kernel's mask keeps ≈ 90 % of the probabilities and scales them by 1/keep, so
    the dropped-out output has the same expectation (mean over many seeds ≈ the no-dropout O)."""
    from bigdl.ops import native_ops as NO
    B, Hh, D, L = 1, 2, 64, 64
    q = torch.randn(B * L, Hh * D, device=dev).to(torch.bfloat16)
    base, _ = NO.attention_forward(q, q, q, B, Hh, L, L, D, D ** -0.5)
    acc = torch.zeros_like(base, dtype=torch.float32)
    n = 64
    for s in range(n):
        o, _ = NO.attention_forward(q, q, q, B, Hh, L, L, D, D ** -0.5, keep=0.9, seed=1000 + s)
        acc += o.float()
    torch.cuda.synchronize()
    assert _cos(acc / n, base.float()) > 0.99
