"""Native layer norm (ops/csrc/layernorm.hip) vs the fp32 torch reference: forward, input and
parameter gradients, fp32 and bf16 I/O, ragged widths; and the LayerNormalization layer on it."""
import pytest
import torch

pytestmark = pytest.mark.gpu

dev = "cuda"


def _ref(x, w, b, eps):
    x = x.double()
    mu = x.mean(-1, keepdim=True)
    var = ((x - mu) ** 2).mean(-1, keepdim=True)
    return (x - mu) * torch.rsqrt(var + eps) * w.double() + b.double()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(4, 7), (3, 50, 512), (2, 768), (1000, 1024), (5, 4096), (33, 100)])
def test_layer_norm_fwd_bwd(dtype, shape):
    from bigdl.ops import native, native_status
    assert native_status()["loaded"]
    torch.manual_seed(0)
    H = shape[-1]
    x = (torch.randn(shape, device=dev) * 3 + 1).to(dtype).requires_grad_()
    w = (torch.rand(H, device=dev) + 0.5).requires_grad_()
    b = torch.randn(H, device=dev).requires_grad_()
    y = native.layer_norm(x, w, b, 1e-6)
    assert y is not NotImplemented and y.dtype == dtype
    gy = torch.randn(shape, device=dev).to(dtype)
    y.backward(gy)

    xr = x.detach().float().requires_grad_()
    wr, br = w.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
    yr = _ref(xr, wr, br, 1e-6)
    yr.backward(gy.double())
    tol = dict(rtol=2e-2, atol=2e-2) if dtype == torch.bfloat16 else dict(rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(y.float(), yr.float(), **tol)
    torch.testing.assert_close(x.grad.float(), xr.grad.float(), **tol)
    rows = x.numel() // H
    ptol = dict(rtol=2e-2, atol=2e-2 * rows ** 0.5) if dtype == torch.bfloat16 else dict(rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(w.grad, wr.grad.float(), **ptol)
    torch.testing.assert_close(b.grad, br.grad.float(), **ptol)


def test_layer_norm_no_affine_and_too_wide():
    from bigdl.ops import native
    x = torch.randn(16, 300, device=dev)
    y = native.layer_norm(x, None, None, 1e-5)
    torch.testing.assert_close(y, torch.nn.functional.layer_norm(x, (300,), eps=1e-5), rtol=1e-4, atol=1e-4)
    assert native.layer_norm(torch.randn(2, 8192, device=dev)) is NotImplemented


def test_layer_normalization_layer_native(monkeypatch):
    from bigdl import nn
    from bigdl.ops import native, native_ops
    calls = []
    fb = []
    monkeypatch.setattr(native, "note_fallback", lambda *a, **k: fb.append(a))
    real = native_ops.layer_norm
    monkeypatch.setattr(native_ops, "layer_norm", lambda *a, **k: calls.append(1) or real(*a, **k))
    m = nn.LayerNormalization(256).cuda()
    x = torch.randn(4, 10, 256, device=dev)
    y = m.forward(x)
    gx = m.backward(x, torch.ones_like(y))
    assert calls and not fb
    ref = _ref(x, torch.ones(256, device=dev), torch.zeros(256, device=dev), 1e-6).float()
    torch.testing.assert_close(y, ref, rtol=1e-4, atol=1e-4)
    assert gx.shape == x.shape and torch.isfinite(gx).all()
    gw = m.parameters()[1][0]
    assert gw.abs().sum() > 0


def test_transformer_lm_step_bf16_on_gpu():
    """Transformer LM on the GPU under the bf16 config: native LayerNorm in the graph, fp32 master
    gradients; output within bf16 tolerance of the fp32 CPU model."""
    from bigdl.utils import config
    from bigdl.nn import Transformer
    old = config.get_property("bigdl.compute.dtype")
    config.set_property("bigdl.compute.dtype", "bf16")
    try:
        torch.manual_seed(0)
        m = Transformer(50, 64, 4, 128, 2, 1.0, 1.0, 1.0, transformer_type="LanguageModel")
        x = torch.randint(1, 50, (2, 12)).float()
        ref = m.forward(x).detach().clone()
        m.cuda()
        y = m.forward(x.cuda())
        assert y.is_cuda
        torch.testing.assert_close(y.float().cpu(), ref, rtol=5e-2, atol=5e-2)
        m.backward(x.cuda(), torch.ones_like(y))
        w, g = m.parameters()
        assert all(t.dtype == torch.float32 for t in g) and all(torch.isfinite(t).all() for t in g)
        assert sum(float(t.abs().sum()) for t in g) > 0
    finally:
        config.set_property("bigdl.compute.dtype", old)
