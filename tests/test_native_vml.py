"""Vector-math kernels (ops/csrc/vml.hip — the reference's MKL VML role, TensorNumeric.scala:
600-700) against plain torch fp32: unary / binary / gradient forms, dimension reductions, the
Tensor facade and the elementwise layers on the device."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def NO():
    from bigdl.ops import native
    from bigdl.utils.engine import Engine
    Engine.init(device="cuda:0")
    assert native.status()["loaded"] and native.has("vml_unary") and native.has("reduce")
    return native.native_ops


def _x(op, n, dt):
    g = torch.Generator().manual_seed(n)
    x = torch.randn(n, generator=g)
    if op in ("log", "sqrt", "inv", "pow"):
        x = x.abs() + 0.1
    if op == "log1p":
        x = x.abs()
    return x.to(dt).cuda()


REF = {"abs": torch.abs, "exp": torch.exp, "log": torch.log, "log1p": torch.log1p, "sqrt": torch.sqrt,
       "tanh": torch.tanh, "sigmoid": torch.sigmoid, "pow": lambda x: x ** 1.7, "square": lambda x: x * x,
       "inv": torch.reciprocal, "neg": torch.neg, "affine": lambda x: x * 1.7 - 0.3}


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n", [1, 7, 4096, 100003])
@pytest.mark.parametrize("op", sorted(REF))
def test_unary(NO, op, n, dt):
    x = _x(op, n, dt)
    p, q = (1.7, -0.3)
    y = NO.vml_unary(x, op, p, q)
    ref = REF[op](x.float())
    tol = dict(rtol=1e-5, atol=1e-6) if dt == torch.float32 else dict(rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(y.float(), ref if dt == torch.float32 else ref.to(dt).float(), **tol)


BREF = {"add": lambda a, b: a + 0.5 * b, "sub": lambda a, b: a - 0.5 * b, "mul": lambda a, b: a * b,
        "div": lambda a, b: a / b, "tanh_bwd": lambda g, y: g * (1 - y * y),
        "sigmoid_bwd": lambda g, y: g * y * (1 - y), "sqrt_bwd": lambda g, y: 0.5 * g / y,
        "log_bwd": lambda g, x: g / x, "exp_bwd": lambda g, y: g * y, "square_bwd": lambda g, x: 2 * g * x,
        "abs_bwd": lambda g, x: g * torch.sign(x), "pow_bwd": lambda g, x: g * 0.5 * x ** (0.5 - 1)}


@pytest.mark.parametrize("op", sorted(BREF))
def test_binary(NO, op):
    g = torch.Generator().manual_seed(1)
    a = torch.randn(10007, generator=g).cuda()
    b = torch.randn(10007, generator=g).cuda()
    if op in ("div", "sqrt_bwd", "log_bwd", "pow_bwd"):
        b = b.abs() + 0.2
    p = 0.5
    z = NO.vml_binary(a, b, op, p)
    torch.testing.assert_close(z, BREF[op](a, b), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("shape,dim", [((1 << 22,), None), ((37, 5000), 1), ((37, 5000), 0), ((4, 3, 50, 7), 2),
                                       ((100000, 10), 1), ((3, 1000003), None)])
@pytest.mark.parametrize("op", ["sum", "mean", "max", "min"])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_reduce(NO, shape, dim, op, dt):
    x = torch.randn(shape).to(dt).cuda()
    r = NO.reduce(x, op, dim)
    xf = x.double()
    if dim is None:
        ref = {"sum": xf.sum(), "mean": xf.mean(), "max": xf.max(), "min": xf.min()}[op]
    else:
        ref = {"sum": lambda: xf.sum(dim), "mean": lambda: xf.mean(dim), "max": lambda: xf.amax(dim),
               "min": lambda: xf.amin(dim)}[op]()
    n = x.numel() if dim is None else shape[dim]
    tol = 1e-5 * max(1.0, n ** 0.5)
    torch.testing.assert_close(r.double(), ref, rtol=1e-5, atol=tol)


def test_reduce_is_deterministic(NO):
    x = torch.randn(3, 1 << 21, device="cuda")
    a = NO.reduce(x, "sum", 1)
    b = NO.reduce(x, "sum", 1)
    assert torch.equal(a, b)


def test_tensor_facade_uses_vml(NO):
    from bigdl.tensor import Tensor
    from bigdl.ops import native
    native.reset_fallbacks()
    d = torch.rand(1000, 24, device="cuda") + 0.5
    t = Tensor(d.clone())
    t.log().exp().sqrt()
    torch.testing.assert_close(t.data, d.sqrt(), rtol=1e-5, atol=1e-6)
    u = Tensor(d.clone())
    u.cmul(Tensor(d)).add(2.0, Tensor(d)).cdiv(Tensor(d))
    torch.testing.assert_close(u.data, d + 2.0, rtol=1e-5, atol=1e-5)
    assert abs(Tensor(d).sum() - float(d.double().sum())) < 1e-2
    torch.testing.assert_close(Tensor(d).mean(2).data.view(-1), d.mean(1), rtol=1e-5, atol=1e-6)
    assert Tensor(d).max() == float(d.max())
    assert not any(k[0].startswith("vml") for k in native.fallback_counts())


@pytest.mark.parametrize("name", ["Tanh", "Sigmoid", "Exp", "Log", "Sqrt", "Square", "Abs"])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_layers_on_device(NO, name, dt):
    import bigdl.nn as nn
    g = torch.Generator().manual_seed(3)
    x = torch.randn(64, 129, generator=g)
    if name in ("Log", "Sqrt"):
        x = x.abs() + 0.2
    gy = torch.randn(64, 129, generator=g)
    host = getattr(nn, name)()
    yh = host.forward(x.clone())
    gh = host.backward(x.clone(), gy)
    dev = getattr(nn, name)()
    yd = dev.forward(x.to(dt).cuda())
    gd = dev.backward(x.to(dt).cuda(), gy.to(dt).cuda())
    tol = dict(rtol=1e-5, atol=1e-5) if dt == torch.float32 else dict(rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(yd.float().cpu(), yh.float(), **tol)
    torch.testing.assert_close(gd.float().cpu(), gh.float(), **tol)


def test_channels_last_operands(NO):
    x = torch.randn(4, 16, 9, 9, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    y = NO.vml_unary(x, "tanh")
    assert y is not NotImplemented and y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y.float(), torch.tanh(x.float()), rtol=1e-2, atol=1e-2)
    g = torch.randn_like(x)
    z = NO.vml_binary(g, y, "tanh_bwd")
    torch.testing.assert_close(z.float(), (g.float() * (1 - y.float() ** 2)), rtol=2e-2, atol=2e-2)
    # mixed layouts are refused (caller falls back)
    assert NO.vml_binary(g.contiguous(), y, "mul") is NotImplemented
