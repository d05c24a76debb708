"""TF backward / training-graph ops (``DL/nn/tf/NNOps.scala``, ``MathOps.scala``, ``ArrayOps.scala``,
``ParsingOps.scala``; loaders ``DL/utils/tf/loaders/*Grad*.scala``) against independent torch
oracles (plain autograd of the corresponding torch forward), and loaded from a GraphDef."""
import pytest
import torch
import torch.nn.functional as F

from bigdl.utils.table import Table
import bigdl.nn.tf as T
from bigdl.nn import ops as O


def _T(*xs):
    return Table(*xs)


def _grad(fn, x, g):
    x = x.clone().requires_grad_(True)
    (gx,) = torch.autograd.grad(fn(x), x, g)
    return gx


def test_elementwise_grads_match_autograd():
    torch.manual_seed(0)
    x = torch.randn(5, 7)
    g = torch.randn(5, 7)
    torch.testing.assert_close(T.ReluGrad().forward(_T(g, x)), _grad(torch.relu, x, g))
    torch.testing.assert_close(T.Relu6Grad().forward(_T(g, x * 4)), _grad(lambda v: F.relu6(v), x * 4, g))
    y = F.elu(x)
    torch.testing.assert_close(T.EluGrad().forward(_T(g, y)), _grad(F.elu, x, g))
    torch.testing.assert_close(T.SoftplusGrad().forward(_T(g, x)), _grad(F.softplus, x, g))
    torch.testing.assert_close(T.SoftsignGrad().forward(_T(g, x)), _grad(F.softsign, x, g))
    torch.testing.assert_close(T.TanhGrad().forward(_T(torch.tanh(x), g)), _grad(torch.tanh, x, g))
    torch.testing.assert_close(T.SigmoidGrad().forward(_T(torch.sigmoid(x), g)), _grad(torch.sigmoid, x, g))
    p = x.abs() + 0.5
    torch.testing.assert_close(T.SqrtGrad().forward(_T(p.sqrt(), g)), _grad(torch.sqrt, p, g))
    torch.testing.assert_close(T.RsqrtGrad().forward(_T(p.rsqrt(), g)), _grad(torch.rsqrt, p, g))
    torch.testing.assert_close(T.InvGrad().forward(_T(1 / p, g)), _grad(torch.reciprocal, p, g))
    torch.testing.assert_close(T.Mod().forward(_T(torch.tensor([7., -7.]), torch.tensor([3., 3.]))),
                               torch.tensor([1., -1.]))  # truncating remainder (C fmod)


def test_bias_add_grad_and_broadcast_args():
    g = torch.randn(2, 3, 4, 5)
    torch.testing.assert_close(T.BiasAddGrad("NHWC").forward(g), g.sum((0, 1, 2)))
    torch.testing.assert_close(T.BiasAddGrad("NCHW").forward(g), g.sum((0, 2, 3)))
    r = T.BroadcastGradientArgs().forward(_T(torch.tensor([2, 3, 1]), torch.tensor([3, 4])))
    assert r[1].tolist() == [2] and r[2].tolist() == [0]
    r = T.BroadcastGradientArgs().forward(_T(torch.tensor([1, 3]), torch.tensor([5, 1, 3])))
    assert r[1].tolist() == [0, 1] and r[2].tolist() == [1]


@pytest.mark.parametrize("padding,stride", [("SAME", 2), ("VALID", 1), ("SAME", 1)])
def test_conv2d_backprop_input_filter(padding, stride):
    torch.manual_seed(1)
    x = torch.randn(2, 9, 8, 3)            # NHWC
    f = torch.randn(3, 3, 3, 4)            # HWIO
    strides = [1, stride, stride, 1]

    def fwd(xx, ff):  # independent TF-SAME oracle: explicit asymmetric pad + torch conv
        xc = xx.permute(0, 3, 1, 2)
        ph = T._tf_pads(9, 3, stride, padding)
        pw = T._tf_pads(8, 3, stride, padding)
        xc = F.pad(xc, (pw[0], pw[1], ph[0], ph[1]))
        return F.conv2d(xc, ff.permute(3, 2, 0, 1), stride=stride).permute(0, 2, 3, 1)
    y = fwd(x, f)
    dy = torch.randn_like(y)
    gx = T.Conv2DTranspose(strides, padding, "NHWC").forward(_T(torch.tensor(list(x.shape)), f, dy))
    torch.testing.assert_close(gx, _grad(lambda v: fwd(v, f), x, dy), rtol=1e-4, atol=1e-4)
    gf = T.Conv2DBackFilter(strides, padding, "NHWC").forward(_T(x, torch.tensor(list(f.shape)), dy))
    torch.testing.assert_close(gf, _grad(lambda w: fwd(x, w), f, dy), rtol=1e-4, atol=1e-4)


def test_conv3d_and_grads():
    torch.manual_seed(2)
    x = torch.randn(1, 5, 6, 7, 2)     # NDHWC
    f = torch.randn(2, 3, 3, 2, 3)     # DHWIO
    op = T.Conv3D([1, 1, 1, 1, 1], "VALID")
    y = op.forward(_T(x, f))
    ref = F.conv3d(x.permute(0, 4, 1, 2, 3), f.permute(4, 3, 0, 1, 2)).permute(0, 2, 3, 4, 1)
    torch.testing.assert_close(y, ref, rtol=1e-4, atol=1e-4)
    dy = torch.randn_like(y)
    gx = T.Conv3DBackpropInputV2([1, 1, 1, 1, 1], "VALID").forward(_T(torch.tensor(list(x.shape)), f, dy))
    gx1 = T.Conv3DBackpropInput([1, 1, 1, 1, 1], "VALID").forward(_T(x, f, dy))
    gf = T.Conv3DBackpropFilterV2([1, 1, 1, 1, 1], "VALID").forward(_T(x, torch.tensor(list(f.shape)), dy))
    gf1 = T.Conv3DBackpropFilter([1, 1, 1, 1, 1], "VALID").forward(_T(x, f, dy))
    fx = lambda v: F.conv3d(v.permute(0, 4, 1, 2, 3), f.permute(4, 3, 0, 1, 2)).permute(0, 2, 3, 4, 1)  # noqa
    fw = lambda w: F.conv3d(x.permute(0, 4, 1, 2, 3), w.permute(4, 3, 0, 1, 2)).permute(0, 2, 3, 4, 1)  # noqa
    for a, b in ((gx, _grad(fx, x, dy)), (gx1, _grad(fx, x, dy)), (gf, _grad(fw, f, dy)), (gf1, _grad(fw, f, dy))):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-4)


def test_pool_lrn_grads():
    torch.manual_seed(3)
    x = torch.randn(2, 6, 6, 3)
    g = torch.randn(2, 3, 3, 3)
    mp = lambda v: F.max_pool2d(v.permute(0, 3, 1, 2), 2, 2).permute(0, 2, 3, 1)  # noqa
    got = T.MaxPoolGrad([1, 2, 2, 1], [1, 2, 2, 1], "VALID").forward(_T(x, mp(x), g))
    torch.testing.assert_close(got, _grad(mp, x, g))
    ap = lambda v: F.avg_pool2d(v.permute(0, 3, 1, 2), 2, 2).permute(0, 2, 3, 1)  # noqa
    got = T.AvgPoolGrad([1, 2, 2, 1], [1, 2, 2, 1], "VALID").forward(_T(torch.tensor([2, 6, 6, 3]), g))
    torch.testing.assert_close(got, _grad(ap, x, g))
    lrn = T.LRN(2, 1.0, 0.5, 0.75)
    gl = torch.randn_like(x)
    got = T.LRNGrad(2, 1.0, 0.5, 0.75).forward(_T(gl, x, lrn.forward(x)))

    def lrn_ref(v):  # TF LRN: x / (bias + alpha·Σ_{|d-c|≤r} x_d²)^beta over the last dim
        sq = v ** 2
        C = v.shape[-1]
        s = torch.stack([sq[..., max(0, c - 2):c + 3].sum(-1) for c in range(C)], -1)
        return v / (1.0 + 0.5 * s) ** 0.75
    torch.testing.assert_close(got, _grad(lrn_ref, x, gl), rtol=1e-4, atol=1e-5)


def test_fused_batch_norm_grad_matches_autograd():
    torch.manual_seed(4)
    x = torch.randn(4, 3, 3, 5)
    sc = torch.rand(5) + 0.5
    off = torch.randn(5)
    mean, var = x.mean((0, 1, 2)), x.var((0, 1, 2), unbiased=False)
    dy = torch.randn_like(x)
    out = T.FusedBatchNormGrad(1e-3, "NHWC", True).forward(_T(dy, x, sc, mean, var))

    def bn(v, s, o):
        return F.batch_norm(v.permute(0, 3, 1, 2), None, None, s, o, training=True, eps=1e-3).permute(0, 2, 3, 1)
    xr, sr, orr = x.clone().requires_grad_(), sc.clone().requires_grad_(), off.clone().requires_grad_()
    gx, gs, go = torch.autograd.grad(bn(xr, sr, orr), (xr, sr, orr), dy)
    torch.testing.assert_close(out[1], gx, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(out[2], gs, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(out[3], go, rtol=1e-4, atol=1e-4)


def test_dilation2d_grads_and_resize_grad():
    torch.manual_seed(5)
    x = torch.randn(1, 6, 6, 2)
    f = torch.randn(2, 2, 2)
    d = O.Dilation2D([1, 1, 1, 1], [1, 1, 1, 1], "VALID")
    y = d.forward(_T(x, f))
    g = torch.randn_like(y)
    gi = T.Dilation2DBackpropInput([1, 1, 1, 1], [1, 1, 1, 1], "VALID").forward(_T(x, f, g))
    gf = T.Dilation2DBackpropFilter([1, 1, 1, 1], [1, 1, 1, 1], "VALID").forward(_T(x, f, g))

    def dil(v, w):  # direct max over the 2×2 window + filter
        out = torch.full((1, 5, 5, 2), -1e30)
        for a in range(2):
            for b in range(2):
                out = torch.maximum(out, v[:, a:a + 5, b:b + 5, :] + w[a, b])
        return out
    torch.testing.assert_close(gi, _grad(lambda v: dil(v, f), x, g))
    torch.testing.assert_close(gf, _grad(lambda w: dil(x, w), f, g))
    img = torch.randn(1, 4, 4, 2)
    gr = torch.randn(1, 8, 8, 2)
    from bigdl.ops.reference import resize_bilinear  # the reference's TF-style sampling
    up = lambda v: resize_bilinear(v.permute(0, 3, 1, 2), 8, 8, False).permute(0, 2, 3, 1)  # noqa
    torch.testing.assert_close(T.ResizeBilinearGrad(False).forward(_T(gr, img)), _grad(up, img, gr))


def test_parse_single_example():
    from bigdl.utils.tf.proto import example_classes
    cl = example_classes()
    ex = cl["tensorflow.Example"]()
    ex.features.feature["a"].float_list.value.extend([1.0, 2.0, 3.0])
    ex.features.feature["s"].int64_list.value.extend([7, 8])
    op = T.ParseSingleExample(["a", "b"], [torch.float32, torch.int64], [[3], [1]], ["s"], [torch.int64])
    out = op.forward(_T(ex.SerializeToString(), torch.zeros(0), torch.tensor([5])))
    # sparse (indices, values, shape) then dense
    assert out[1].tolist() == [[0], [1]] and out[2].tolist() == [7, 8] and out[3].tolist() == [2]
    assert out[4].tolist() == [1.0, 2.0, 3.0] and out[5].tolist() == [5]  # b missing → its default


def test_loader_builds_grad_ops_from_graphdef(tmp_path):
    """A GraphDef using ReluGrad / BiasAddGrad / Conv2DBackpropInput loads and runs."""
    from bigdl.utils.tf.proto import graph_classes
    from bigdl.utils.tf.loader import TensorflowLoader
    classes, _ = graph_classes()
    gd = classes["tensorflow.GraphDef"]()

    def node(name, op, inputs=(), **attrs):
        n = gd.node.add()
        n.name, n.op = name, op
        n.input.extend(inputs)
        for k, v in attrs.items():
            if isinstance(v, str):
                n.attr[k].s = v.encode()
            elif isinstance(v, list):
                n.attr[k].list.i.extend(v)
        return n
    node("g", "Placeholder")
    node("x", "Placeholder")
    node("rg", "ReluGrad", ["g", "x"])
    node("bg", "BiasAddGrad", ["rg"], data_format="NHWC")
    p = tmp_path / "g.pb"
    p.write_bytes(gd.SerializeToString())
    model = TensorflowLoader.load(str(p), ["g", "x"], ["bg"])
    g, x = torch.randn(2, 3, 3, 4), torch.randn(2, 3, 3, 4)
    out = model.forward(Table(g, x))
    torch.testing.assert_close(out, (g * (x > 0)).sum((0, 1, 2)))
