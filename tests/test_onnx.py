"""ONNX loader (``pyspark/bigdl/contrib/onnx``): models are built with the bundled ``helper`` (the
``onnx`` package is not installed), serialised to ``.onnx`` bytes, loaded back and compared
against plain torch functional references of the same graph (parity unpinned vs onnxruntime,
which is not available)."""
import numpy as np
import torch
import torch.nn.functional as F

from bigdl.contrib.onnx import helper, load, load_model_proto, onnx_classes
from bigdl.nn.onnx import Gemm, Reshape
from bigdl.utils.table import Table


def _save_load(model, tmp_path):
    p = tmp_path / "m.onnx"
    p.write_bytes(model.SerializeToString())
    return load(str(p))


def test_conv_bn_relu_pool_gemm_softmax(tmp_path):
    rng = np.random.RandomState(0)
    W = rng.randn(4, 3, 3, 3).astype(np.float32) * 0.3
    B = rng.randn(4).astype(np.float32)
    sc, bi = rng.rand(4).astype(np.float32) + 0.5, rng.randn(4).astype(np.float32)
    mu, var = rng.randn(4).astype(np.float32), rng.rand(4).astype(np.float32) + 0.5
    FW = rng.randn(5, 4 * 4 * 4).astype(np.float32) * 0.1
    FB = rng.randn(5).astype(np.float32)
    inits = [helper.make_tensor(n, v) for n, v in
             [("W", W), ("B", B), ("sc", sc), ("bi", bi), ("mu", mu), ("var", var), ("FW", FW), ("FB", FB),
              ("shape", np.array([0, -1], dtype=np.int64))]]
    nodes = [
        helper.make_node("Conv", ["x", "W", "B"], ["c"], kernel_shape=[3, 3], pads=[1, 1, 1, 1]),
        helper.make_node("BatchNormalization", ["c", "sc", "bi", "mu", "var"], ["b"], epsilon=1e-5),
        helper.make_node("Relu", ["b"], ["r"]),
        helper.make_node("MaxPool", ["r"], ["p"], kernel_shape=[2, 2], strides=[2, 2]),
        helper.make_node("Reshape", ["p", "shape"], ["f"]),
        helper.make_node("Gemm", ["f", "FW", "FB"], ["g"], transB=1),
        helper.make_node("Softmax", ["g"], ["y"], axis=1),
    ]
    g = helper.make_graph(nodes, "net", [helper.make_value_info("x", ["N", 3, 8, 8])],
                          [helper.make_value_info("y", ["N", 5])], inits)
    m = _save_load(helper.make_model(g), tmp_path)
    m.evaluate()
    x = torch.randn(2, 3, 8, 8)
    t = F.conv2d(x, torch.from_numpy(W), torch.from_numpy(B), padding=1)
    t = (t - torch.from_numpy(mu).view(1, -1, 1, 1)) / torch.sqrt(torch.from_numpy(var).view(1, -1, 1, 1) + 1e-5)
    t = t * torch.from_numpy(sc).view(1, -1, 1, 1) + torch.from_numpy(bi).view(1, -1, 1, 1)
    t = F.max_pool2d(torch.relu(t), 2).reshape(2, -1)
    ref = torch.softmax(t @ torch.from_numpy(FW).t() + torch.from_numpy(FB), 1)
    torch.testing.assert_close(m.forward(x), ref, atol=1e-5, rtol=1e-4)


def test_branches_concat_sum_and_elementwise(tmp_path):
    nodes = [
        helper.make_node("Relu", ["x"], ["a"]),
        helper.make_node("Sigmoid", ["x"], ["b"]),
        helper.make_node("Concat", ["a", "b"], ["c"], axis=1),
        helper.make_node("Sum", ["c", "c"], ["s"]),
        helper.make_node("Mul", ["s", "k"], ["m"]),
        helper.make_node("GlobalAveragePool", ["m"], ["gp"]),
        helper.make_node("Flatten", ["gp"], ["y"], axis=1),
    ]
    g = helper.make_graph(nodes, "br", [helper.make_value_info("x", [2, 3, 4, 4])], [helper.make_value_info("y", [2, 6])],
                          [helper.make_tensor("k", np.array(0.5, dtype=np.float32))])
    m = load_model_proto(helper.make_model(g))
    x = torch.randn(2, 3, 4, 4)
    c = torch.cat([torch.relu(x), torch.sigmoid(x)], 1)
    torch.testing.assert_close(m.forward(x), (2 * c * 0.5).mean((2, 3)))


def test_tensor_roundtrip_dtypes():
    for arr in (np.arange(6, dtype=np.float32).reshape(2, 3), np.array([1, -2], dtype=np.int64),
                np.array([True, False]), np.arange(4, dtype=np.float64)):
        t = helper.make_tensor("t", arr)
        back = onnx_classes()["onnx.TensorProto"].FromString(t.SerializeToString())
        from bigdl.contrib.onnx import to_array
        np.testing.assert_array_equal(to_array(back), arr)


def test_onnx_layers():
    a, b, c = torch.randn(3, 4), torch.randn(5, 4), torch.randn(3, 5)
    y = Gemm(2.0, 0.5, False, True).forward(Table(a, b, c))
    torch.testing.assert_close(y, 2.0 * a @ b.t() + 0.5 * c)
    assert Reshape([0, -1]).forward(torch.randn(2, 3, 4)).shape == (2, 12)
