"""TF checkpoint (V2 tensor bundle) I/O without TensorFlow, variables in the GraphDef loader, and
the training Session (reference DL/utils/tf/Session.scala, TensorflowLoader.scala:88,142-172)."""
import numpy as np
import torch

from bigdl.utils.tf import TensorflowLoader
from bigdl.utils.tf.checkpoint import read_checkpoint, write_checkpoint, read_index, crc32c


def _mlp_graphdef(path):
    """x[?,4] → MatMul(Identity(w1)) → BiasAdd(b1) → Relu → MatMul(w2/read) → BiasAdd(b2) = out,
    with the weights as VariableV2 nodes (TF 1.x style) — values come from a checkpoint."""
    from bigdl.utils.tf.proto import graph_classes
    classes, _ = graph_classes()
    gd = classes["tensorflow.GraphDef"]()

    def node(name, op, inputs=()):
        n = gd.node.add()
        n.name, n.op = name, op
        n.input.extend(inputs)
        return n
    node("x", "Placeholder")
    for v in ("w1", "b1", "w2", "b2"):
        node(v, "VariableV2")
        node(v + "/read", "Identity", [v])
    node("mm1", "MatMul", ["x", "w1/read"])
    node("h1", "BiasAdd", ["mm1", "b1/read"])
    node("r1", "Relu", ["h1"])
    node("mm2", "MatMul", ["r1", "w2/read"])
    node("out", "BiasAdd", ["mm2", "b2/read"])
    with open(path, "wb") as f:
        f.write(gd.SerializeToString())


def _weights(seed=0):
    g = np.random.default_rng(seed)
    return {"w1": g.normal(0, 0.5, (4, 8)).astype(np.float32), "b1": g.normal(0, 0.1, 8).astype(np.float32),
            "w2": g.normal(0, 0.5, (8, 2)).astype(np.float32), "b2": g.normal(0, 0.1, 2).astype(np.float32)}


def _ref(x, w):
    return np.maximum(x @ w["w1"] + w["b1"], 0) @ w["w2"] + w["b2"]


def test_crc32c_known_value():
    assert crc32c(b"123456789") == 0xE3069283  # the CRC-32C check value


def test_checkpoint_roundtrip(tmp_path):
    w = _weights()
    w["step"] = np.array(7, dtype=np.int64)
    w["half"] = np.arange(6, dtype=np.float16).reshape(2, 3)
    prefix = str(tmp_path / "model.ckpt-7")
    write_checkpoint(prefix, w)
    hdr, entries = read_index(prefix)
    assert hdr["num_shards"] == 1 and set(entries) == set(w)
    back = read_checkpoint(prefix)
    for k, v in w.items():
        assert back[k].dtype == v.dtype and back[k].shape == v.shape
        np.testing.assert_array_equal(back[k], v)


def test_loader_reads_variables_from_checkpoint(tmp_path):
    gp, prefix = str(tmp_path / "mlp.pb"), str(tmp_path / "ck")
    _mlp_graphdef(gp)
    w = _weights()
    write_checkpoint(prefix, w)
    model = TensorflowLoader.load(gp, ["x"], ["out"], bin_file=prefix)
    x = np.random.default_rng(1).normal(0, 1, (5, 4)).astype(np.float32)
    y = model.forward(torch.from_numpy(x))
    np.testing.assert_allclose(y.numpy(), _ref(x, w), rtol=1e-5, atol=1e-5)
    # the variables became trainable parameters (two Linear layers: weight + bias each)
    assert len(model.parameters()[0]) == 4
    # npz variable files work the same way
    np.savez(str(tmp_path / "v.npz"), **w)
    m2 = TensorflowLoader.load(gp, ["x"], ["out"], bin_file=str(tmp_path / "v.npz"))
    np.testing.assert_allclose(m2.forward(torch.from_numpy(x)).numpy(), y.numpy(), rtol=1e-6, atol=1e-6)


def test_session_train_predict_save(tmp_path):
    from bigdl.dataset import MiniBatch
    from bigdl.nn import MSECriterion
    from bigdl.optim import SGD, MaxIteration
    gp, prefix = str(tmp_path / "mlp.pb"), str(tmp_path / "ck")
    _mlp_graphdef(gp)
    w0 = _weights()
    write_checkpoint(prefix, w0)
    sess = TensorflowLoader.checkpoints(gp, prefix)
    g = np.random.default_rng(2)
    x = g.normal(0, 1, (64, 4)).astype(np.float32)
    target = (x[:, :2] * 1.5 - 0.5).astype(np.float32)
    data = [MiniBatch(torch.from_numpy(x[i:i + 16]), torch.from_numpy(target[i:i + 16])) for i in range(0, 64, 16)]
    before = float(((sess.predict(["out"], x).numpy() - target) ** 2).mean())
    sess.train(["out"], data, SGD(learningrate=0.05), MSECriterion(), MaxIteration(200), batch_size=16)
    after = float(((sess.predict(["out"], x).numpy() - target) ** 2).mean())
    assert after < 0.5 * before, (before, after)
    # the trained weights went back into the session's variables and out as a TF checkpoint
    out = str(tmp_path / "trained")
    sess.saveParameters(out)
    w1 = read_checkpoint(out)
    assert not np.allclose(w1["w1"], w0["w1"])
    np.testing.assert_allclose(_ref(x, w1), sess.predict(["out"], x).numpy(), rtol=1e-4, atol=1e-4)
