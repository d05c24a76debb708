"""Two stacked Recurrent(LSTM) layers on the layer wavefront (rnn_step.hip bigdl_lstm2_seq_*, fusion
``lstmstack``): forward output, hidden states, every parameter gradient and the embedding-side
input gradient match the layer-by-layer fused-step execution of the same weights (PTBModel.lstm
topology, ``DL/example/languagemodel/PTBModel.scala``)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _models(V, H, B, T):
    from bigdl.utils import config
    from bigdl.utils.engine import Engine
    from bigdl.models.rnn import PTBModel
    config.set_property("bigdl.compute.dtype", "bf16")
    Engine.init(device="cuda:0")
    torch.manual_seed(0)
    a = PTBModel.lstm(V, H, V, 2)
    b = PTBModel.lstm(V, H, V, 2)
    pa, pb = a.parameters()[0], b.parameters()[0]
    for x, y in zip(pa, pb):
        y.data.copy_(x.data)
    return a.to(device="cuda"), b.to(device="cuda")


@pytest.mark.parametrize("T", [1, 7, 20])
def test_stacked_lstm_matches_layer_by_layer(T):
    from bigdl.nn.fusion import _fuse_lstm_stacks
    from bigdl.nn.layers.recurrent import Recurrent
    from bigdl import ops
    V, H, B = 64, 200, 20
    a, b = _models(V, H, B, T)
    a.training()
    b.training()
    _fuse_lstm_stacks(a)
    recs = [m for m in a.flattened_modules() if type(m) is Recurrent]
    assert recs[0]._stack_next is recs[1]
    ops.reset_fallbacks()
    x = (torch.randint(0, V, (B, T)) + 1).float().cuda()
    ya = a.forward(x)
    assert recs[1]._rec is not None and recs[1]._rec[0] == "lstm2"  # the wavefront path ran
    yb = b.forward(x)
    torch.testing.assert_close(ya.float(), yb.float(), rtol=2e-2, atol=2e-2)
    gy = (torch.randn(B, T, V, device="cuda") * 0.1).to(ya.dtype)
    a.zeroGradParameters()
    b.zeroGradParameters()
    a.backward(x, gy)
    b.backward(x, gy)
    ga, gb = a.parameters()[1], b.parameters()[1]
    for i, (u, v) in enumerate(zip(ga, gb)):
        scale = float(v.float().abs().max()) + 1e-6
        torch.testing.assert_close(u.float() / scale, v.float() / scale, rtol=0, atol=3e-2, msg=f"grad {i}")
    rb = [m for m in b.flattened_modules() if type(m) is Recurrent]
    for ra_, rb_ in zip(recs, rb):
        for u, v in zip(ra_.getGradHiddenState(), rb_.getGradHiddenState()):
            scale = float(v.float().abs().max()) + 1e-6
            torch.testing.assert_close(u.float() / scale, v.float() / scale, rtol=0, atol=3e-2)
    assert ops.fallback_counts() == {}


def test_stacked_lstm_inference():
    from bigdl.nn.fusion import _fuse_lstm_stacks
    V, H, B, T = 64, 200, 4, 9
    a, b = _models(V, H, B, T)
    a.evaluate()
    b.evaluate()
    _fuse_lstm_stacks(a)
    x = (torch.randint(0, V, (B, T)) + 1).float().cuda()
    with torch.no_grad():
        torch.testing.assert_close(a.forward(x).float(), b.forward(x).float(), rtol=2e-2, atol=2e-2)
