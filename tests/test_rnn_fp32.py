"""fp32 recurrence on the GPU (rnn_step.hip k_rnn_step<…, F32>: one launch per step, bf16x3 recurrent
products on the matrix cores) against the fp64 CPU ``Recurrent`` of the same weights
(``DL/nn/Recurrent.scala:283-400``, ``LSTM.scala``, ``GRU.scala``): outputs, input and parameter
gradients within 1e-4 relative."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-12))


@pytest.mark.parametrize("cell", ["lstm", "gru"])
def test_fp32_recurrent_matches_fp64(cell):
    import bigdl.nn as nn
    from bigdl.utils import config
    from bigdl.utils.engine import Engine
    config.set_property("bigdl.compute.dtype", "fp32")
    Engine.init(device="cuda:0")
    Engine.set_compute_dtype("fp32")
    try:
        torch.manual_seed(0)
        B, T, I, H = 4, 6, 24, 64
        mk = (lambda: nn.LSTM(I, H)) if cell == "lstm" else (lambda: nn.GRU(I, H))
        ref = nn.Recurrent().add(mk())
        ref.training()
        gpu = ref.cloneModule().to(device="cuda")
        ref = ref.to(dtype=torch.float64)  # the fp64 CPU reference of the same weights
        x = torch.randn(B, T, I)
        gy = torch.randn(B, T, H)
        y_ref = ref.forward(x.double())
        ref.zeroGradParameters()
        gi_ref = ref.backward(x.double(), gy.double())
        gpu.training()
        y = gpu.forward(x.cuda())
        gpu.zeroGradParameters()
        gi = gpu.backward(x.cuda(), gy.cuda())
        assert y.dtype == torch.float32
        assert _rel(y, y_ref) < 1e-4
        assert _rel(gi, gi_ref) < 1e-4
        for a, b in zip(gpu.parameters()[1], ref.parameters()[1]):
            assert _rel(a, b) < 1e-4
    finally:
        Engine.set_compute_dtype("bf16")
        config.set_property("bigdl.compute.dtype", "auto")


def test_fp32_recurrent_uses_the_fused_step(monkeypatch):
    """The fp32 device path is the native one-launch-per-step loop, not the per-step torch.mm."""
    import bigdl.nn as nn
    from bigdl.utils import config
    from bigdl.utils.engine import Engine
    from bigdl.ops import native_ops as NO
    config.set_property("bigdl.compute.dtype", "fp32")
    Engine.init(device="cuda:0")
    Engine.set_compute_dtype("fp32")
    try:
        calls = []
        f, b = NO.lstm_seq_forward32, NO.lstm_seq_backward32
        monkeypatch.setattr(NO, "lstm_seq_forward32", lambda *a: (calls.append("f"), f(*a))[1])
        monkeypatch.setattr(NO, "lstm_seq_backward32", lambda *a: (calls.append("b"), b(*a))[1])
        m = nn.Recurrent().add(nn.LSTM(16, 32)).to(device="cuda")
        m.training()
        x = torch.randn(2, 5, 16, device="cuda")
        m.forward(x)
        m.backward(x, torch.randn(2, 5, 32, device="cuda"))
        assert calls == ["f", "b"]
    finally:
        Engine.set_compute_dtype("bf16")
        config.set_property("bigdl.compute.dtype", "auto")
