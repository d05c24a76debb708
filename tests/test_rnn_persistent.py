"""Persistent whole-sequence LSTM kernels (both opt-in; the per-step launches are faster at the PTB
shape, profiles/r3_ptb_persist_ab.txt) — the resident-weight multi-workgroup kernels
(k_lstm_seq_fwd_mp / k_lstm_seq_bwd_mp, BIGDL_RNN_PERSIST=2: U slices in registers, grid barrier per
step, both exchange protocols; =3 the same confined to one XCD; =4 / =5 the barrier-free granule
hand-off, spread over the XCDs / confined to one) and the single-workgroup ones (k_lstm_seq_fwd_p / k_lstm_seq_bwd_p, BIGDL_RNN_PERSIST=1: h / dg_{t+1} in an
LDS double buffer) — one launch per layer-direction, c / dc in registers, against the per-step
launches of the same cell (BIGDL_RNN_PERSIST=0) and the fp32 host LSTM (``Recurrent.scala:283-400``,
``LSTM.scala:124-187``): outputs, input gradients and parameter gradients at the PTB shape
(B 20, H 200, T 20), the B ≤ 16 variant and the H = 256 upper bound."""
import copy
import os

import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"


def _run(rec, x, gy):
    rec.zeroGradParameters()
    y = rec.forward(x)
    gi = rec.backward(x, gy)
    torch.cuda.synchronize()
    return y.float().cpu(), gi.float().cpu(), [p.float().cpu().clone() for p in rec.parameters()[1]]


def _rel(a, b):
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.parametrize("mode", ["2", "2sc0", "3", "4", "5", "6", "7", "1"])
@pytest.mark.parametrize("B,T,IN,H", [(20, 20, 200, 200), (12, 7, 64, 48), (32, 5, 96, 256), (3, 33, 16, 8)])
def test_persistent_lstm_matches_step_path_and_host(B, T, IN, H, mode):
    from bigdl.nn import LSTM, Recurrent
    torch.manual_seed(0)
    cpu = Recurrent().add(LSTM(IN, H))
    gpu = copy.deepcopy(cpu).cuda()
    gpu.training()
    x = torch.randn(B, T, IN)
    gy = torch.randn(B, T, H)
    yc, gic, pc = _run(cpu, x, gy)
    old = os.environ.get("BIGDL_RNN_PERSIST")
    try:
        os.environ["BIGDL_RNN_PERSIST"] = mode[0]
        os.environ["BIGDL_RNN_MP_SYNC"] = "0" if mode.endswith("sc0") else "1"
        yp, gip, pp = _run(gpu, x.to(dev), gy.to(dev))
        from bigdl.ops.native_ops import rnn_sync_errors
        assert rnn_sync_errors(dev) == 0, "a resident-weight tile gave up waiting"
        os.environ["BIGDL_RNN_PERSIST"] = "0"
        ys, gis, ps = _run(gpu, x.to(dev), gy.to(dev))
    finally:
        os.environ.pop("BIGDL_RNN_MP_SYNC", None)
        if old is None:
            os.environ.pop("BIGDL_RNN_PERSIST", None)
        else:
            os.environ["BIGDL_RNN_PERSIST"] = old
    assert _rel(yp, ys) < 1e-2 and _rel(gip, gis) < 2e-2
    for a, b in zip(pp, ps):
        assert _rel(a, b) < 2e-2
    assert _rel(yp, yc) < 3e-2 and _rel(gip, gic) < 5e-2
    for a, b in zip(pp, pc):
        assert _rel(a, b) < 5e-2


def test_mp_lstm_launch_count(monkeypatch):
    """The multi-workgroup path runs a layer-direction as ONE kernel (plus its sync-word memset)."""
    from bigdl.nn import LSTM, Recurrent
    monkeypatch.setenv("BIGDL_RNN_PERSIST", "2")
    torch.manual_seed(2)
    rec = Recurrent().add(LSTM(200, 200)).cuda()
    rec.training()
    x = torch.randn(20, 20, 200, device=dev)
    rec.forward(x)
    torch.cuda.synchronize()
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
        y = rec.forward(x)
        rec.backward(x, torch.randn_like(y))
        torch.cuda.synchronize()
    names = [e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA]
    assert sum("k_lstm_seq_fwd_mp" in n for n in names) == 1, names
    assert sum("k_lstm_seq_bwd_mp" in n for n in names) == 1, names
    assert not any("k_rnn_step" in n for n in names), names


def test_persistent_lstm_inference_final_state():
    """Inference (no saves): the c ping-pong buffer path gives the training forward's output."""
    from bigdl.nn import LSTM, Recurrent
    torch.manual_seed(1)
    rec = Recurrent().add(LSTM(64, 200)).cuda()
    x = torch.randn(20, 20, 64, device=dev)
    y_train = rec.forward(x).float()
    rec.evaluate()
    y_eval = rec.forward(x).float()
    torch.cuda.synchronize()
    torch.testing.assert_close(y_eval, y_train, rtol=0, atol=0)
