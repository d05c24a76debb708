"""Recurrent family vs plain-torch fp32 oracles (reference specs: TS/nn/RecurrentSpec.scala,
LSTMSpec, GRUSpec, BiRecurrentSpec, TimeDistributedSpec, RecurrentDecoderSpec)."""
import pytest
import torch

from bigdl.nn import (BiRecurrent, ConvLSTMPeephole, GRU, Linear, LSTM, LSTMPeephole, MultiRNNCell, Recurrent,
                      RecurrentDecoder, RnnCell, Tanh, TimeDistributed, CAddTable)
from bigdl.utils.table import T


def _lstm_oracle(x, wi, bi, wh, h0=None, c0=None):
    B, Tn, _ = x.shape
    H = wh.shape[1]
    h = torch.zeros(B, H) if h0 is None else h0
    c = torch.zeros(B, H) if c0 is None else c0
    outs = []
    for t in range(Tn):
        g = x[:, t] @ wi.t() + bi + h @ wh.t()
        i, gg, f, o = g[:, :H].sigmoid(), g[:, H:2 * H].tanh(), g[:, 2 * H:3 * H].sigmoid(), g[:, 3 * H:].sigmoid()
        c = i * gg + f * c
        h = o * c.tanh()
        outs.append(h)
    return torch.stack(outs, 1)


@pytest.mark.parametrize("fast", [True, False])
def test_lstm_matches_oracle(fast):
    torch.manual_seed(0)
    rec = Recurrent().add(LSTM(5, 6))
    rec.fast_lstm = fast
    x = torch.randn(3, 4, 5)
    y = rec.forward(x)
    ws = [p.detach().clone().requires_grad_(True) for p in rec.parameters()[0]]
    xr = x.clone().requires_grad_(True)
    yr = _lstm_oracle(xr, *ws)
    torch.testing.assert_close(y, yr, rtol=1e-5, atol=1e-5)
    gy = torch.randn_like(y)
    rec.zeroGradParameters()
    gi = rec.backward(x, gy)
    yr.backward(gy)
    torch.testing.assert_close(gi, xr.grad, rtol=1e-4, atol=1e-5)
    for g, w in zip(rec.parameters()[1], ws):
        torch.testing.assert_close(g, w.grad, rtol=1e-4, atol=1e-5)


def test_lstm_hidden_state_roundtrip():
    torch.manual_seed(1)
    rec = Recurrent().add(LSTM(3, 4))
    x = torch.randn(2, 6, 3)
    full = rec.forward(x).clone()
    rec.forward(x[:, :3])
    hs = rec.getHiddenState()
    rec.setHiddenState(T(hs[1].clone(), hs[2].clone()))
    second = rec.forward(x[:, 3:])
    torch.testing.assert_close(second, full[:, 3:], rtol=1e-5, atol=1e-6)


def test_gru_matches_oracle():
    torch.manual_seed(2)
    cell = GRU(4, 5)
    rec = Recurrent().add(cell)
    x = torch.randn(2, 3, 4)
    y = rec.forward(x)
    wi, bi, wrz, wh = [p.detach().clone().requires_grad_(True) for p in rec.parameters()[0]]
    xr = x.clone().requires_grad_(True)
    H = 5
    h = torch.zeros(2, H)
    outs = []
    for t in range(3):
        xp = xr[:, t] @ wi.t() + bi
        rz = xp[:, :2 * H] + h @ wrz.t()
        r, z = rz[:, :H].sigmoid(), rz[:, H:].sigmoid()
        hh = (xp[:, 2 * H:] + (h * r) @ wh.t()).tanh()
        h = (1 - z) * hh + z * h
        outs.append(h)
    yr = torch.stack(outs, 1)
    torch.testing.assert_close(y, yr, rtol=1e-5, atol=1e-6)
    gy = torch.randn_like(y)
    gi = rec.backward(x, gy)
    yr.backward(gy)
    torch.testing.assert_close(gi, xr.grad, rtol=1e-4, atol=1e-5)
    for g, w in zip(rec.parameters()[1], [wi, bi, wrz, wh]):
        torch.testing.assert_close(g, w.grad, rtol=1e-4, atol=1e-5)


def test_rnncell_matches_oracle():
    torch.manual_seed(3)
    rec = Recurrent().add(RnnCell(3, 4, Tanh()))
    x = torch.randn(2, 5, 3)
    y = rec.forward(x)
    wi, bi, wh, bh = [p.detach() for p in rec.parameters()[0]]
    h = torch.zeros(2, 4)
    outs = []
    for t in range(5):
        h = torch.tanh(x[:, t] @ wi.t() + bi + h @ wh.t() + bh)
        outs.append(h)
    torch.testing.assert_close(y, torch.stack(outs, 1), rtol=1e-5, atol=1e-6)


def _numgrad_check(module, x, eps=1e-3, n=4):
    y = module.forward(x)
    gy = torch.randn_like(y)
    gi = module.backward(x, gy).clone()
    flat = x.reshape(-1)
    idx = torch.randperm(flat.numel())[:n]
    for i in idx:
        xp = flat.clone()
        xp[i] += eps
        xm = flat.clone()
        xm[i] -= eps
        fp = (module.forward(xp.reshape(x.shape)) * gy).sum()
        fm = (module.forward(xm.reshape(x.shape)) * gy).sum()
        num = (fp - fm) / (2 * eps)
        assert abs(float(num) - float(gi.reshape(-1)[i])) < 2e-2 * max(1.0, abs(float(num))), (float(num),
                                                                                              float(gi.reshape(-1)[i]))


def test_lstm_peephole_gradcheck():
    torch.manual_seed(4)
    rec = Recurrent().add(LSTMPeephole(3, 4))
    _numgrad_check(rec, torch.randn(2, 3, 3))


def test_convlstm_shapes_and_grad():
    torch.manual_seed(5)
    rec = Recurrent().add(ConvLSTMPeephole(2, 3, 3, 3, 1))
    x = torch.randn(2, 3, 2, 5, 5)
    y = rec.forward(x)
    assert y.shape == (2, 3, 3, 5, 5)
    _numgrad_check(rec, x, n=3)
    assert all(g.abs().sum() > 0 for g in rec.parameters()[1])


def test_mask_zero_carries_state():
    torch.manual_seed(6)
    rec = Recurrent(maskZero=True).add(LSTM(3, 4))
    x = torch.randn(2, 4, 3)
    x[1, 2:] = 0
    y = rec.forward(x)
    assert torch.all(y[1, 2:] == 0)
    ref = Recurrent().add(LSTM(3, 4))
    ref.getCell().h2g.weight.copy_(rec.getCell().h2g.weight)
    ref.preTopology.layer.weight.copy_(rec.preTopology.layer.weight)
    ref.preTopology.layer.bias.copy_(rec.preTopology.layer.bias)
    y2 = ref.forward(x[1:, :2])
    torch.testing.assert_close(y[1:, :2], y2, rtol=1e-5, atol=1e-6)
    h = rec.getHiddenState()[1]
    torch.testing.assert_close(h[1:], y2[:, -1], rtol=1e-5, atol=1e-6)


def test_birecurrent():
    torch.manual_seed(7)
    bi = BiRecurrent(CAddTable()).add(LSTM(3, 4))
    x = torch.randn(2, 5, 3)
    y = bi.forward(x)
    yf = bi.layer.forward(x)
    yb = torch.flip(bi.revLayer.forward(torch.flip(x, [1])), [1])
    torch.testing.assert_close(y, yf + yb)
    assert bi.backward(x, torch.ones_like(y)).shape == x.shape
    assert len(bi.parameters()[0]) == 6


def test_time_distributed_linear():
    torch.manual_seed(8)
    lin = Linear(4, 3)
    td = TimeDistributed(lin)
    x = torch.randn(2, 5, 4)
    y = td.forward(x)
    torch.testing.assert_close(y, x @ lin.weight.t() + lin.bias)
    gi = td.backward(x, torch.ones_like(y))
    torch.testing.assert_close(gi, torch.ones(2, 5, 3) @ lin.weight)


def test_recurrent_decoder_multicell():
    torch.manual_seed(9)
    cells = [LSTM(4, 4), LSTM(4, 4)]
    dec = RecurrentDecoder(3).add(MultiRNNCell(cells))
    x = torch.randn(2, 4)
    y = dec.forward(x)
    assert y.shape == (2, 3, 4)
    gi = dec.backward(x, torch.randn_like(y))
    assert gi.shape == x.shape
    _numgrad_check(dec, x, n=3)


def test_ptb_lstm_trains():
    from bigdl.models import PTBModel
    from bigdl.nn import TimeDistributedCriterion, CrossEntropyCriterion
    from bigdl.optim import Adagrad
    from bigdl.optim.optimizer import LocalOptimizer
    from bigdl.optim.trigger import Trigger
    from bigdl.dataset import MiniBatch
    torch.manual_seed(10)
    V = 30
    model = PTBModel.lstm(V, 16, V, 2)
    g = torch.Generator().manual_seed(0)
    seq = torch.randint(0, V, (8, 7), generator=g)
    x = (seq[:, :-1] + 1).float()
    y = (seq[:, 1:] + 1).float()
    crit = TimeDistributedCriterion(CrossEntropyCriterion(), size_average=False, dimension=2)
    opt = LocalOptimizer(model, [MiniBatch(x, y)], crit, Adagrad(learningrate=0.1))
    opt.prepare()
    l0 = float(opt.train_step(MiniBatch(x, y)))
    for _ in range(30):
        l = float(opt.train_step(MiniBatch(x, y)))
    assert l < 0.7 * l0
