"""Finite-difference gradient checks (float64, host) over the layer library and the criteria —
the reference's oracle method (spark/dl/src/test/scala/.../nn/GradientChecker.scala:33-256 and its
~60 *Spec users).  Independent of autograd: the analytic gradients come from each module's own
updateGradInput / accGradParameters."""
import pytest
import torch

import bigdl.nn as nn
from bigdl.nn.gradient_checker import GradientChecker

D = torch.float64


def _x(*shape, lo=None, seed=3):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(*shape, generator=g, dtype=D)
    if lo is not None:
        x = x.abs() + lo
    return x


# (id, module factory, input factory, check weights)
LAYERS = [
    ("Linear", lambda: nn.Linear(5, 4), lambda: _x(3, 5), True),
    ("Bilinear", lambda: nn.Bilinear(3, 4, 2), None, True),
    ("SpatialConvolution", lambda: nn.SpatialConvolution(2, 3, 3, 3, 1, 1, 1, 1), lambda: _x(2, 2, 5, 5), True),
    ("SpatialConvolution_s2", lambda: nn.SpatialConvolution(3, 4, 3, 3, 2, 2, 0, 0), lambda: _x(1, 3, 7, 7), True),
    ("SpatialConvolution_group", lambda: nn.SpatialConvolution(4, 4, 3, 3, 1, 1, 1, 1, 2), lambda: _x(1, 4, 5, 5), True),
    ("SpatialDilatedConvolution", lambda: nn.SpatialDilatedConvolution(2, 2, 3, 3, 1, 1, 2, 2, 2, 2), lambda: _x(1, 2, 7, 7), True),
    ("SpatialFullConvolution", lambda: nn.SpatialFullConvolution(2, 3, 3, 3, 2, 2, 1, 1), lambda: _x(1, 2, 4, 4), True),
    ("VolumetricConvolution", lambda: nn.VolumetricConvolution(2, 2, 2, 2, 2), lambda: _x(1, 2, 4, 4, 4), True),
    ("TemporalConvolution", lambda: nn.TemporalConvolution(4, 3, 3), lambda: _x(2, 6, 4), True),
    ("LocallyConnected2D", lambda: nn.LocallyConnected2D(2, 5, 5, 3, 3, 3), lambda: _x(1, 2, 5, 5), True),
    ("BatchNormalization", lambda: nn.BatchNormalization(4), lambda: _x(6, 4), True),
    ("SpatialBatchNormalization", lambda: nn.SpatialBatchNormalization(3), lambda: _x(2, 3, 3, 3), True),
    ("LayerNormalization", lambda: nn.LayerNormalization(6), lambda: _x(3, 6), True),
    ("CMul", lambda: nn.CMul([1, 4]), lambda: _x(3, 4), True),
    ("CAdd", lambda: nn.CAdd([1, 4]), lambda: _x(3, 4), True),
    ("Add", lambda: nn.Add(4), lambda: _x(3, 4), True),
    ("Mul", lambda: nn.Mul(), lambda: _x(3, 4), True),
    ("PReLU", lambda: nn.PReLU(3), lambda: _x(2, 3, 4, 4), True),
    ("Euclidean", lambda: nn.Euclidean(4, 3), lambda: _x(2, 4), True),
    ("Cosine", lambda: nn.Cosine(4, 3), lambda: _x(2, 4), True),
    ("LookupTable", lambda: nn.LookupTable(7, 3), None, True),
    ("Tanh", lambda: nn.Tanh(), lambda: _x(3, 4), False),
    ("Sigmoid", lambda: nn.Sigmoid(), lambda: _x(3, 4), False),
    ("SoftMax", lambda: nn.SoftMax(), lambda: _x(3, 5), False),
    ("LogSoftMax", lambda: nn.LogSoftMax(), lambda: _x(3, 5), False),
    ("SoftMin", lambda: nn.SoftMin(), lambda: _x(3, 5), False),
    ("ELU", lambda: nn.ELU(), lambda: _x(3, 4), False),
    ("SoftPlus", lambda: nn.SoftPlus(), lambda: _x(3, 4), False),
    ("SoftSign", lambda: nn.SoftSign(), lambda: _x(3, 4), False),
    ("LogSigmoid", lambda: nn.LogSigmoid(), lambda: _x(3, 4), False),
    ("TanhShrink", lambda: nn.TanhShrink(), lambda: _x(3, 4), False),
    ("Power", lambda: nn.Power(2.0, 1.5, 0.3), lambda: _x(3, 4), False),
    ("Sqrt", lambda: nn.Sqrt(), lambda: _x(3, 4, lo=0.5), False),
    ("Square", lambda: nn.Square(), lambda: _x(3, 4), False),
    ("Log", lambda: nn.Log(), lambda: _x(3, 4, lo=0.5), False),
    ("Exp", lambda: nn.Exp(), lambda: _x(3, 4), False),
    ("Normalize", lambda: nn.Normalize(2.0), lambda: _x(3, 4), False),
    ("SpatialMaxPooling", lambda: nn.SpatialMaxPooling(2, 2, 2, 2), lambda: _x(1, 2, 4, 4), False),
    ("SpatialAveragePooling", lambda: nn.SpatialAveragePooling(3, 3, 2, 2, 1, 1), lambda: _x(1, 2, 5, 5), False),
    ("SpatialCrossMapLRN", lambda: nn.SpatialCrossMapLRN(3, 1.0, 0.75, 1.0), lambda: _x(1, 5, 3, 3), False),
    ("SpatialWithinChannelLRN", lambda: nn.SpatialWithinChannelLRN(3, 1.0, 0.75), lambda: _x(1, 2, 4, 4), False),
    ("VolumetricMaxPooling", lambda: nn.VolumetricMaxPooling(2, 2, 2, 2, 2, 2), lambda: _x(1, 2, 4, 4, 4), False),
    ("TemporalMaxPooling", lambda: nn.TemporalMaxPooling(2), lambda: _x(2, 6, 3), False),
    ("Mean", lambda: nn.Mean(2), lambda: _x(3, 4), False),
    ("Sum", lambda: nn.Sum(2), lambda: _x(3, 4), False),
    ("Max", lambda: nn.Max(2), lambda: _x(3, 4), False),
    ("Transpose", lambda: nn.Transpose([(1, 2)]), lambda: _x(3, 4), False),
    ("Replicate", lambda: nn.Replicate(3, 2), lambda: _x(2, 4), False),
    ("ResizeBilinear", lambda: nn.ResizeBilinear(6, 6), lambda: _x(1, 2, 4, 4), False),
    ("UpSampling2D", lambda: nn.UpSampling2D([2, 2]), lambda: _x(1, 2, 3, 3), False),
    ("SpatialZeroPadding", lambda: nn.SpatialZeroPadding(1, 1, 2, 0), lambda: _x(1, 2, 3, 3), False),
]


def _bilinear_in():
    from bigdl.utils.table import T
    return T(_x(2, 3, seed=1), _x(2, 4, seed=2))


def _lookup_in():
    return torch.tensor([[1.0, 3.0, 7.0], [2.0, 2.0, 5.0]], dtype=D)


@pytest.mark.parametrize("name,make,inp,weights", LAYERS, ids=[l[0] for l in LAYERS])
def test_layer_gradients_finite_difference(name, make, inp, weights):
    m = make().to(dtype=D)
    m.training()
    checker = GradientChecker(1e-6, 1e-5)
    if name == "Bilinear":
        x = _bilinear_in()
    elif name == "LookupTable":
        x = _lookup_in()
    else:
        x = inp()
    if name not in ("Bilinear", "LookupTable"):
        assert checker.checkLayer(m, x, num=None), (name, checker.last_report)
    if weights:
        assert checker.checkWeight(m, x, num=None), (name, checker.last_report)


def _lstm():
    return nn.Recurrent().add(nn.LSTM(3, 4))


def _gru():
    return nn.Recurrent().add(nn.GRU(3, 4))


def _rnn():
    return nn.Recurrent().add(nn.RnnCell(3, 4, nn.Tanh()))


@pytest.mark.parametrize("make", [_lstm, _gru, _rnn], ids=["LSTM", "GRU", "RnnCell"])
def test_recurrent_gradients_finite_difference(make):
    m = make().to(dtype=D)
    x = _x(2, 3, 3)
    checker = GradientChecker(1e-6, 1e-5)
    assert checker.checkLayer(m, x, num=None), checker.last_report
    assert checker.checkWeight(m, x, num=None), checker.last_report


def _cls_target():
    return torch.tensor([1.0, 3.0, 2.0], dtype=D)


CRITERIA = [
    ("MSECriterion", lambda: nn.MSECriterion(), lambda: _x(3, 4), lambda: _x(3, 4, seed=9)),
    ("AbsCriterion", lambda: nn.AbsCriterion(), lambda: _x(3, 4), lambda: _x(3, 4, seed=9)),
    ("SmoothL1Criterion", lambda: nn.SmoothL1Criterion(), lambda: _x(3, 4), lambda: _x(3, 4, seed=9)),
    ("ClassNLLCriterion", lambda: nn.ClassNLLCriterion(), lambda: _x(3, 4), _cls_target),
    ("CrossEntropyCriterion", lambda: nn.CrossEntropyCriterion(), lambda: _x(3, 4), _cls_target),
    ("BCECriterion", lambda: nn.BCECriterion(), lambda: torch.sigmoid(_x(3, 4)),
     lambda: (_x(3, 4, seed=9) > 0).to(D)),
    ("SoftMarginCriterion", lambda: nn.SoftMarginCriterion(), lambda: _x(3, 4),
     lambda: torch.sign(_x(3, 4, seed=9))),
    ("MarginCriterion", lambda: nn.MarginCriterion(), lambda: _x(3, 4) * 0.3, lambda: torch.sign(_x(3, 4, seed=9))),
    ("MultiMarginCriterion", lambda: nn.MultiMarginCriterion(), lambda: _x(3, 4) * 0.3, _cls_target),
    ("MultiLabelSoftMarginCriterion", lambda: nn.MultiLabelSoftMarginCriterion(), lambda: _x(3, 4),
     lambda: (_x(3, 4, seed=9) > 0).to(D)),
    ("DistKLDivCriterion", lambda: nn.DistKLDivCriterion(), lambda: torch.log_softmax(_x(3, 4), 1),
     lambda: torch.softmax(_x(3, 4, seed=9), 1)),
    ("KullbackLeiblerDivergenceCriterion", lambda: nn.KullbackLeiblerDivergenceCriterion(),
     lambda: torch.softmax(_x(3, 4), 1), lambda: torch.softmax(_x(3, 4, seed=9), 1)),
    ("PoissonCriterion", lambda: nn.PoissonCriterion(), lambda: _x(3, 4, lo=0.5), lambda: _x(3, 4, lo=0.1, seed=9)),
    ("MeanSquaredLogarithmicCriterion", lambda: nn.MeanSquaredLogarithmicCriterion(), lambda: _x(3, 4, lo=0.5),
     lambda: _x(3, 4, lo=0.1, seed=9)),
    ("MeanAbsolutePercentageCriterion", lambda: nn.MeanAbsolutePercentageCriterion(), lambda: _x(3, 4),
     lambda: _x(3, 4, lo=0.5, seed=9)),
    ("CosineProximityCriterion", lambda: nn.CosineProximityCriterion(), lambda: _x(3, 4), lambda: _x(3, 4, seed=9)),
    ("CategoricalCrossEntropy", lambda: nn.CategoricalCrossEntropy(), lambda: torch.softmax(_x(3, 4), 1),
     lambda: torch.eye(4, dtype=D)[:3]),
    ("L1Cost", lambda: nn.L1Cost(), lambda: _x(3, 4), lambda: _x(3, 4, seed=9)),
]


@pytest.mark.parametrize("name,make,inp,tgt", CRITERIA, ids=[c[0] for c in CRITERIA])
def test_criterion_gradients_finite_difference(name, make, inp, tgt):
    c = make()
    x, t = inp(), tgt()
    checker = GradientChecker(1e-6, 1e-5)
    assert checker.checkCriterion(c, x, t, num=None), (name, checker.last_report)


def _T(*ts):
    from bigdl.utils.table import T
    return T(*ts)


MORE_LAYERS = [
    ("HardTanh", lambda: nn.HardTanh(), lambda: _x(3, 4) * 0.7, False),
    ("LeakyReLU", lambda: nn.LeakyReLU(0.1), lambda: _x(3, 4), False),
    ("ReLU", lambda: nn.ReLU(), lambda: _x(3, 4), False),
    ("ReLU6", lambda: nn.ReLU6(), lambda: _x(3, 4) * 3, False),
    ("Threshold", lambda: nn.Threshold(0.2, -1.0), lambda: _x(3, 4), False),
    ("Clamp", lambda: nn.Clamp(-0.5, 0.5), lambda: _x(3, 4), False),
    ("HardShrink", lambda: nn.HardShrink(0.3), lambda: _x(3, 4), False),
    ("SoftShrink", lambda: nn.SoftShrink(0.3), lambda: _x(3, 4), False),
    ("HardSigmoid", lambda: nn.HardSigmoid(), lambda: _x(3, 4), False),
    ("Abs", lambda: nn.Abs(), lambda: _x(3, 4), False),
    ("MulConstant", lambda: nn.MulConstant(1.7), lambda: _x(3, 4), False),
    ("AddConstant", lambda: nn.AddConstant(0.3), lambda: _x(3, 4), False),
    ("Negative", lambda: nn.Negative(), lambda: _x(3, 4), False),
    ("SReLU", lambda: nn.SReLU([4]), lambda: _x(3, 4), True),
    ("Maxout", lambda: nn.Maxout(4, 3, 2), lambda: _x(3, 4), True),
    ("Highway", lambda: nn.Highway(4), lambda: _x(3, 4), True),
    ("Scale", lambda: nn.Scale([1, 3, 1, 1]), lambda: _x(2, 3, 2, 2), True),
    ("NormalizeScale", lambda: nn.NormalizeScale(2.0, scale=2.0, size=[1, 3, 1, 1]), lambda: _x(2, 3, 2, 2), True),
    ("SpatialSeparableConvolution", lambda: nn.SpatialSeparableConvolution(2, 4, 2, 3, 3), lambda: _x(1, 2, 5, 5), True),
    ("VolumetricFullConvolution", lambda: nn.VolumetricFullConvolution(2, 2, 2, 2, 2, 1, 1, 1), lambda: _x(1, 2, 3, 3, 3), True),
    ("VolumetricAveragePooling", lambda: nn.VolumetricAveragePooling(2, 2, 2, 1, 1, 1), lambda: _x(1, 2, 3, 3, 3), False),
    ("LocallyConnected1D", lambda: nn.LocallyConnected1D(6, 3, 2, 3), lambda: _x(2, 6, 3), True),
    ("SpatialSubtractiveNormalization", lambda: nn.SpatialSubtractiveNormalization(2), lambda: _x(1, 2, 6, 6), False),
    ("SpatialDivisiveNormalization", lambda: nn.SpatialDivisiveNormalization(2), lambda: _x(1, 2, 6, 6), False),
    ("UpSampling1D", lambda: nn.UpSampling1D(2), lambda: _x(2, 3, 4), False),
    ("Cropping2D", lambda: nn.Cropping2D([1, 0], [0, 1]), lambda: _x(1, 2, 4, 4), False),
    ("Padding", lambda: nn.Padding(2, 2, 2), lambda: _x(3, 4), False),
    ("Narrow", lambda: nn.Narrow(2, 2, 2), lambda: _x(3, 4), False),
    ("Select", lambda: nn.Select(2, 3), lambda: _x(3, 4), False),
    ("Reshape", lambda: nn.Reshape([2, 2]), lambda: _x(3, 4), False),
    ("Squeeze", lambda: nn.Squeeze(2), lambda: _x(3, 1, 4), False),
    ("Unsqueeze", lambda: nn.Unsqueeze(2), lambda: _x(3, 4), False),
    ("Contiguous", lambda: nn.Contiguous(), lambda: _x(3, 4), False),
    ("GradientReversal", lambda: nn.GradientReversal(0.5), lambda: _x(3, 4), None),
    ("TimeDistributed_Linear", lambda: nn.TimeDistributed(nn.Linear(4, 3)), lambda: _x(2, 3, 4), True),
    ("Bottle_Linear", lambda: nn.Bottle(nn.Linear(4, 3), 2, 2), lambda: _x(2, 3, 4), True),
    ("Sequential_MLP", lambda: nn.Sequential().add(nn.Linear(4, 5)).add(nn.Tanh()).add(nn.Linear(5, 2)),
     lambda: _x(3, 4), True),
    ("Concat", lambda: nn.Concat(2).add(nn.Linear(4, 2)).add(nn.Linear(4, 3)), lambda: _x(3, 4), True),
]


@pytest.mark.parametrize("name,make,inp,weights", MORE_LAYERS, ids=[l[0] for l in MORE_LAYERS])
def test_more_layer_gradients_finite_difference(name, make, inp, weights):
    m = make().to(dtype=D)
    m.training()
    x = inp()
    checker = GradientChecker(1e-6, 1e-5)
    if weights is None:  # GradientReversal: backward = −λ · forward gradient by design
        m.forward(x)
        gi = m.updateGradInput(x, x.clone())
        torch.testing.assert_close(gi, -0.5 * x)
        return
    assert checker.checkLayer(m, x, num=None), (name, checker.last_report)
    if weights:
        assert checker.checkWeight(m, x, num=None), (name, checker.last_report)


TABLE_LAYERS = [
    ("CAddTable", lambda: nn.CAddTable(), lambda: _T(_x(3, 4, seed=1), _x(3, 4, seed=2))),
    ("CSubTable", lambda: nn.CSubTable(), lambda: _T(_x(3, 4, seed=1), _x(3, 4, seed=2))),
    ("CMulTable", lambda: nn.CMulTable(), lambda: _T(_x(3, 4, seed=1), _x(3, 4, seed=2))),
    ("CDivTable", lambda: nn.CDivTable(), lambda: _T(_x(3, 4, seed=1), _x(3, 4, lo=0.5, seed=2))),
    ("CMaxTable", lambda: nn.CMaxTable(), lambda: _T(_x(3, 4, seed=1), _x(3, 4, seed=2))),
    ("JoinTable", lambda: nn.JoinTable(2, 2), lambda: _T(_x(3, 4, seed=1), _x(3, 2, seed=2))),
    ("MM", lambda: nn.MM(), lambda: _T(_x(2, 3, 4, seed=1), _x(2, 4, 2, seed=2))),
    ("MV", lambda: nn.MV(), lambda: _T(_x(2, 3, 4, seed=1), _x(2, 4, seed=2))),
    ("DotProduct", lambda: nn.DotProduct(), lambda: _T(_x(3, 4, seed=1), _x(3, 4, seed=2))),
    ("CosineDistance", lambda: nn.CosineDistance(), lambda: _T(_x(3, 4, seed=1), _x(3, 4, seed=2))),
    ("PairwiseDistance", lambda: nn.PairwiseDistance(2), lambda: _T(_x(3, 4, seed=1), _x(3, 4, seed=2))),
    ("CrossProduct", lambda: nn.CrossProduct(), lambda: _T(_x(3, 4, seed=1), _x(3, 4, seed=2), _x(3, 4, seed=5))),
    ("MixtureTable", lambda: nn.MixtureTable(), lambda: _T(torch.softmax(_x(3, 2, seed=1), 1),
                                                          _T(_x(3, 4, seed=2), _x(3, 4, seed=3)))),
]


@pytest.mark.parametrize("name,make,inp", TABLE_LAYERS, ids=[l[0] for l in TABLE_LAYERS])
def test_table_layer_gradients_finite_difference(name, make, inp):
    m = make().to(dtype=D)
    x = inp()
    checker = GradientChecker(1e-6, 1e-5)
    assert checker.checkLayer(m, x, num=None), (name, checker.last_report)


def test_lstm_peephole_and_birecurrent_gradients():
    checker = GradientChecker(1e-6, 1e-5)
    for make in (lambda: nn.Recurrent().add(nn.LSTMPeephole(3, 4)),
                 lambda: nn.BiRecurrent().add(nn.LSTM(3, 4))):
        m = make().to(dtype=D)
        x = _x(2, 3, 3)
        assert checker.checkLayer(m, x, num=None), checker.last_report
        assert checker.checkWeight(m, x, num=None), checker.last_report
