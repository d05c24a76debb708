"""IR graph (``DL/utils/intermediate``): module → IR → device graph; inference lowering folds
BatchNorm into the preceding conv/linear and drops Dropout; training lowering keeps parameters
shared with the source model."""
import torch

from bigdl.nn import (Sequential, SpatialConvolution, SpatialBatchNormalization, ReLU, SpatialMaxPooling, View,
                      Linear, BatchNormalization, Dropout, LogSoftMax, SpatialBatchNormalization as SBN)
from bigdl.utils.intermediate import to_ir, ConversionUtils, IRGraph, IRSpatialConvolution


def _net():
    torch.manual_seed(0)
    m = (Sequential()
         .add(SpatialConvolution(3, 8, 3, 3, 1, 1, 1, 1)).add(SpatialBatchNormalization(8)).add(ReLU())
         .add(SpatialMaxPooling(2, 2, 2, 2))
         .add(SpatialConvolution(8, 16, 3, 3, 1, 1, 1, 1, with_bias=False)).add(SBN(16)).add(ReLU())
         .add(View(16 * 4 * 4)).add(Dropout(0.5))
         .add(Linear(256, 32)).add(BatchNormalization(32)).add(ReLU()).add(Linear(32, 10)).add(LogSoftMax()))
    # non-trivial running statistics
    m.training()
    for _ in range(3):
        m.forward(torch.randn(4, 3, 8, 8) * 2 + 0.5)
    return m


def test_ir_inference_folds_bn_and_matches():
    m = _net()
    m.evaluate()
    x = torch.randn(5, 3, 8, 8)
    ref = m.forward(x).clone()
    ir = to_ir(m)
    assert any(isinstance(n.element.op, IRSpatialConvolution) for n in ir.order)
    ir.evaluate()
    ir.build()
    assert isinstance(ir, IRGraph) and ir.isBuild()
    kinds = [type(n.element).__name__ for n in ir.graph.forward_order]
    assert "SpatialBatchNormalization" not in kinds and "BatchNormalization" not in kinds and "Dropout" not in kinds
    torch.testing.assert_close(ir.forward(x), ref, rtol=1e-4, atol=1e-4)
    # the source model is untouched (its BNs still run)
    torch.testing.assert_close(m.forward(x), ref, rtol=0, atol=0)


def test_ir_training_shares_parameters_and_trains():
    m = _net()
    ir = ConversionUtils.convert(m)
    x = torch.randn(6, 3, 8, 8)
    y = torch.randint(1, 11, (6,)).float()
    from bigdl.nn import ClassNLLCriterion
    crit = ClassNLLCriterion()
    w_ir, _ = ir.parameters()
    w_m, _ = m.parameters()
    assert all(a is b for a, b in zip(w_ir, w_m))
    out = ir.forward(x)
    loss0 = float(crit.forward(out, y))
    ir.zeroGradParameters()
    ir.backward(x, crit.backward(out, y))
    for w, g in zip(*ir.parameters()):
        w.add_(g, alpha=-0.05)
    ir.evaluate()
    ir.training()
    loss1 = float(crit.forward(ir.forward(x), y))
    assert loss1 < loss0
    # evaluate() re-folds from the updated weights
    ir.evaluate()
    m.evaluate()
    torch.testing.assert_close(ir.forward(x), m.forward(x), rtol=1e-4, atol=1e-4)


def test_to_ir_graph_method():
    m = _net()
    m.evaluate()
    x = torch.randn(2, 3, 8, 8)
    ir = m.toIRgraph()
    torch.testing.assert_close(ir.forward(x), m.forward(x), rtol=1e-4, atol=1e-4)


def test_ir_resnet_block_tail_fuses_conv_sum():
    from bigdl.models.resnet import ResNet, DatasetType, model_init
    from bigdl.nn.layers.conv import FusedConvSum
    torch.manual_seed(0)
    m = model_init(ResNet(10, depth=20, dataset=DatasetType.CIFAR10))
    m.training()
    m.forward(torch.randn(4, 3, 32, 32))
    m.evaluate()
    x = torch.randn(3, 3, 32, 32)
    ref = m.forward(x).clone()
    ir = m.toIRgraph()
    kinds = [type(n.element).__name__ for n in ir.graph.forward_order]
    assert kinds.count("FusedConvSum") >= 8, kinds
    assert "SpatialBatchNormalization" not in kinds and "CAddTable" not in kinds
    torch.testing.assert_close(ir.forward(x), ref, rtol=1e-4, atol=1e-4)
