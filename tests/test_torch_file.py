"""Torch7 .t7 reader/writer (TorchFile.scala): real fixtures from the reference's test resources
and module round trips (forward equality after save → load)."""
import os

import numpy as np
import pytest
import torch

from bigdl import nn
from bigdl.nn.module import Module
from bigdl.serialization.torch_file import load_torch_file, save_torch_file
from bigdl.utils.table import Table

FIX = "/root/reference/spark/dl/src/test/resources/torch"


@pytest.mark.skipif(not os.path.isdir(FIX), reason="reference fixtures not mounted")
def test_reads_reference_tensor_fixture():
    t = load_torch_file(os.path.join(FIX, "n02110063_11239.t7"))
    assert isinstance(t, torch.Tensor) and t.shape == (3, 224, 224) and t.dtype == torch.float32
    assert torch.isfinite(t).all()


def test_tensor_table_roundtrip(tmp_path):
    p = str(tmp_path / "a.t7")
    t = Table()
    t[1] = torch.randn(3, 4)
    t["name"] = "abc"
    t["flag"] = True
    t["n"] = 3.5
    t["ids"] = torch.arange(5)
    t["d"] = torch.randn(2).double()
    save_torch_file(t, p)
    r = load_torch_file(p)
    torch.testing.assert_close(r[1], t[1])
    assert r["name"] == "abc" and r["flag"] is True and r["n"] == 3.5
    assert r["ids"].tolist() == list(range(5)) and r["d"].dtype == torch.float64


def _net():
    m = nn.Sequential()
    m.add(nn.SpatialZeroPadding(1, 1, 1, 1))
    m.add(nn.SpatialConvolution(3, 8, 3, 3, 1, 1, 0, 0))
    m.add(nn.SpatialBatchNormalization(8))
    m.add(nn.ReLU())
    m.add(nn.SpatialCrossMapLRN(3, 1e-3, 0.75, 1.0))
    m.add(nn.SpatialMaxPooling(2, 2, 2, 2).ceil())
    ct = nn.ConcatTable().add(nn.Threshold(0.1, 0.0)).add(nn.LeakyReLU(0.2))
    m.add(ct)
    m.add(nn.CAddTable())
    c = nn.Concat(2).add(nn.SpatialAveragePooling(2, 2, 2, 2)).add(nn.SpatialAveragePooling(2, 2, 2, 2))
    m.add(c)
    m.add(nn.View([16 * 2 * 2]).setNumInputDims(3))
    m.add(nn.Dropout(0.3))
    m.add(nn.Linear(64, 10))
    m.add(nn.Reshape([2, 5]))
    return m


def test_module_roundtrip_forward_equal(tmp_path):
    m = _net()
    m.evaluate()
    x = torch.randn(2, 3, 8, 8)
    y = m.forward(x).clone()
    p = str(tmp_path / "m.t7")
    m.saveTorch(p)
    m2 = Module.loadTorch(p)
    m2.evaluate()
    assert [type(a).__name__ for a in m2.modules] == [type(a).__name__ for a in m.modules]
    torch.testing.assert_close(m2.forward(x), y, rtol=1e-5, atol=1e-5)
