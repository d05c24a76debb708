"""Tensor / TensorMath compatibility surface added in round 4 (``DL/tensor/TensorMath.scala:222-824``,
``DL/tensor/Tensor.scala:113-725``), with golden values from the reference's own specs
(``spark/dl/src/test/scala/.../tensor/TensorConvSpec.scala``, ``DenseTensorMathSpec.scala``)."""
import numpy as np
import pytest
import torch

from bigdl.tensor import Tensor, Storage


def _t34():
    return Tensor(torch.tensor([[1., 2, 3, 4], [2, 3, 4, 5], [3, 4, 5, 6]], dtype=torch.float64))


def _k22():
    return Tensor(torch.tensor([[1., 2], [3, 4]], dtype=torch.float64))


def test_conv2_xcorr2_golden():
    # TensorConvSpec.scala: "Valid conv", "Full conv", "Valid xcorr", "Full Xcorr"
    assert _t34().conv2(_k22()).toArray() == [17, 27, 37, 27, 37, 47]
    r = _t34().conv2(_k22(), "F")
    assert r.shape == (4, 5)
    assert r.toArray() == [1, 4, 7, 10, 8, 5, 17, 27, 37, 26, 9, 27, 37, 47, 32, 9, 24, 31, 38, 24]
    assert _t34().xcorr2(_k22()).toArray() == [23, 33, 43, 33, 43, 53]
    r = _t34().xcorr2(_k22(), "F")
    assert r.toArray() == [4, 11, 18, 25, 12, 10, 23, 33, 43, 19, 16, 33, 43, 53, 23, 6, 11, 14, 17, 6]
    with pytest.raises(ValueError):
        _t34().conv2(_k22(), "X")


def test_uniform_golden_ranges():
    # DenseTensorMathSpec.scala:473-500
    t = Tensor(1)
    for _ in range(100):
        assert 0.0 <= t.uniform() < 1.0
    assert t.uniform(1.0) == 1.0
    for _ in range(100):
        assert 1.0 <= t.uniform(11.0) <= 11.0
    assert t.uniform(1.0, 1.0) == 1.0 and t.uniform(-2.0, -2.0) == -2.0
    for _ in range(100):
        assert -11.0 <= t.uniform(-11.0, 11.0) <= 11.0


def test_ge_sign_cmax_cmin():
    x = Tensor(torch.tensor([-2., 0., 3.]))
    assert Tensor(3).ge(x, 0.0).toArray() == [0, 1, 1]
    assert x.clone().sign().toArray() == [-1, 0, 1]
    assert x.clone().cmax(1.0).toArray() == [1, 1, 3]
    assert x.clone().cmin(1.0).toArray() == [-2, 0, 1]
    y = Tensor(torch.tensor([1., -1., 5.]))
    assert x.clone().cmax(y).toArray() == [1, 0, 5]
    assert Tensor(3).cmin(x, y).toArray() == [-2, -1, 3]
    assert x.notEqualValue(0.0) and not Tensor(torch.zeros(3)).notEqualValue(0.0)


def test_reduce_apply_zip_cast():
    t = Tensor(torch.tensor([[1., 2, 3], [4, 5, 6]]))
    r = t.reduce(2, Tensor(2, 1), lambda a, b: a + b)
    assert r.toArray() == [6, 15]
    r = t.reduce(1, Tensor(1, 3), max)
    assert r.toArray() == [4, 5, 6]
    d = Tensor(torch.zeros(2, 3, dtype=torch.float64)).applyFun(t, lambda v: v * v)
    assert d.toArray() == [1, 4, 9, 16, 25, 36] and d.data.dtype == torch.float64
    z = Tensor(2, 3).zipWith(t, t, lambda a, b: a - 2 * b)
    assert z.toArray() == [-1, -2, -3, -4, -5, -6]
    i = t.cast(Tensor(torch.zeros(1, dtype=torch.int32)))
    assert i.data.dtype == torch.int32 and i.shape == (2, 3) and i.toArray() == [1, 2, 3, 4, 5, 6]
    f = Tensor(torch.zeros(2, dtype=torch.int64)).forceFill(3.7)
    assert f.toArray() == [3, 3]


def test_storage_shared_and_offsets():
    t = Tensor(torch.arange(6, dtype=torch.float32).view(2, 3))
    s = t.storage()
    assert isinstance(s, Storage) and s.length() == 6 and s.apply(4) == 4.0
    s.update(0, 10.0)
    assert t.valueAt(1, 1) == 10.0  # shared, not a copy
    col = t.select(2, 2)  # a strided view: its storage is the whole buffer
    assert col.storage().length() == 6
    s.fill(-1.0, 5, 2)  # 1-based offset
    assert t.toArray() == [10, 1, 2, 3, -1, -1]
    s2 = Storage(torch.zeros(4))
    s2.copy(s, 2, 1, 3)
    assert s2.array().tolist() == [0, 10, 1, 2]
    assert s2.resize(2).length() == 2


def test_value_dims_clone_update(tmp_path):
    assert Tensor.scalar(2.5).value() == 2.5
    with pytest.raises(ValueError):
        Tensor(2, 2).value()
    t = Tensor(torch.ones(3, 1, 2))
    assert t.dim() == 3 and t.squeezeNewTensor().shape == (3, 2) and t.shape == (3, 1, 2)
    sc = t.shallowClone()
    sc.data[0, 0, 0] = 7.0
    assert t.valueAt(1, 1, 1) == 7.0
    assert t.emptyInstance().nElement() == 0
    a = Tensor(torch.ones(2, 3)).addSingletonDimension(dim=2)
    assert a.shape == (2, 1, 3)
    b = Tensor(torch.ones(2, 3)).addMultiDimension(dims=[1, 3])
    assert b.shape == (1, 2, 3, 1)
    u = Tensor(torch.zeros(2, 2))
    u.update(1, 5.0)
    u.update([2, 2], 3.0)
    u.update(lambda v: v == 0, -1.0)
    assert u.toArray() == [5, 5, -1, 3]
    assert Tensor(torch.tensor([[0., 1], [2, 3]])).numNonZeroByRow() == [1, 2]
    p = str(tmp_path / "t.npy")
    Tensor(torch.tensor([[1., 2], [3, 4]])).save(p)
    with pytest.raises(FileExistsError):
        Tensor(1).save(p)
    assert Tensor.load(p).toArray() == [1, 2, 3, 4]
    assert not Tensor(torch.ones(2)).diff(Tensor(torch.ones(2)))
    assert Tensor(torch.ones(2)).diff(Tensor(torch.zeros(2)), count=2)
    assert Tensor(torch.ones(2)).diff(Tensor(torch.ones(3)))
    assert Tensor(torch.zeros(1)).getTensorType() == "DenseType"
    assert Tensor(torch.zeros(1, dtype=torch.float64)).getTensorNumeric() == "double"
