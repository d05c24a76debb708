"""Native CSR SpMM (ops/csrc/sparse.hip, K27) against fp32 dense references: the raw kernel,
SparseLinear forward/backward and SparseTensor.mm (reference SparseTensorBLAS.coomm,
SparseLinear.scala)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"


def _native():
    from bigdl.ops import native as N
    from bigdl.utils.engine import Engine
    Engine.init(device="cuda:0")
    assert N.status()["loaded"] and N.has("spmm")
    return N


def _sparse(M, K, density, seed=0):
    g = torch.Generator().manual_seed(seed)
    d = torch.randn(M, K, generator=g) * (torch.rand(M, K, generator=g) < density)
    d[3] = 0  # an empty row
    return d


@pytest.mark.parametrize("M,K,N,bdt", [(37, 50, 16, torch.float32), (128, 300, 64, torch.bfloat16),
                                       (5, 8, 260, torch.float32)])
def test_spmm_matches_dense(M, K, N, bdt):
    N_ = _native()
    d = _sparse(M, K, 0.1)
    b = torch.randn(K, N).to(bdt)
    out = N_.native_ops.spmm(d.to_sparse().to(dev), b.to(dev), alpha=0.5)
    ref = 0.5 * (d @ b.float())
    torch.testing.assert_close(out.cpu(), ref, rtol=1e-5, atol=1e-5)


def test_sparse_linear_forward_backward_native():
    N_ = _native()
    from bigdl.nn import SparseLinear, Linear
    N_.reset_fallbacks()
    torch.manual_seed(0)
    d = _sparse(32, 40, 0.15)
    lin = SparseLinear(40, 12)
    ref = Linear(40, 12)
    ref.weight.data.copy_(lin.weight.data)
    ref.bias.data.copy_(lin.bias.data)
    lin.cuda()
    y = lin.forward(d.to_sparse().to(dev))
    yr = ref.forward(d)
    torch.testing.assert_close(y.cpu(), yr, rtol=1e-5, atol=1e-5)
    g = torch.randn(32, 12)
    lin.backward(d.to_sparse().to(dev), g.to(dev))
    ref.backward(d, g)
    torch.testing.assert_close(lin.gradWeight.cpu(), ref.gradWeight, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(lin.gradBias.cpu(), ref.gradBias, rtol=1e-4, atol=1e-5)
    assert not [k for k in N_.fallback_counts() if k[0] == "spmm"]


def test_sparse_tensor_mm_native():
    _native()
    from bigdl.tensor.sparse import SparseTensor
    d = _sparse(20, 30, 0.2)
    st = SparseTensor.from_dense(d)
    b = torch.randn(30, 8)
    torch.testing.assert_close(st.mm(b.to(dev)).cpu(), d @ b, rtol=1e-5, atol=1e-5)
