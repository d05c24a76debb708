"""Layout / wire kernels (elementwise.hip): the truncating fp32→bf16 wire cast of the reference's
compressed gradient format (FP16CompressedTensor.scala:43-277) and the one-pass NCHW → NHWC bf16
relayout at the host/device boundary — each against the plain torch formulation."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def N():
    from bigdl.ops import native
    from bigdl.utils.engine import Engine
    Engine.init(device="cuda:0")
    assert native.status()["loaded"] and native.has("trunc_bf16") and native.has("nchw_to_nhwc_bf16")
    return native


@pytest.mark.parametrize("n", [1, 3, 4, 1000, 1 << 20, (1 << 20) + 3])
def test_trunc_bf16_matches_bit_shift(N, n):
    from bigdl.parallel import comm
    g = torch.randn(n, device="cuda") * 3.0
    wire = torch.empty(n, dtype=torch.bfloat16, device="cuda")
    assert N.native_ops.trunc_bf16(g, wire) is wire
    ref = comm.bf16_truncate(g)
    assert torch.equal(wire.view(torch.int16), ref.view(torch.int16))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(2, 3, 224, 224), (4, 64, 7, 7), (1, 33, 5, 13), (3, 1, 1, 1)])
def test_nchw_to_nhwc_bf16(N, dtype, shape):
    x = torch.randn(shape, device="cuda").to(dtype)
    y = N.native_ops.nchw_to_nhwc_bf16(x)
    ref = x.float().to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    assert y.is_contiguous(memory_format=torch.channels_last) and y.dtype == torch.bfloat16
    assert torch.equal(y, ref)


def test_to_device_layout_uses_native_relayout(N):
    from bigdl.nn.layers.conv import to_device_layout
    from bigdl.utils.engine import Engine
    if Engine.compute_dtype() != torch.bfloat16:
        pytest.skip("compute dtype is not bf16")
    x = torch.randn(2, 3, 32, 32, device="cuda")
    y = to_device_layout(x)
    assert torch.equal(y, x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last))
