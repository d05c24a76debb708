"""GPU checks for the distributed hot path's kernels and the embedding id check.

* ``bigdl_sgd_g16``: the fused SGD reading the bf16 reduce-scatter output directly must equal the
  fp32 reference update fed the widened gradient (no separate unpack pass).
* ``LookupTable`` ids outside [1, nIndex] raise (``LookupTable.scala:96-98``) via the device error
  flag; masked padding ids are accepted."""
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"


@pytest.mark.parametrize("n", [4096, 1003])
@pytest.mark.parametrize("nesterov,per_elem", [(True, True), (False, False)])
def test_sgd_bf16_grad_matches_fp32_reference(n, nesterov, per_elem):
    from bigdl.ops import native_ops as NO, reference as R
    torch.manual_seed(0)
    w = torch.randn(n, device=dev)
    g16 = torch.randn(n, device=dev).to(torch.bfloat16)
    buf = torch.randn(n, device=dev)
    wds = torch.rand(n, device=dev) if per_elem else None
    w2, buf2 = w.clone(), buf.clone()
    sh = torch.empty(n, dtype=torch.bfloat16, device=dev)
    assert NO.sgd_step(w, g16, buf, 0.1, 0.9, 0.0, 1e-4 if not per_elem else 1.0, nesterov, False, 0.125, sh,
                       None, wds) is not NotImplemented
    R.sgd_step(w2, g16.float(), buf2, 0.1, 0.9, 0.0, 1e-4 if not per_elem else 1.0, nesterov, False, 0.125, None,
               None, wds)
    torch.testing.assert_close(w, w2, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(buf, buf2, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(sh, w2.to(torch.bfloat16), rtol=0, atol=0)


def test_embedding_out_of_range_id_raises():
    from bigdl.ops import native_ops as NO
    w = torch.randn(10, 16, device=dev)
    ok = torch.tensor([[1.0, 10.0], [3.0, 4.0]], device=dev)
    out = NO.embedding_forward(w, ok)
    NO.embedding_check(sync=True)  # in-range ids: no error
    torch.testing.assert_close(out, w[ok.long() - 1])
    for bad in (11.0, 0.0):
        NO.embedding_forward(w, torch.tensor([[1.0, bad]], device=dev))
        with pytest.raises(IndexError, match="outside"):
            NO.embedding_check(sync=True)
    # the error is reported lazily by the next lookup too
    NO.embedding_forward(w, torch.tensor([12.0], device=dev))
    torch.cuda.synchronize()
    with pytest.raises(IndexError):
        NO.embedding_forward(w, ok)
    NO.embedding_check(sync=True)
    # maskZero: the padding id is accepted
    NO.embedding_forward(w, torch.tensor([0.0, 2.0], device=dev), 0.0, True)
    NO.embedding_check(sync=True)


def test_bn_apply_relu_bits_match_output():
    """The fused block-tail BN writes its output's ReLU mask as bits (one byte per 8 channels,
    NHWC chunk order) — must equal (y > 0) of the stored bf16 output."""
    from bigdl.ops import native_ops as NO, reference as R
    torch.manual_seed(0)
    x = torch.randn(4, 64, 7, 9, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    res = torch.randn_like(x)
    C = 64
    g, b = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    bits = torch.empty(x.numel() // 8, dtype=torch.uint8, device=dev)
    y, _, _ = NO.batchnorm_forward_train(x, g, b, rm, rv, 0.1, 1e-3, relu=True, residual=res, bits_out=bits)
    ref_bits = torch.empty_like(bits)
    pos = (y.permute(0, 2, 3, 1).reshape(-1, 8) > 0).to(torch.int32)
    ref_bits.copy_((pos * (2 ** torch.arange(8, device=dev, dtype=torch.int32))).sum(1).to(torch.uint8))
    assert torch.equal(bits, ref_bits)
    bits2 = torch.empty_like(bits)
    R.batchnorm_forward_train(x.float(), g, b, rm.clone(), rv.clone(), 0.1, 1e-3, relu=True, residual=res.float(),
                              bits_out=bits2)
    assert (bits2 != bits).float().mean() < 0.01  # fp32 vs bf16 rounding at the ReLU edge only
