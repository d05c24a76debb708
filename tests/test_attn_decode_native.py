"""Decode attention kernel (ops/csrc/attn_decode.hip) against the fp32 PyTorch reference of the same
bf16 operands: head dims 32/64/96/128/256, cache lengths around the 64-key tile and the 4-wave split,
one and two new queries, broadcast additive bias in the reference's newest-first order; and a GPU
Transformer beam search on in-place caches that runs no torch attention (no fallback recorded)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"


def _native():
    from bigdl.ops import native_status
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert native_status()["loaded"]
    from bigdl.ops import native_ops as NO
    return NO


@pytest.mark.parametrize("D", [32, 64, 96, 128, 256])
@pytest.mark.parametrize("L", [1, 5, 64, 65, 257])
@pytest.mark.parametrize("Lq", [1, 2])
def test_attention_decode_matches_fp32(D, L, Lq):
    NO = _native()
    from bigdl.ops import reference as R
    torch.manual_seed(D + L + Lq)
    rows, Hh, Lmax = 6, 3, 300
    H = Hh * D
    q = torch.randn(rows, Lq, H, device=dev).bfloat16()
    kc = torch.randn(rows, Lmax, H, device=dev).bfloat16()
    vc = torch.randn(rows, Lmax, H, device=dev).bfloat16()
    for bias in (None, torch.randn(rows, 1, Lq, L, device=dev), torch.randn(1, Hh, 1, L, device=dev)):
        o = NO.attention_decode(q, kc, vc, L, Hh, D, D ** -0.5, bias, True)
        assert o is not NotImplemented
        ref = R.attention_decode(q.float(), kc.float(), vc.float(), L, Hh, D, D ** -0.5, bias, True)
        torch.testing.assert_close(o.float(), ref, rtol=2e-2, atol=2e-2)


def test_attention_decode_masked_bias():
    NO = _native()
    from bigdl.ops import reference as R
    rows, Hh, D, L = 2, 2, 64, 70
    q = torch.randn(rows, 1, Hh * D, device=dev).bfloat16()
    kc = torch.randn(rows, 80, Hh * D, device=dev).bfloat16()
    vc = torch.randn(rows, 80, Hh * D, device=dev).bfloat16()
    bias = torch.zeros(rows, 1, 1, L, device=dev)
    bias[0, ..., :66] = -1e9  # row 0: only 4 keys live (newest-first order: the 4 oldest positions)
    o = NO.attention_decode(q, kc, vc, L, Hh, D, 0.125, bias, True)
    ref = R.attention_decode(q.float(), kc.float(), vc.float(), L, Hh, D, 0.125, bias, True)
    torch.testing.assert_close(o.float(), ref, rtol=2e-2, atol=2e-2)


def test_transformer_beam_search_gpu_in_place_cache_no_fallback():
    _native()
    from bigdl.ops import fallback_counts, reset_fallbacks
    from bigdl.nn.layers.attention import Transformer, SequenceBeamSearch
    from bigdl.utils.table import T
    torch.manual_seed(2)
    V, H = 40, 128
    bs = SequenceBeamSearch(V, 4, 0.6, 8, 3, 0, 2, H)
    tr = Transformer(V, H, 2, 256, 2, 1.0, 1.0, 1.0, with_share_weights_linear=True, transformer_type="Translation",
                     beam_search=bs)
    tr.evaluate()
    src = torch.randint(1, V, (3, 7)).float()
    cpu = tr.forward(src)
    trg = tr.cuda()
    reset_fallbacks()
    out = trg.forward(src.cuda())
    fb = {k: v for k, v in fallback_counts().items() if "attention" in k[0]}
    assert not fb, fb
    assert out[1].shape == cpu[1].shape
    # bf16 decoding can legitimately pick a different beam where two scores tie within rounding:
    # the best hypothesis' score must agree
    best = lambda t: t.float().cpu().reshape(t.shape[0], -1)[:, 0]  # noqa: E731 - [B] or [B, beam]
    torch.testing.assert_close(best(out[2]), best(cpu[2]), rtol=5e-2, atol=5e-2)
