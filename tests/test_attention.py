"""Attention / Transformer / beam search (reference specs: TS/nn/AttentionSpec, TransformerSpec,
SequenceBeamSearchSpec)."""
import math

import torch

from bigdl.nn import Attention, FeedForwardNetwork, SequenceBeamSearch, Transformer
from bigdl.nn.layers.attention import lower_triangle_bias, position_signal
from bigdl.utils.table import T


def test_attention_matches_manual():
    torch.manual_seed(0)
    att = Attention(8, 2, 1.0)  # rate 1.0 → keep everything (reference Dropout(1 - rate))
    x = torch.randn(2, 5, 8)
    y = torch.randn(2, 4, 8)
    bias = torch.zeros(2, 1, 1, 4)
    bias[1, ..., 3] = -1e9
    out = att.forward(T(x, y, bias))
    wq, wk, wv, wo = [p.detach() for p in att.parameters()[0]]

    def heads(t):
        return t.reshape(2, -1, 2, 4).transpose(1, 2)

    q = heads(x @ wq.t()) * 4 ** -0.5
    k = heads(y @ wk.t())
    v = heads(y @ wv.t())
    w = torch.softmax(q @ k.transpose(-1, -2) + bias, -1)
    ref = (w @ v).transpose(1, 2).reshape(2, 5, 8) @ wo.t()
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)
    gi = att.backward(T(x, y, bias), torch.ones_like(out))
    assert gi[1].shape == x.shape and gi[2].shape == y.shape
    assert all(g.abs().sum() > 0 for g in att.parameters()[1])


def test_ffn():
    torch.manual_seed(1)
    f = FeedForwardNetwork(6, 12, 1.0)
    x = torch.randn(3, 4, 6)
    w1, b1, w2, b2 = [p.detach() for p in f.parameters()[0]]
    torch.testing.assert_close(f.forward(x), torch.relu(x @ w1.t() + b1) @ w2.t() + b2, rtol=1e-5, atol=1e-5)


def test_position_signal_and_mask():
    s = position_signal(3, 4)
    inv = torch.tensor([1.0, 1e-4])
    t = torch.arange(3.0).unsqueeze(1) * inv
    torch.testing.assert_close(s, torch.cat([t.sin(), t.cos()], 1))
    m = lower_triangle_bias(3)[0, 0]
    assert m[0, 1] == -1e9 and m[1, 0] == 0 and m[2, 2] == 0


def test_transformer_lm_trains():
    torch.manual_seed(2)
    from bigdl.nn import Sequential, TimeDistributed, Linear, TimeDistributedCriterion, CrossEntropyCriterion
    from bigdl.optim import Adam
    from bigdl.optim.optimizer import LocalOptimizer
    from bigdl.dataset import MiniBatch
    V = 20
    model = Sequential().add(Transformer(V, 16, 2, 32, 2, 1.0, 1.0, 1.0)).add(TimeDistributed(Linear(16, V)))
    seq = torch.randint(1, V, (6, 8))
    x, y = seq.float(), ((seq % (V - 1)) + 1).float()
    crit = TimeDistributedCriterion(CrossEntropyCriterion(), size_average=True, dimension=2)
    opt = LocalOptimizer(model, [MiniBatch(x, y)], crit, Adam(learningrate=0.01))
    opt.prepare()
    l0 = float(opt.train_step(MiniBatch(x, y)))
    for _ in range(40):
        l = float(opt.train_step(MiniBatch(x, y)))
    assert l < 0.5 * l0


def test_incremental_decoding_matches_full_decoder():
    """Cached step-by-step decoding (symbols) == the full teacher-forced decoder."""
    torch.manual_seed(3)
    V, H = 30, 16
    bs = SequenceBeamSearch(V, 2, 0.6, 6, 3, 0, 2, H)
    tr = Transformer(V, H, 4, 32, 2, 1.0, 1.0, 1.0, with_share_weights_linear=True, transformer_type="Translation",
                     beam_search=bs)
    tr.evaluate()
    src = torch.randint(1, V, (2, 6)).float()
    tgt = torch.randint(1, V, (2, 6)).float()
    full = tr.forward(T(src, tgt))  # (2, 6, V) logits
    # encoder side as in _translate
    from bigdl.nn.layers.attention import PaddingMask
    mask = PaddingMask().forward(src)
    emb = tr._emb_seq.forward(src)
    enc = tr.encoderStack.forward(T(emb + position_signal(6, H), mask))
    ids = torch.cat([torch.zeros(2, 1), tgt], 1).long()
    cache = T()
    for j in range(1, 3):
        cache[f"layer_{j}_k"] = torch.empty(0)
        cache[f"layer_{j}_v"] = torch.empty(0)
    for i in range(6):
        logits, cache = tr.symbols(ids, i, 6, enc, mask, cache)
        torch.testing.assert_close(logits, full[:, i], rtol=1e-4, atol=1e-4)


def test_beam_search_prefers_high_prob_path():
    V = 5
    table = torch.full((V,), -10.0)

    def fn(ids, i, max_len, enc, bias, cache):
        n = ids.shape[0]
        logits = table.repeat(n, 1).clone()
        last = ids[:, -1]
        # token 3 then eos (2)
        logits[:, 2] = torch.where(last == 3, torch.tensor(5.0), torch.tensor(-10.0))
        logits[:, 2] = torch.where(last == 0, torch.tensor(-10.0), logits[:, 2])
        logits[:, 1] = torch.where(last == 0, torch.tensor(5.0), torch.tensor(-10.0))  # id 2 (1-based)
        return logits, cache

    bs = SequenceBeamSearch(V, 2, 0.6, 4, 3.0, 0, 0, 4).setLogitFn(fn)
    out = bs.forward(T(torch.zeros(1, 3, 4), torch.zeros(1, 1, 1, 3)))
    seq, scores = out[1], out[2]
    assert seq.shape[0] == 1 and seq.shape[1] == 2
    assert seq[0, 0, 1].item() == 2 and seq[0, 0, 2].item() == 3  # 1-based ids: 2 then eos 3
    assert math.isfinite(scores[0, 0].item())


def test_incremental_decoding_in_place_cache_matches_full_decoder():
    """The same step-by-step decoding on preallocated in-place KV caches (DecodeCache +
    ops.attention_decode) == the full teacher-forced decoder."""
    from bigdl.nn.layers.attention import DecodeCache, PaddingMask
    torch.manual_seed(3)
    V, H = 30, 16
    bs = SequenceBeamSearch(V, 2, 0.6, 6, 3, 0, 2, H)
    tr = Transformer(V, H, 4, 32, 2, 1.0, 1.0, 1.0, with_share_weights_linear=True, transformer_type="Translation",
                     beam_search=bs)
    tr.evaluate()
    src = torch.randint(1, V, (2, 6)).float()
    tgt = torch.randint(1, V, (2, 6)).float()
    full = tr.forward(T(src, tgt))
    mask = PaddingMask().forward(src)
    emb = tr._emb_seq.forward(src)
    enc = tr.encoderStack.forward(T(emb + position_signal(6, H), mask))
    ids = torch.cat([torch.zeros(2, 1), tgt], 1).long()
    cache = T()
    for j in range(1, 3):
        dc = DecodeCache(2, 3, H)  # deliberately short: exercises the in-place growth
        cache[f"layer_{j}_k"] = dc
        cache[f"layer_{j}_v"] = dc
    for i in range(6):
        logits, cache = tr.symbols(ids, i, 6, enc, mask, cache)
        torch.testing.assert_close(logits, full[:, i], rtol=1e-4, atol=1e-4)
    assert cache["layer_1_k"].length == 6


def test_beam_search_in_place_cache_matches_tensor_cache():
    from bigdl.nn.layers.attention import PaddingMask
    torch.manual_seed(5)
    V, H = 24, 16
    bs = SequenceBeamSearch(V, 3, 0.6, 7, 3, 0, 2, H)
    tr = Transformer(V, H, 4, 32, 2, 1.0, 1.0, 1.0, with_share_weights_linear=True, transformer_type="Translation",
                     beam_search=bs)
    tr.evaluate()
    src = torch.randint(1, V, (3, 5)).float()
    a = tr.forward(src)
    bs.inPlaceCache = False
    b = tr.forward(src)
    torch.testing.assert_close(a[1], b[1])
    torch.testing.assert_close(a[2], b[2], rtol=1e-4, atol=1e-4)


def test_attention_decode_reference_bias_order():
    """Reference semantics: keys are [new; cache] (newest first); a bias over keys is indexed in
    that order — the in-place cache (oldest first) reads it reversed."""
    from bigdl.ops import reference as R
    torch.manual_seed(0)
    rows, Lq, Hh, D, L = 2, 1, 2, 8, 5
    q = torch.randn(rows, Lq, Hh * D)
    kc = torch.randn(rows, 7, Hh * D)
    vc = torch.randn(rows, 7, Hh * D)
    bias = torch.randn(rows, 1, Lq, L)
    o = R.attention_decode(q, kc, vc, L, Hh, D, 0.3, bias, True)
    # explicit: newest-first keys with the bias as given
    k = kc[:, :L].flip(1)
    v = vc[:, :L].flip(1)
    qh = q.reshape(rows, Lq, Hh, D).transpose(1, 2)
    kh = k.reshape(rows, L, Hh, D).transpose(1, 2)
    vh = v.reshape(rows, L, Hh, D).transpose(1, 2)
    ref = torch.softmax(qh @ kh.transpose(-1, -2) * 0.3 + bias, -1) @ vh
    torch.testing.assert_close(o, ref.transpose(1, 2).reshape(rows, Lq, Hh * D))


def test_decode_cache_multi_position_append_bias_order():
    """Appends of more than one position keep the reference's per-call ``[new; cache]`` order
    (``DL/nn/Attention.scala:136-141``): with a key-dependent bias the in-place DecodeCache path equals
    the tensor-cache path when a call appends 2 positions."""
    from bigdl.nn.layers.attention import DecodeCache, Attention
    torch.manual_seed(11)
    H, nh = 16, 4
    att = Attention(H, nh, 0.0)
    att.evaluate()
    steps = [torch.randn(2, 2, H), torch.randn(2, 1, H), torch.randn(2, 3, H)]
    dc = DecodeCache(2, 2, H)
    c_inplace = T()
    c_inplace[f"{att.get_name()}_k"] = dc
    c_inplace[f"{att.get_name()}_v"] = dc
    c_tensor = T()
    c_tensor[f"{att.get_name()}_k"] = torch.empty(2, 0, H)
    c_tensor[f"{att.get_name()}_v"] = torch.empty(2, 0, H)
    L = 0
    for x in steps:
        L += x.shape[1]
        bias = torch.randn(2, 1, x.shape[1], L)  # key-dependent: order matters
        a = att.forward(T(x, x, T(bias, c_inplace)))
        b = att.forward(T(x, x, T(bias, c_tensor)))
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(dc.keys(), c_tensor[f"{att.get_name()}_k"])
