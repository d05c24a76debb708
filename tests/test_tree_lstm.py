"""BinaryTreeLSTM (``DL/nn/BinaryTreeLSTM.scala``) level-batched execution vs a node-by-node
recursive oracle written from the reference's leaf/composer equations (fp32, CPU)."""
import torch

from bigdl.nn import BinaryTreeLSTM, TensorTree
from bigdl.utils.table import Table

# the reference's doc example (BinaryTreeLSTM.scala:495-507) plus a second, smaller tree padded
TREE1 = [[11, 10, -1], [0, 0, 1], [0, 0, 2], [0, 0, 3], [0, 0, 4], [0, 0, 5], [0, 0, 6],
         [4, 5, 0], [6, 7, 0], [8, 9, 0], [2, 3, 0], [-1, -1, -1], [-1, -1, -1]]
TREE2 = [[2, 3, -1], [0, 0, 1], [4, 5, 0], [0, 0, 2], [0, 0, 3]] + [[-1, -1, -1]] * 8


def _oracle(m, x, trees):
    B, N = trees.shape[0], trees.shape[1]
    H = m.hiddenSize
    G = 5 if m.gateOutput else 4
    out = torch.zeros(B, N, H)

    def rec(b, tree, i):
        if tree.noChild(i):
            xi = x[b, tree.leafIndex(i) - 1]
            c = m.leaf_c_weight @ xi + m.leaf_c_bias
            h = torch.sigmoid(m.leaf_o_weight @ xi + m.leaf_o_bias) * torch.tanh(c) if m.gateOutput else torch.tanh(c)
        else:
            l, r = tree.children(i)[:2]
            lc, lh = rec(b, tree, l)
            rc, rh = rec(b, tree, r)
            g = (m.left_weight @ lh + m.left_bias + m.right_weight @ rh + m.right_bias).view(G, H)
            c = torch.sigmoid(g[0]) * torch.tanh(g[3]) + torch.sigmoid(g[1]) * lc + torch.sigmoid(g[2]) * rc
            h = torch.sigmoid(g[4]) * torch.tanh(c) if m.gateOutput else torch.tanh(c)
        out[b, i - 1] = h
        return c, h
    for b in range(B):
        t = TensorTree(trees[b])
        rec(b, t, t.getRoot())
    return out


def test_binary_tree_lstm_matches_recursive_oracle():
    torch.manual_seed(0)
    m = BinaryTreeLSTM(6, 5)
    trees = torch.tensor([TREE1, TREE2], dtype=torch.float32)
    x = torch.randn(2, 6, 6)
    y = m.forward(Table(x, trees))
    ref = _oracle(m, x, trees)
    assert y.shape == (2, 13, 5)
    assert torch.allclose(y, ref, atol=1e-6)


def test_binary_tree_lstm_backward_matches_autograd_oracle():
    torch.manual_seed(1)
    for gate in (True, False):
        m = BinaryTreeLSTM(4, 3, gate_output=gate)
        trees = torch.tensor([TREE1, TREE2], dtype=torch.float32)
        x = torch.randn(2, 6, 4)
        gy = torch.randn(2, 13, 3)
        m.zeroGradParameters()
        m.forward(Table(x, trees))
        gi = m.backward(Table(x, trees), gy)
        # oracle gradients through the recursive formulation
        names = [w for w, _ in m._param_slots]
        saved = {n: getattr(m, n) for n in names}
        leaves = {n: saved[n].detach().clone().requires_grad_(True) for n in names}
        for n in names:
            setattr(m, n, leaves[n])
        xr = x.clone().requires_grad_(True)
        (_oracle(m, xr, trees) * gy).sum().backward()
        for n in names:
            setattr(m, n, saved[n])
        assert torch.allclose(gi[1], xr.grad, atol=1e-5)
        for (w, g) in m._param_slots:
            assert torch.allclose(getattr(m, g), leaves[w].grad, atol=1e-5), w


def test_tensor_tree_helpers():
    t = TensorTree(torch.tensor(TREE1, dtype=torch.float32))
    assert t.getRoot() == 1 and t.hasChild(1) and t.noChild(2) and t.leafIndex(2) == 1
    assert t.isPadding(12) and t.exists(13) and not t.exists(14)


def test_tree_lstm_sentiment_trains():
    from bigdl.models.treelstm import TreeLSTMSentiment
    from bigdl.nn import TimeDistributedMaskCriterion, ClassNLLCriterion
    from bigdl.optim.validation import TreeNNAccuracy
    torch.manual_seed(2)
    model = TreeLSTMSentiment(torch.randn(20, 8), 6, 5, p=0.0)
    tokens = torch.randint(1, 21, (2, 6, 1)).float()
    trees = torch.tensor([TREE1, TREE2], dtype=torch.float32)
    labels = torch.randint(1, 6, (2, 13)).float()
    labels[1, 5:] = 0  # padding rows
    crit = TimeDistributedMaskCriterion(ClassNLLCriterion(padding_value=0), padding_value=0)
    x = Table(tokens, trees)
    losses = []
    for _ in range(30):
        model.zeroGradParameters()
        out = model.forward(x)
        losses.append(float(crit.forward(out, labels)))
        model.backward(x, crit.backward(out, labels))
        w, g = model.getParameters()
        w.add_(g, alpha=-0.5)
    assert losses[-1] < losses[0] * 0.9
    r = TreeNNAccuracy()(model.forward(x), labels)
    assert r.result()[1] == 2
