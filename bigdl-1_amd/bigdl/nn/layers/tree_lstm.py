"""Tree-structured LSTMs: ``TreeLSTM`` (base), ``BinaryTreeLSTM`` (constituency Tree-LSTM) and the
``TensorTree`` tree encoding.

Reference: ``DL/nn/TreeLSTM.scala`` and ``DL/nn/BinaryTreeLSTM.scala:40-573`` — leaf module
``c = W_c x``, ``h = σ(W_o x) ⊙ tanh(c)`` (or ``tanh(c)`` without an output gate); composer over the
(left, right) children with one ``Linear(H,H)`` per child per gate:
``i, f_l, f_r, o = σ(L(lh) + R(rh))``, ``u = tanh(L(lh) + R(rh))``,
``c = i⊙u + f_l⊙lc + f_r⊙rc``, ``h = o⊙tanh(c)``.  Input ``Table(embeddings (B, leaves, in),
trees (B, nodes, k+1))``; output ``(B, nodes, H)`` = every node's h (zeros for padding rows).

Execution differs from the reference by design: instead of cloning one cell module per tree node
and recursing node by node (O(nodes) tiny GEMMs), nodes of ALL trees in the batch are grouped by
height and each height level runs as one batched GEMM + fused gate math — O(tree height) kernel
launches for the whole batch, which is what keeps the MFMA units busy on a GPU.  Backward is the
level-reversed adjoint of the same computation.
"""
from __future__ import annotations

import math
from typing import List, Tuple

import torch

from ..abstractnn import AutogradModule
from ..initialization_method import RandomUniform, VariableFormats
from ...utils.table import Table


class TensorTree:
    """Row ``i`` (1-based) of ``content`` is node ``i``: its child node numbers in every column but
    the last; the last column is the leaf number (leaves), ``-1`` (root) or ``0``.  Padding rows are
    all ``-1`` (``BinaryTreeLSTM.scala:477-573``)."""

    def __init__(self, content: torch.Tensor):
        if content.dim() != 2:
            raise ValueError(f"TensorTree content must be 2-D, got {content.dim()}-D")
        self.content = content

    @property
    def size(self):
        return list(self.content.shape)

    @property
    def nodeNumber(self) -> int:
        return self.content.shape[0]

    def children(self, index: int) -> List[int]:
        return [int(v) for v in self.content[index - 1].tolist()]

    def addChild(self, parent: int, child):
        row = self.content[parent - 1]
        for i in range(row.numel() - 1):
            if row[i] == 0:
                row[i] = child
                return

    def markAsRoot(self, index: int):
        self.content[index - 1, -1] = -1

    def getRoot(self) -> int:
        for i in range(self.nodeNumber):
            if int(self.content[i, -1]) == -1 and int(self.content[i, 0]) != -1:
                return i + 1
        for i in range(self.nodeNumber):
            if int(self.content[i, -1]) == -1:
                return i + 1
        raise RuntimeError("There is no root in the tensor tree")

    def markAsLeaf(self, index: int, leaf_index: int):
        self.content[index - 1, -1] = leaf_index

    def leafIndex(self, index: int) -> int:
        return int(self.content[index - 1, -1])

    def hasChild(self, index: int) -> bool:
        return int(self.content[index - 1, 0]) > 0

    def noChild(self, index: int) -> bool:
        return int(self.content[index - 1, 0]) == 0

    def exists(self, index: int) -> bool:
        return 1 <= index <= self.nodeNumber

    def isPadding(self, index: int) -> bool:
        return int(self.content[index - 1, 0]) == -1


class TreeLSTM(AutogradModule):
    """Base of the tree LSTMs (``TreeLSTM.scala``): ``inputSize``, ``hiddenSize`` and the zero
    state used for missing children."""

    def __init__(self, input_size: int, hidden_size: int = 150):
        super().__init__()
        self.inputSize, self.hiddenSize = input_size, hidden_size

    def memZero(self, device, dtype=torch.float32):
        return torch.zeros(self.hiddenSize, device=device, dtype=dtype)


def _schedule(trees: torch.Tensor) -> Tuple[list, list]:
    """Host-side plan: (leaf list, per-height composer lists) of flat node ids ``b*N + (i-1)``."""
    t = trees.detach().to("cpu", torch.int64)
    B, N, K = t.shape
    leaves = []          # (flat node, batch index, 1-based leaf number)
    levels: List[list] = []
    for b in range(B):
        rows = t[b].tolist()
        height = {}

        def h_of(i):  # 1-based node
            if i in height:
                return height[i]
            r = rows[i - 1]
            if r[0] == 0:
                height[i] = 0
            else:
                kids = [c for c in r[:-1] if c > 0]
                height[i] = 1 + max(h_of(c) for c in kids)
            return height[i]
        for i in range(1, N + 1):
            r = rows[i - 1]
            if r[0] == -1:
                continue  # padding
            hh = h_of(i)
            if hh == 0:
                leaves.append((b * N + i - 1, b, r[-1]))
            else:
                while len(levels) < hh:
                    levels.append([])
                kids = [c for c in r[:-1] if c > 0]
                if len(kids) != 2:
                    raise ValueError(f"BinaryTreeLSTM: node {i} of tree {b} has {len(kids)} children")
                levels[hh - 1].append((b * N + i - 1, b * N + kids[0] - 1, b * N + kids[1] - 1))
    return leaves, levels


class BinaryTreeLSTM(TreeLSTM):
    def __init__(self, input_size: int, hidden_size: int, gate_output: bool = True, with_graph: bool = True,
                 bigdl_type="float"):
        super().__init__(input_size, hidden_size)
        self.gateOutput, self.withGraph = gate_output, with_graph
        H = hidden_size
        G = 5 if gate_output else 4   # i, lf, rf, update[, o]
        self._G = G
        self.register_parameter("leaf_c_weight", torch.zeros(H, input_size))
        self.register_parameter("leaf_c_bias", torch.zeros(H))
        if gate_output:
            self.register_parameter("leaf_o_weight", torch.zeros(H, input_size))
            self.register_parameter("leaf_o_bias", torch.zeros(H))
        self.register_parameter("left_weight", torch.zeros(G * H, H))
        self.register_parameter("left_bias", torch.zeros(G * H))
        self.register_parameter("right_weight", torch.zeros(G * H, H))
        self.register_parameter("right_bias", torch.zeros(G * H))
        self.reset()

    def reset(self):
        for w, _ in self._param_slots:
            t = getattr(self, w)
            fan_in = self.inputSize if w.startswith("leaf") else self.hiddenSize
            stdv = 1.0 / math.sqrt(fan_in)   # Linear's default init, per gate Linear
            RandomUniform(-stdv, stdv).init(t, VariableFormats.ONE_D if t.dim() == 1 else VariableFormats.OUT_IN)
        self.zeroGradParameters()
        return self

    def _forward(self, input):
        x, trees = input[1], input[2]
        B, L, _ = x.shape
        N = trees.shape[1]
        H = self.hiddenSize
        leaves, levels = _schedule(trees)
        dev, dt = x.device, x.dtype
        C = torch.zeros(B * N, H, device=dev, dtype=dt)
        Hs = torch.zeros(B * N, H, device=dev, dtype=dt)
        if leaves:
            node_idx = torch.tensor([l[0] for l in leaves], device=dev)
            in_rows = torch.tensor([l[1] * L + (l[2] - 1) for l in leaves], device=dev)
            xl = x.reshape(B * L, -1).index_select(0, in_rows)
            c = torch.nn.functional.linear(xl, self.P("leaf_c_weight").to(dt), self.P("leaf_c_bias").to(dt))
            if self.gateOutput:
                o = torch.sigmoid(torch.nn.functional.linear(xl, self.P("leaf_o_weight").to(dt),
                                                             self.P("leaf_o_bias").to(dt)))
                h = o * torch.tanh(c)
            else:
                h = torch.tanh(c)
            C = C.index_copy(0, node_idx, c)
            Hs = Hs.index_copy(0, node_idx, h)
        Wl, bl = self.P("left_weight").to(dt), self.P("left_bias").to(dt)
        Wr, br = self.P("right_weight").to(dt), self.P("right_bias").to(dt)
        for lvl in levels:
            idx = torch.tensor(lvl, device=dev)
            me, lk, rk = idx[:, 0], idx[:, 1], idx[:, 2]
            lc, lh = C.index_select(0, lk), Hs.index_select(0, lk)
            rc, rh = C.index_select(0, rk), Hs.index_select(0, rk)
            gates = torch.nn.functional.linear(lh, Wl, bl) + torch.nn.functional.linear(rh, Wr, br)
            g = gates.view(-1, self._G, H)
            i, lf, rf = torch.sigmoid(g[:, 0]), torch.sigmoid(g[:, 1]), torch.sigmoid(g[:, 2])
            u = torch.tanh(g[:, 3])
            c = i * u + lf * lc + rf * rc
            h = torch.sigmoid(g[:, 4]) * torch.tanh(c) if self.gateOutput else torch.tanh(c)
            C = C.index_copy(0, me, c)
            Hs = Hs.index_copy(0, me, h)
        return Hs.view(B, N, H)

    def updateGradInput(self, input, gradOutput):
        gi = super().updateGradInput(input, gradOutput)
        if isinstance(gi, Table) and gi.get(2) is None:
            gi[2] = torch.zeros_like(input[2])
        return gi

    def __repr__(self):
        return f"{self.get_name()}({self.inputSize}, {self.hiddenSize}, gateOutput={self.gateOutput})"
