"""Embeddings: ``LookupTable`` (``DL/nn/LookupTable.scala``: 1-based indices, gather forward at
:170, scatter-add accGrad at :204, optional maxNorm renorm at :120-150, paddingValue rows get no
gradient, N(0,1) init) and ``LookupTableSparse`` (``LookupTableSparse.scala``: bag-of-ids with
sum/mean/sqrtn combiners)."""
from __future__ import annotations

import torch

from ... import ops
from ..abstractnn import TensorModule
from ...utils.table import Table
from ...utils import acc_float

DOUBLEMAX = 1.7976931348623157e308


class LookupTable(TensorModule):
    def __init__(self, n_index, n_output, padding_value=0.0, max_norm=DOUBLEMAX, norm_type=2.0,
                 should_scale_grad_by_freq=False, wRegularizer=None, mask_zero=False, bigdl_type="float"):
        super().__init__()
        self.nIndex, self.nOutput = n_index, n_output
        self.maskZero = mask_zero
        self.paddingValue = padding_value
        self.maxNorm, self.normType = max_norm, norm_type
        self.shouldScaleGradByFreq = should_scale_grad_by_freq
        self.wRegularizer = wRegularizer
        self.register_parameter("weight", torch.randn(n_index, n_output))

    def reset(self):
        from ...utils.random import RNG
        with torch.no_grad():
            self.weight.copy_(RNG.normal_tensor(tuple(self.weight.shape)).to(self.weight.device))
        return self

    def _renorm(self, idx):
        if self.maxNorm >= DOUBLEMAX:
            return
        with torch.no_grad():
            rows = torch.unique(idx.long().reshape(-1) - 1)
            rows = rows[(rows >= 0) & (rows < self.nIndex)]
            w = self.weight[rows]
            n = w.norm(p=self.normType, dim=1, keepdim=True)
            scale = torch.where(n > self.maxNorm, self.maxNorm / (n + 1e-7), torch.ones_like(n))
            self.weight[rows] = w * scale

    def updateOutput(self, input):
        if self.maskZero and self.paddingValue != 0:
            with torch.no_grad():
                self.weight[int(self.paddingValue) - 1].zero_()
        self._renorm(input)
        w = self.cw("weight")
        y = ops.embedding_forward(w, input, self.paddingValue, self.maskZero)
        if self.maskZero:
            y = y * (input != self.paddingValue).unsqueeze(-1).to(y.dtype)
        return y

    def updateGradInput(self, input, gradOutput):
        return torch.zeros_like(input, dtype=torch.float32)

    def accGradParameters(self, input, gradOutput):
        scale = self.scale_w
        if self.shouldScaleGradByFreq:
            idx = input.long().reshape(-1)
            uniq, counts = torch.unique(idx, return_counts=True)
            freq = torch.zeros(self.nIndex + 1, device=idx.device)
            freq[uniq] = acc_float(counts)
            g = gradOutput.reshape(idx.numel(), -1) / freq[idx].unsqueeze(1)
            ops.embedding_backward(self.gradWeight, input, g, scale, self.paddingValue)
        else:
            ops.embedding_backward(self.gradWeight, input, gradOutput, scale, self.paddingValue)
        if self.wRegularizer is not None and scale != 0:
            self.wRegularizer.accRegularization(self.weight, self.gradWeight, scale)


class LookupTableSparse(TensorModule):
    """Input Table(ids (sparse or dense N×L, 1-based), optional weights) → combined embedding."""

    def __init__(self, n_index, n_output, combiner="sum", max_norm=-1.0, wRegularizer=None, bigdl_type="float"):
        super().__init__()
        self.nIndex, self.nOutput, self.combiner, self.maxNorm = n_index, n_output, combiner, max_norm
        self.register_parameter("weight", torch.randn(n_index, n_output))

    def _dense(self, input):
        ids = input[1] if isinstance(input, Table) else input
        wts = input[2] if isinstance(input, Table) and input.length() > 1 else None
        if ids.is_sparse:
            ids = ids.coalesce()
            rows = ids.indices()[0]
            vals = ids.values().long()
            w = wts.coalesce().values().float() if wts is not None else torch.ones_like(vals, dtype=torch.float32)
            n = ids.shape[0]
        else:
            n = ids.shape[0]
            rows = torch.arange(n, device=ids.device).repeat_interleave(ids.shape[1])
            vals = ids.reshape(-1).long()
            w = wts.reshape(-1).float() if wts is not None else torch.ones_like(vals, dtype=torch.float32)
            keep = vals > 0
            rows, vals, w = rows[keep], vals[keep], w[keep]
        return n, rows, vals - 1, w

    def updateOutput(self, input):
        n, rows, cols, w = self._dense(input)
        emb = self.weight[cols]
        if self.maxNorm > 0:
            nn_ = emb.norm(dim=1, keepdim=True)
            emb = emb * torch.where(nn_ > self.maxNorm, self.maxNorm / nn_, torch.ones_like(nn_))
        out = torch.zeros(n, self.nOutput, device=emb.device)
        out.index_add_(0, rows, emb * w.unsqueeze(1))
        if self.combiner in ("mean", "sqrtn"):
            den = torch.zeros(n, device=emb.device).index_add_(0, rows, w if self.combiner == "mean" else w * w)
            den = den if self.combiner == "mean" else den.sqrt()
            out = out / den.clamp_min(1e-12).unsqueeze(1)
        self._cache = (n, rows, cols, w)
        return out

    def updateGradInput(self, input, gradOutput):
        return Table(torch.zeros(1), torch.zeros(1)) if isinstance(input, Table) else torch.zeros(1)

    def accGradParameters(self, input, gradOutput):
        n, rows, cols, w = self._cache
        g = gradOutput[rows] * w.unsqueeze(1)
        if self.combiner in ("mean", "sqrtn"):
            den = torch.zeros(n, device=g.device).index_add_(0, rows, w if self.combiner == "mean" else w * w)
            den = den if self.combiner == "mean" else den.sqrt()
            g = g / den.clamp_min(1e-12)[rows].unsqueeze(1)
        self.gradWeight.index_add_(0, cols, g * self.scale_w)
