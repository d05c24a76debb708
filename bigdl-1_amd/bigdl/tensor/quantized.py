"""int8 tensor with per-window symmetric scales (``DL/tensor/QuantizedTensor.scala:26``; the
quantisation math of ``DL/nn/quantized/Quantization.scala:26-180``: q = round(v / max|window| ·
127)).  Used by ``bigdl.nn.quantized``."""
from __future__ import annotations

import torch


class QuantizedTensor:
    def __init__(self, q: torch.Tensor, scale: torch.Tensor, axis: int = 0):
        self.q = q  # int8
        self.scale = scale  # fp32 per window: max|v|/127
        self.axis = axis

    @staticmethod
    def quantize(v: torch.Tensor, axis: int = 0) -> "QuantizedTensor":
        vf = v.float()
        red = [d for d in range(vf.dim()) if d != axis]
        amax = vf.abs().amax(dim=red, keepdim=True) if red else vf.abs()
        scale = (amax / 127.0).clamp_min(1e-12)
        q = torch.round(vf / scale).clamp(-127, 127).to(torch.int8)
        return QuantizedTensor(q, scale.reshape(-1), axis)

    def dequantize(self) -> torch.Tensor:
        shape = [1] * self.q.dim()
        shape[self.axis] = -1
        return self.q.float() * self.scale.view(shape)

    def size(self):
        return list(self.q.shape)

    def __repr__(self):
        return f"QuantizedTensor(shape={tuple(self.q.shape)})"
