"""Weight regularisers applied inside ``accGradParameters`` (``DL/optim/Regularizer.scala:30-193``)."""
from __future__ import annotations

import torch


class Regularizer:
    SCALA_PACKAGE = "com.intel.analytics.bigdl.optim"

    def __init__(self):
        self.isRegualrized = True

    def accRegularization(self, parameter: torch.Tensor, gradParameter: torch.Tensor, scale: float):
        raise NotImplementedError

    def disable(self):
        self.isRegualrized = False
        return self

    def enable(self):
        self.isRegualrized = True
        return self


class L1L2Regularizer(Regularizer):
    def __init__(self, l1, l2, bigdl_type="float"):
        super().__init__()
        self.l1, self.l2 = l1, l2

    #: set by an optimizer that folded this L2 term into its fused update kernel (per-element decay)
    _folded = False

    def accRegularization(self, p, g, scale):
        if not self.isRegualrized or self._folded:
            return
        with torch.no_grad():
            if self.l1 != 0:
                g.add_(torch.sign(p), alpha=self.l1 * scale)
            if self.l2 != 0:
                g.add_(p, alpha=self.l2 * scale)


class L1Regularizer(L1L2Regularizer):
    def __init__(self, l1, bigdl_type="float"):
        super().__init__(l1, 0.0)


class L2Regularizer(L1L2Regularizer):
    def __init__(self, l2, bigdl_type="float"):
        super().__init__(0.0, l2)
