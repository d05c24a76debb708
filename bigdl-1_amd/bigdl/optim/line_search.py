"""Line searches for LBFGS (``DL/optim/LineSearch.scala``: ``LineSearch`` trait and
``LswolfeLineSearch``, the torch-optim ``lswolfe``): a strong-Wolfe search along a descent
direction with cubic interpolation and a zoom phase.

``apply(opfunc, x, t, d, f, g, gtd, options)`` evaluates ``opfunc(x + t·d)`` and returns
``(f_new, g_new, x_new, t, n_evals)``; ``x`` is restored before returning (the caller applies the
step).  Defaults as the reference: c1 = 1e-4, c2 = 0.9, tolX = 1e-9, maxIter = 20.
"""
from __future__ import annotations

import math
from typing import Callable

import torch


def _cubic_min(x1, f1, g1, x2, f2, g2, lo=None, hi=None):
    """Minimiser of the cubic through (x1, f1, g1), (x2, f2, g2), clamped to [lo, hi]."""
    lo, hi = (min(x1, x2), max(x1, x2)) if lo is None else (lo, hi)
    d1 = g1 + g2 - 3 * (f1 - f2) / (x1 - x2)
    sq = d1 * d1 - g1 * g2
    if sq >= 0:
        d2 = math.sqrt(sq)
        if x1 > x2:
            d2 = -d2
        t = x2 - (x2 - x1) * ((g2 + d2 - d1) / (g2 - g1 + 2 * d2))
        return min(max(t, lo), hi)
    return (lo + hi) / 2.0


class LineSearch:
    def apply(self, opfunc: Callable, x: torch.Tensor, t: float, d: torch.Tensor, f: float, g: torch.Tensor,
              gtd: float, options=None):
        raise NotImplementedError


class LswolfeLineSearch(LineSearch):
    def __init__(self, c1: float = 1e-4, c2: float = 0.9, tol_x: float = 1e-9, max_iter: int = 20):
        self.c1, self.c2, self.tolX, self.maxIter = c1, c2, tol_x, max_iter

    def apply(self, opfunc, x, t, d, f, g, gtd, options=None):
        x0 = x.clone()

        def ev(step):
            x.copy_(x0).add_(d, alpha=step)
            fx, gx = opfunc(x)
            return float(fx), gx.clone(), float((gx * d).sum())
        d_norm = float(d.abs().max())
        f_new, g_new, gtd_new = ev(t)
        n = 1
        t_prev, f_prev, g_prev, gtd_prev = 0.0, f, g.clone(), gtd
        done = False
        it = 0
        bracket = bracket_f = bracket_g = bracket_gtd = None
        while it < self.maxIter:
            if f_new > f + self.c1 * t * gtd or (it > 1 and f_new >= f_prev):
                bracket, bracket_f = [t_prev, t], [f_prev, f_new]
                bracket_g, bracket_gtd = [g_prev, g_new], [gtd_prev, gtd_new]
                break
            if abs(gtd_new) <= -self.c2 * gtd:
                bracket, bracket_f, bracket_g = [t], [f_new], [g_new]
                done = True
                break
            if gtd_new >= 0:
                bracket, bracket_f = [t_prev, t], [f_prev, f_new]
                bracket_g, bracket_gtd = [g_prev, g_new], [gtd_prev, gtd_new]
                break
            min_step = t + 0.01 * (t - t_prev)
            max_step = t * 10
            tmp = t
            t = _cubic_min(t_prev, f_prev, gtd_prev, t, f_new, gtd_new, min_step, max_step)
            t_prev, f_prev, g_prev, gtd_prev = tmp, f_new, g_new, gtd_new
            f_new, g_new, gtd_new = ev(t)
            n += 1
            it += 1
        if it == self.maxIter:
            bracket, bracket_f, bracket_g = [0.0, t], [f, f_new], [g, g_new]
            bracket_gtd = [gtd, gtd_new]
        # zoom
        insuf = False
        lo, hi = (0, 1) if len(bracket) == 2 and bracket_f[0] <= bracket_f[-1] else (1, 0)
        while not done and it < self.maxIter and len(bracket) == 2:
            if abs(bracket[1] - bracket[0]) * d_norm < self.tolX:
                break
            t = _cubic_min(bracket[0], bracket_f[0], bracket_gtd[0], bracket[1], bracket_f[1], bracket_gtd[1])
            blo, bhi = min(bracket), max(bracket)
            eps = 0.1 * (bhi - blo)
            if min(bhi - t, t - blo) < eps:
                if insuf or t >= bhi or t <= blo:
                    t = bhi - eps if abs(t - bhi) < abs(t - blo) else blo + eps
                    insuf = False
                else:
                    insuf = True
            else:
                insuf = False
            f_new, g_new, gtd_new = ev(t)
            n += 1
            it += 1
            if f_new > f + self.c1 * t * gtd or f_new >= bracket_f[lo]:
                bracket[hi], bracket_f[hi], bracket_g[hi], bracket_gtd[hi] = t, f_new, g_new, gtd_new
                lo, hi = (0, 1) if bracket_f[0] <= bracket_f[1] else (1, 0)
            else:
                if abs(gtd_new) <= -self.c2 * gtd:
                    done = True
                elif gtd_new * (bracket[hi] - bracket[lo]) >= 0:
                    bracket[hi], bracket_f[hi], bracket_g[hi], bracket_gtd[hi] = (
                        bracket[lo], bracket_f[lo], bracket_g[lo], bracket_gtd[lo])
                bracket[lo], bracket_f[lo], bracket_g[lo], bracket_gtd[lo] = t, f_new, g_new, gtd_new
        t = bracket[lo] if len(bracket) == 2 else bracket[0]
        f_new = bracket_f[lo] if len(bracket) == 2 else bracket_f[0]
        g_new = bracket_g[lo] if len(bracket) == 2 else bracket_g[0]
        x.copy_(x0)
        return f_new, g_new, x0.add(d, alpha=t), t, n
