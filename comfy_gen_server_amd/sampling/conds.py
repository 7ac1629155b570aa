"""Per-key conditioning containers with batching rules (parity: ``comfy/conds.py:1-78``).

CONDRegular      — batch by concat along dim 0 (ADM ``y``...)
CONDNoiseShape   — area-cropped like the latent (``c_concat``)
CONDCrossAttn    — sequences of different length are concatenated by repeat-padding to their
                   LCM length, at most 4x the longest (``c_crossattn``)
CONDConstant     — must be equal to batch; passed through once
"""
from __future__ import annotations

import math

import torch


def repeat_to_batch_size(t: torch.Tensor, batch_size: int, dim: int = 0) -> torch.Tensor:
    n = t.shape[dim]
    if n > batch_size:
        return t.narrow(dim, 0, batch_size)
    if n < batch_size:
        reps = [1] * t.ndim
        reps[dim] = math.ceil(batch_size / n)
        return t.repeat(reps).narrow(dim, 0, batch_size)
    return t


class CONDRegular:
    def __init__(self, cond):
        self.cond = cond

    def _copy_with(self, cond):
        return self.__class__(cond)

    def process_cond(self, batch_size, device, **kwargs):
        return self._copy_with(repeat_to_batch_size(self.cond, batch_size).to(device))

    def can_concat(self, other):
        return self.cond.shape == other.cond.shape

    def concat(self, others):
        return torch.cat([self.cond] + [o.cond for o in others])


class CONDNoiseShape(CONDRegular):
    def process_cond(self, batch_size, device, area=None, **kwargs):
        data = self.cond
        if area is not None:
            h, w, y, x = area
            data = data[:, :, y:y + h, x:x + w]
        return self._copy_with(repeat_to_batch_size(data, batch_size).to(device))


class CONDCrossAttn(CONDRegular):
    def can_concat(self, other):
        a, b = self.cond.shape, other.cond.shape
        if a == b:
            return True
        if a[0] != b[0] or a[2] != b[2]:
            return False
        lcm = math.lcm(a[1], b[1])
        return lcm // min(a[1], b[1]) <= 4

    def concat(self, others):
        conds = [self.cond] + [o.cond for o in others]
        lcm = conds[0].shape[1]
        for c in conds[1:]:
            lcm = math.lcm(lcm, c.shape[1])
        out = [c.repeat(1, lcm // c.shape[1], 1) if c.shape[1] != lcm else c for c in conds]
        return torch.cat(out)


class CONDConstant(CONDRegular):
    def process_cond(self, batch_size, device, **kwargs):
        return self._copy_with(self.cond)

    def can_concat(self, other):
        return self.cond == other.cond

    def concat(self, others):
        return self.cond
