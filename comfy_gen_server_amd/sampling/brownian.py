"""Reproducible Brownian-motion noise for SDE samplers (replaces torchsde.BrownianTree used at
``comfy/k_diffusion/sampling.py:64-123``).

A virtual Brownian tree (Li et al. 2020): W over [t0, t1] is defined by recursive midpoint
bisection, the midpoint of each dyadic interval drawn from the Brownian bridge with a
counter-based seed (seed, depth, index). Any query W(t) is reproducible from the seed alone, so
``W(b) - W(a)`` is consistent across calls, samplers and devices. Draws use a Philox
``torch.Generator`` on the requested device (``cpu=False`` -> on the GPU, the ``*_gpu`` samplers).
"""
from __future__ import annotations

import math

import torch


class VirtualBrownianTree:
    def __init__(self, shape, t0: float, t1: float, seed: int, device, dtype, tol: float = 1e-4, max_depth: int = 24):
        self.shape = tuple(shape)
        self.t0, self.t1 = float(t0), float(t1)
        self.seed = int(seed) & 0x7FFFFFFF
        self.device = device
        self.dtype = dtype
        self.tol = tol
        self.max_depth = max_depth
        self._cache = {}
        self.w1 = self._normal(0, 0) * math.sqrt(self.t1 - self.t0)

    def _normal(self, depth, index):
        g = torch.Generator(device=self.device)
        g.manual_seed((self.seed * 1000003 + depth * 7919 + index * 104729) & 0x7FFFFFFFFFFFFFFF)
        return torch.randn(self.shape, generator=g, device=self.device, dtype=self.dtype)

    def __call__(self, t: float) -> torch.Tensor:
        t = min(max(float(t), self.t0), self.t1)
        key = round(t, 12)
        if key in self._cache:
            return self._cache[key]
        a, b = self.t0, self.t1
        wa = torch.zeros(self.shape, device=self.device, dtype=self.dtype)
        wb = self.w1
        idx = 0
        depth = 0
        while (b - a) > self.tol and depth < self.max_depth:
            m = 0.5 * (a + b)
            # Brownian bridge midpoint: mean (wa+wb)/2, var (b-a)/4
            wm = 0.5 * (wa + wb) + self._normal(depth + 1, idx) * math.sqrt((b - a) / 4.0)
            if t <= m:
                b, wb = m, wm
                idx = 2 * idx
            else:
                a, wa = m, wm
                idx = 2 * idx + 1
            depth += 1
        # linear interpolation inside the final (tiny) interval
        w = wa + (wb - wa) * ((t - a) / (b - a) if b > a else 0.0)
        if len(self._cache) > 256:
            self._cache.clear()
        self._cache[key] = w
        return w


class BrownianTreeNoiseSampler:
    """noise(sigma, sigma_next) = (W(t1) - W(t0)) / sqrt(|t1 - t0|), t = transform(sigma)."""

    def __init__(self, x, sigma_min, sigma_max, seed=None, transform=lambda v: v, cpu=False):
        self.transform = transform
        t0, t1 = float(transform(float(sigma_min))), float(transform(float(sigma_max)))
        self.sign = 1.0 if t0 < t1 else -1.0
        lo, hi = min(t0, t1), max(t0, t1)
        if seed is None:
            seed = int(torch.randint(0, 2 ** 31 - 1, []).item())
        dev = torch.device("cpu") if cpu else x.device
        seeds = seed if isinstance(seed, (list, tuple)) else [seed]
        shape = x.shape[1:] if len(seeds) > 1 else x.shape
        self.batched = len(seeds) > 1
        self.trees = [VirtualBrownianTree(shape, lo, hi, s, dev, torch.float32) for s in seeds]
        self.out_device = x.device
        self.out_dtype = x.dtype

    def __call__(self, sigma, sigma_next):
        t0, t1 = float(self.transform(float(sigma))), float(self.transform(float(sigma_next)))
        sign = 1.0 if t0 < t1 else -1.0
        a, b = min(t0, t1), max(t0, t1)
        ws = [tr(b) - tr(a) for tr in self.trees]
        w = torch.stack(ws) if self.batched else ws[0]
        w = w * (self.sign * sign)
        return (w / math.sqrt(max(abs(t1 - t0), 1e-12))).to(self.out_device, self.out_dtype)
