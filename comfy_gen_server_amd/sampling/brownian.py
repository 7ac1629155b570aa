"""Reproducible Brownian-motion noise for SDE samplers (replaces torchsde.BrownianTree used at
``comfy/k_diffusion/sampling.py:64-123``; SURVEY §2.3 "torchsde -> device Brownian sampler").

A virtual Brownian tree (Li et al. 2020) per image: W over [t0, t1] is defined by recursive
midpoint bisection, the midpoint of each dyadic interval drawn from the Brownian bridge with a
counter-based Philox draw keyed by (seed, global image index, tree node). Any query W(t) is
reproducible from the key alone, so ``W(b) - W(a)`` is consistent across calls, samplers, devices
and data-parallel rank splits.

Each query is ONE kernel launch (``cgs_brownian_increment``): every thread walks the ~log2(T/tol)
levels of the tree for its 4 elements in registers, for both interval ends — no generator objects,
no per-level full-tensor temporaries. On the CPU the bit-exact torch mirror (``rng.py``) runs.
"""
from __future__ import annotations

import math

import torch

from .. import ops


class BrownianTreeNoiseSampler:
    """noise(sigma, sigma_next) = (W(t1) - W(t0)) / sqrt(|t1 - t0|), t = transform(sigma).

    ``seed``: int (one tree per image, keyed by its global index ``inds[b]``), or a list of ints
    (reference-style explicit per-image seeds: image b uses key (seed[b], 0)). ``cpu`` is accepted
    for API parity; results do not depend on the device."""

    def __init__(self, x, sigma_min, sigma_max, seed=None, transform=lambda v: v, cpu=False, inds=None,
                 tol: float = 1e-4, max_depth: int = 24):
        self.transform = transform
        t0, t1 = float(transform(float(sigma_min))), float(transform(float(sigma_max)))
        self.sign = 1.0 if t0 < t1 else -1.0
        self.lo, self.hi = min(t0, t1), max(t0, t1)
        if seed is None:
            seed = int(torch.randint(0, 2 ** 31 - 1, []).item())
        self.shape = tuple(x.shape)
        self.out_device, self.out_dtype = x.device, x.dtype
        self.tol, self.max_depth = tol, max_depth
        if isinstance(seed, (list, tuple)):
            self.keys = [(int(s), [0]) for s in seed]
        else:
            ids = list(range(x.shape[0])) if inds is None else [int(i) for i in inds]
            self.keys = [(int(seed), ids)]

    def __call__(self, sigma, sigma_next):
        t0, t1 = float(self.transform(float(sigma))), float(self.transform(float(sigma_next)))
        sign = 1.0 if t0 < t1 else -1.0
        a, b = min(max(min(t0, t1), self.lo), self.hi), min(max(max(t0, t1), self.lo), self.hi)
        scale = self.sign * sign / math.sqrt(max(abs(t1 - t0), 1e-12))
        parts = []
        for seed, ids in self.keys:
            shape = (len(ids),) + self.shape[1:]
            parts.append(ops.brownian_increment(shape, seed, ids, self.lo, self.hi, a, b, self.tol, self.max_depth,
                                                scale, device=self.out_device))
        w = parts[0] if len(parts) == 1 else torch.cat(parts)
        return w.to(self.out_dtype)
