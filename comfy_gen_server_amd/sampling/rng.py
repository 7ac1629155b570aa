"""Counter-based noise keyed by (seed, GLOBAL image index, stream) — SURVEY §2.4 K18.

The device path is ``csrc/kernels/rng.hip`` (Philox4x32-10 + Box-Muller, and a virtual Brownian
tree walked in registers); this module holds the bit-exact torch mirror used on the CPU and as the
numerics oracle, plus the dispatching helpers the samplers call.

Why per image: the reference draws ``torch.randn_like(x)`` for the whole batch from one global RNG
(``comfy/k_diffusion/sampling.py:60-61``). With one process per GPU, a shared per-rank stream would
give image j on every rank the same ancestral noise. Keying every draw by the image's global batch
index makes a data-parallel run of a batch identical to the one-GPU run of the same batch, for any
rank split (the same replay rule ``prepare_noise`` uses for the initial latent noise,
``comfy/sample.py:8-25``).
"""
from __future__ import annotations

import math

import torch

_M64 = (1 << 64) - 1
_M32 = 0xFFFFFFFF
PH_M0, PH_M1 = 0xD2511F53, 0xCD9E8D57
PH_W0, PH_W1 = 0x9E3779B9, 0xBB67AE85
TWO_PI = 6.2831853  # rounded to fp32 exactly as the kernel's literal
TREE_DOMAIN = 1 << 63


def _mix64(z: int) -> int:
    z &= _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def image_key(seed: int, index: int) -> int:
    return _mix64(_mix64(int(seed) & _M64) ^ ((int(index) * 0x9E3779B97F4A7C15 + 0x632BE59BD9B4E019) & _M64))


def tree_stream(depth: int, idx: int) -> int:
    return TREE_DOMAIN | (int(depth) << 40) | int(idx)


def _mulhilo(m: int, c: torch.Tensor):
    p = c * m   # int64 wrap-around keeps the low 64 bits of the 32x32 product exact
    return (p >> 32) & _M32, p & _M32


def _philox10(c0, c1, c2, c3, k0: torch.Tensor, k1: torch.Tensor):
    for _ in range(10):
        hi0, lo0 = _mulhilo(PH_M0, c0)
        hi1, lo1 = _mulhilo(PH_M1, c2)
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        k0 = (k0 + PH_W0) & _M32
        k1 = (k1 + PH_W1) & _M32
    return c0, c1, c2, c3


def _u01(v: torch.Tensor) -> torch.Tensor:
    return ((v >> 8).to(torch.float32) + 0.5) * (1.0 / 16777216.0)


def _key_tensors(seed: int, inds):
    keys = [image_key(seed, i) for i in inds]
    k0 = torch.tensor([k & _M32 for k in keys], dtype=torch.int64).view(-1, 1)
    k1 = torch.tensor([k >> 32 for k in keys], dtype=torch.int64).view(-1, 1)
    return k0, k1


def normal_groups(seed: int, inds, groups: int, stream: int) -> torch.Tensor:
    """[len(inds), groups*4] fp32 normals (CPU), element 4g+j = normal j of Philox group g."""
    k0, k1 = _key_tensors(seed, inds)
    g = torch.arange(groups, dtype=torch.int64).view(1, -1)
    s = int(stream) & _M64
    c0 = (g & _M32).expand(len(inds), -1)
    c1 = (g >> 32).expand(len(inds), -1)
    c2 = torch.full_like(c0, s & _M32)
    c3 = torch.full_like(c0, s >> 32)
    k0 = k0.expand_as(c0)
    k1 = k1.expand_as(c0)
    c0, c1, c2, c3 = _philox10(c0, c1, c2, c3, k0, k1)
    two_pi = torch.tensor(TWO_PI, dtype=torch.float32)
    r0 = torch.sqrt(-2.0 * torch.log(_u01(c0)))
    t0 = two_pi * _u01(c1)
    r1 = torch.sqrt(-2.0 * torch.log(_u01(c2)))
    t1 = two_pi * _u01(c3)
    z = torch.stack([r0 * torch.cos(t0), r0 * torch.sin(t0), r1 * torch.cos(t1), r1 * torch.sin(t1)], dim=-1)
    return z.reshape(len(inds), groups * 4)


def randn_reference(shape, seed: int, inds, stream: int) -> torch.Tensor:
    """CPU mirror of ``cgs_philox_randn``: fp32 [B, ...] with B == len(inds)."""
    B = shape[0]
    assert B == len(inds), (shape, len(inds))
    n = 1
    for d in shape[1:]:
        n *= int(d)
    z = normal_groups(seed, inds, (n + 3) // 4, stream)[:, :n]
    return z.reshape(shape).contiguous()


def _tree_value(seed, inds, groups, t, t0, t1, tol, max_depth):
    if t <= t0:
        return torch.zeros(len(inds), groups * 4)
    s1 = torch.tensor(math.sqrt(t1 - t0), dtype=torch.float32)
    wa = torch.zeros(len(inds), groups * 4)
    wb = normal_groups(seed, inds, groups, tree_stream(0, 0)) * s1
    a, b, idx, depth = t0, t1, 0, 0
    while (b - a) > tol and depth < max_depth:
        m = 0.5 * (a + b)
        sd = torch.tensor(math.sqrt((b - a) / 4.0), dtype=torch.float32)
        wm = 0.5 * (wa + wb) + normal_groups(seed, inds, groups, tree_stream(depth + 1, idx)) * sd
        if t <= m:
            b, wb, idx = m, wm, 2 * idx
        else:
            a, wa, idx = m, wm, 2 * idx + 1
        depth += 1
    f = torch.tensor((t - a) / (b - a) if b > a else 0.0, dtype=torch.float32)
    return wa + (wb - wa) * f


def brownian_reference(shape, seed, inds, t0, t1, ta, tb, tol, max_depth, scale) -> torch.Tensor:
    """CPU mirror of ``cgs_brownian_increment``: (W(tb) - W(ta)) * scale per image."""
    n = 1
    for d in shape[1:]:
        n *= int(d)
    groups = (n + 3) // 4
    wb = _tree_value(seed, inds, groups, tb, t0, t1, tol, max_depth)
    wa = _tree_value(seed, inds, groups, ta, t0, t1, tol, max_depth)
    out = (wb - wa) * torch.tensor(scale, dtype=torch.float32)
    return out[:, :n].reshape(shape).contiguous()


def contiguous_inds(inds):
    """(index0, True) when ``inds`` is index0, index0+1, ... (the kernels take an offset)."""
    inds = [int(i) for i in inds]
    if inds and inds == list(range(inds[0], inds[0] + len(inds))):
        return inds[0], True
    return None, False


class StepNoise:
    """Ancestral / SDE noise sampler: call k returns N(seed, image, stream=k) for every image.

    ``inds`` are the images' global batch indices (default ``range(B)``). Device tensors draw through
    the HIP kernel (one launch, no generator state), CPU tensors through the torch mirror."""

    def __init__(self, x: torch.Tensor, seed: int, inds=None):
        self.shape = tuple(x.shape)
        self.device, self.dtype = x.device, x.dtype
        self.seed = int(seed)
        self.inds = list(range(x.shape[0])) if inds is None else [int(i) for i in inds]
        self.calls = 0

    def draw(self, stream: int) -> torch.Tensor:
        from .. import ops
        return ops.philox_randn(self.shape, self.seed, self.inds, stream, device=self.device, dtype=self.dtype)

    def __call__(self, sigma=None, sigma_next=None):
        z = self.draw(self.calls)
        self.calls += 1
        return z
