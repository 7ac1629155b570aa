"""Parameter-holding layers whose forward runs through the op layer (``ops``).

Parameter names match PyTorch's (``weight``/``bias``) so ldm/diffusers state dicts load directly.
Initialisation is skipped (modules are created empty, like ``comfy/ops.py:disable_weight_init``);
``init_random_`` fills random weights on the device for synthetic-checkpoint benchmarks.

Derived device layouts (conv weights in [Cout, kh, kw, Cin], fused QKV, interleaved GEGLU rows)
are cached per layer and dropped by ``invalidate_derived`` whenever weights are patched.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from .. import ops


class DerivedMixin:
    def _derived_get(self, key, fn):
        d = self.__dict__.setdefault("_derived", {})
        v = d.get(key)
        if v is None:
            v = fn()
            d[key] = v
        return v

    def invalidate_derived(self):
        self.__dict__["_derived"] = {}


# Bumped whenever weights may have moved or changed (patch / unpatch / device move): captured
# hipGraph plans (runtime/graphs.py) hold raw weight pointers and are retired on a new epoch.
WEIGHTS_EPOCH = 0


def bump_weights_epoch():
    global WEIGHTS_EPOCH
    WEIGHTS_EPOCH += 1


def invalidate_all(module: nn.Module):
    bump_weights_epoch()
    for m in module.modules():
        if isinstance(m, DerivedMixin):
            m.invalidate_derived()


class Linear(nn.Module, DerivedMixin):
    def __init__(self, in_features, out_features, bias=True, dtype=None, device=None):
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.weight = nn.Parameter(torch.empty((out_features, in_features), dtype=dtype, device=device),
                                   requires_grad=False)
        if bias:
            self.bias = nn.Parameter(torch.empty(out_features, dtype=dtype, device=device), requires_grad=False)
        else:
            self.register_parameter("bias", None)

    def forward(self, x, residual=None):
        w, b = self.weight, self.bias
        if w.dtype != x.dtype or w.device != x.device:  # manual cast (comfy/ops.py:22-32)
            w = w.to(device=x.device, dtype=x.dtype)
            b = None if b is None else b.to(device=x.device, dtype=x.dtype)
        return ops.linear(x, w, b, residual=residual)


class Conv2d(nn.Module, DerivedMixin):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, bias=True,
                 groups=1, dtype=None, device=None, padding_mode="zeros"):
        super().__init__()
        if isinstance(kernel_size, int):
            kernel_size = (kernel_size, kernel_size)
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.kernel_size = kernel_size
        self.stride = stride
        self.padding = padding
        self.groups = groups
        self.weight = nn.Parameter(torch.empty((out_channels, in_channels // groups) + tuple(kernel_size),
                                               dtype=dtype, device=device), requires_grad=False)
        if bias:
            self.bias = nn.Parameter(torch.empty(out_channels, dtype=dtype, device=device), requires_grad=False)
        else:
            self.register_parameter("bias", None)

    def weight_nhwc(self):
        return self._derived_get("w_nhwc", lambda: self.weight.permute(0, 2, 3, 1).contiguous())

    def forward(self, x, residual=None, upsample2x=False):
        w, b = self.weight, self.bias
        wn = None
        if w.dtype != x.dtype or w.device != x.device:
            w = w.to(device=x.device, dtype=x.dtype)
            b = None if b is None else b.to(device=x.device, dtype=x.dtype)
        elif x.is_cuda and self.groups == 1 and self.in_channels % 32 and x.dtype == torch.bfloat16 \
                and residual is None and not upsample2x:
            # narrow-input convs (UNet conv_in: 4 or 8 latent channels, 3-channel image stems):
            # zero-pad Cin to 32 so the MFMA implicit-GEMM kernel runs them too (no library conv
            # on the hot path, and the forward stays hipGraph-capturable).
            cp = (self.in_channels + 31) // 32 * 32
            pad = cp - self.in_channels
            w = self._derived_get("w_pad", lambda: torch.nn.functional.pad(self.weight, (0, 0, 0, 0, 0, pad)))
            wn = self._derived_get("w_nhwc_pad", lambda: w.permute(0, 2, 3, 1).contiguous())
            xp = torch.empty((x.shape[0], cp, x.shape[2], x.shape[3]), device=x.device, dtype=x.dtype,
                             memory_format=torch.channels_last)
            xp[:, self.in_channels:].zero_()
            xp[:, :self.in_channels] = x
            x = xp
        elif x.is_cuda and self.groups == 1:
            wn = self.weight_nhwc()
        return ops.conv2d(x, w, b, self.stride, self.padding, residual=residual, weight_nhwc=wn,
                          groups=self.groups, upsample2x=upsample2x)


class GroupNorm(nn.Module):
    def __init__(self, num_groups, num_channels, eps=1e-5, affine=True, dtype=None, device=None):
        super().__init__()
        self.num_groups = num_groups
        self.num_channels = num_channels
        self.eps = eps
        if affine:
            self.weight = nn.Parameter(torch.empty(num_channels, dtype=dtype, device=device), requires_grad=False)
            self.bias = nn.Parameter(torch.empty(num_channels, dtype=dtype, device=device), requires_grad=False)
        else:
            self.register_parameter("weight", None)
            self.register_parameter("bias", None)

    def forward(self, x, silu=False):
        w, b = self.weight, self.bias
        if w is not None and (w.dtype != x.dtype or w.device != x.device):
            w = w.to(device=x.device, dtype=x.dtype)
            b = b.to(device=x.device, dtype=x.dtype)
        return ops.group_norm(x, self.num_groups, w, b, self.eps, silu=silu)


class LayerNorm(nn.Module):
    def __init__(self, normalized_shape, eps=1e-5, elementwise_affine=True, bias=True, dtype=None, device=None):
        super().__init__()
        if isinstance(normalized_shape, int):
            normalized_shape = (normalized_shape,)
        self.normalized_shape = tuple(normalized_shape)
        self.eps = eps
        if elementwise_affine:
            self.weight = nn.Parameter(torch.empty(self.normalized_shape, dtype=dtype, device=device),
                                       requires_grad=False)
            if bias:
                self.bias = nn.Parameter(torch.empty(self.normalized_shape, dtype=dtype, device=device),
                                         requires_grad=False)
            else:
                self.register_parameter("bias", None)
        else:
            self.register_parameter("weight", None)
            self.register_parameter("bias", None)

    def forward(self, x):
        w, b = self.weight, self.bias
        if w is not None and (w.dtype != x.dtype or w.device != x.device):
            w = w.to(device=x.device, dtype=x.dtype)
            b = None if b is None else b.to(device=x.device, dtype=x.dtype)
        return ops.layer_norm(x, w, b, self.eps)


class Embedding(nn.Module):
    def __init__(self, num_embeddings, embedding_dim, dtype=None, device=None):
        super().__init__()
        self.weight = nn.Parameter(torch.empty((num_embeddings, embedding_dim), dtype=dtype, device=device),
                                   requires_grad=False)

    def forward(self, idx, out_dtype=None):
        w = self.weight
        r = torch.nn.functional.embedding(idx, w)
        return r if out_dtype is None else r.to(out_dtype)


@torch.no_grad()
def init_random_(module: nn.Module, seed: int = 0, std_scale: float = 1.0):
    """Random-init every parameter in place (used for synthetic checkpoints / benchmarks).

    Weights ~ N(0, std_scale/sqrt(fan_in)); norm scales = 1, biases small. Runs on whatever device
    the parameters live on (fast on the GPU).
    """
    g = torch.Generator(device="cpu").manual_seed(seed)
    for name, p in module.named_parameters():
        if p.dtype not in (torch.float32, torch.float16, torch.bfloat16):
            continue
        leaf = name.rsplit(".", 1)[-1]
        is_norm = any(s in name for s in ("norm", "ln_", "layer_norm")) and p.dim() == 1
        if is_norm and leaf == "weight":
            p.fill_(1.0)
            continue
        if p.dim() <= 1:
            t = torch.randn(p.shape, generator=g) * 0.02
        else:
            fan_in = p[0].numel()
            t = torch.randn(p.shape, generator=g) * (std_scale / math.sqrt(max(1, fan_in)))
        p.copy_(t.to(p.dtype))


@torch.no_grad()
def init_random_fast_(module: nn.Module, seed: int = 0, std_scale: float = 1.0):
    """Like init_random_ but draws on the parameter's own device (GPU-fast for 2.6B params)."""
    for i, (name, p) in enumerate(module.named_parameters()):
        leaf = name.rsplit(".", 1)[-1]
        is_norm = any(s in name for s in ("norm", "ln_", "layer_norm")) and p.dim() == 1
        if is_norm and leaf == "weight":
            p.fill_(1.0)
            continue
        gen = torch.Generator(device=p.device).manual_seed(seed * 100003 + i)
        if p.dim() == 1:
            p.normal_(0.0, 0.02, generator=gen)
        else:
            fan_in = p[0].numel()
            p.normal_(0.0, std_scale / math.sqrt(max(1, fan_in)), generator=gen)
