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


def stamp_epoch(module: nn.Module) -> int:
    """Bump the global epoch and record it on every submodule of ``module``: captured graphs key on
    ``module_epoch`` of the model they hold pointers into, so patching / moving one model (Cascade
    Stage B) does not retire the plans of another (Stage C)."""
    bump_weights_epoch()
    for m in module.modules():
        m.__dict__["_cgs_epoch"] = WEIGHTS_EPOCH
    return WEIGHTS_EPOCH


def module_epoch(module) -> int:
    """Weight epoch of ``module``'s tree (0 until it is first patched / moved)."""
    return module.__dict__.get("_cgs_epoch", 0) if module is not None else 0


def invalidate_all(module: nn.Module):
    stamp_epoch(module)
    for m in module.modules():
        if isinstance(m, DerivedMixin):
            m.invalidate_derived()


class CastWeightBiasOp:
    """Per-layer weight / bias hooks (``comfy/ops.py:34``): custom nodes set ``weight_function`` /
    ``bias_function`` on a layer to transform its parameters on every forward (on-the-fly LoRA,
    dequantisation, ...); ``cast_bias_weight`` applies them after the device / dtype cast."""
    comfy_cast_weights = False
    weight_function = None
    bias_function = None


def cast_bias_weight(s, input):
    """(weight, bias) of layer ``s`` cast to ``input``'s device / dtype, hooks applied (``comfy/ops.py:22``)."""
    bias = None
    if s.bias is not None:
        bias = s.bias.to(device=input.device, dtype=input.dtype)
        if s.bias_function is not None:
            bias = s.bias_function(bias)
    weight = s.weight.to(device=input.device, dtype=input.dtype)
    if s.weight_function is not None:
        weight = s.weight_function(weight)
    return weight, bias


def _hooked(s) -> bool:
    return s.weight_function is not None or s.bias_function is not None


class Linear(nn.Module, DerivedMixin, CastWeightBiasOp):
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

    def forward(self, x, residual=None, act=None, row_stats=False):
        """``act="gelu"``: GELU fused into the GEMM epilogue (before the residual). ``row_stats``: the
        next op is a LayerNorm over the output (``ops.linear`` row-statistics partials)."""
        if _hooked(self):
            w, b = cast_bias_weight(self, x)
            return ops.linear(x, w, b, residual=residual, act=act, row_stats=row_stats)
        w, b = self.weight, self.bias
        if w.dtype == torch.float8_e4m3fn and w.device == x.device and x.dtype == torch.bfloat16 and x.is_cuda:
            # fp8-stored weights go to the fp8-weight GEMM as they are (widened inside the kernel)
            return ops.linear(x, w, None if b is None else b.to(dtype=x.dtype), residual=residual, act=act)
        if w.dtype != x.dtype or w.device != x.device:  # manual cast (comfy/ops.py:22-32)
            w = w.to(device=x.device, dtype=x.dtype)
            b = None if b is None else b.to(device=x.device, dtype=x.dtype)
        return ops.linear(x, w, b, residual=residual, act=act, row_stats=row_stats)

    def weight_bias_for(self, x):
        """(weight, bias) as the forward would use them for ``x`` (hooks applied, cast to x's dtype)."""
        if _hooked(self):
            return cast_bias_weight(self, x)
        w, b = self.weight, self.bias
        if w.dtype != x.dtype or w.device != x.device:
            w = w.to(device=x.device, dtype=x.dtype)
            b = None if b is None else b.to(device=x.device, dtype=x.dtype)
        return w, b


class Conv2d(nn.Module, DerivedMixin, CastWeightBiasOp):
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

    def forward(self, x, residual=None, upsample2x=False, x2=None, gn_stats=False):
        """``x2``: convolve cat([x, x2], 1) without materialising the concat (K14). ``gn_stats``: the next op
        is a GroupNorm over the output (``ops.conv2d`` statistics partials from the epilogue)."""
        if _hooked(self):    # per-call weight / bias hooks: transformed weights, no cached layouts
            if x2 is not None:
                x = torch.cat([x, x2], dim=1)
            w, b = cast_bias_weight(self, x)
            return ops.conv2d(x, w, b, self.stride, self.padding, residual=residual, groups=self.groups,
                              upsample2x=upsample2x)
        w, b = self.weight, self.bias
        wn = None
        if x2 is not None:
            if x.is_cuda and self.groups == 1 and w.dtype == x.dtype and w.device == x.device:
                return ops.conv2d(x, w, b, self.stride, self.padding, residual=residual,
                                  weight_nhwc=self.weight_nhwc(), groups=self.groups, x2=x2, gn_stats=gn_stats)
            x = torch.cat([x, x2], dim=1)
        if w.dtype != x.dtype or w.device != x.device:
            w = w.to(device=x.device, dtype=x.dtype)
            b = None if b is None else b.to(device=x.device, dtype=x.dtype)
        elif x.is_cuda and self.groups == 1 and self.in_channels % 32 and x.dtype == torch.bfloat16 \
                and residual is None and not upsample2x:
            # narrow-input convs (UNet conv_in: 4 or 8 latent channels, 3-channel image stems):
            # zero-pad Cin to 32 so the MFMA implicit-GEMM kernel runs them too (no library conv
            # on the hot path, and the forward stays hipGraph-capturable).
            q = 32 if self.out_channels % 8 == 0 else 64      # kernel legality: Cout % 8 or Cin % 64
            cp = (self.in_channels + q - 1) // q * q
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
                          groups=self.groups, upsample2x=upsample2x, gn_stats=gn_stats)


class Conv3d(nn.Module, DerivedMixin):
    """3-D convolution for the video blocks (SVD time-mixing ResBlocks, AE3DConv of the temporal VAE).

    Activations stay in the 2-D frame layout ``[(b t), C, H, W]`` (channels_last on the device);
    ``forward(x, frames)`` convolves over (t, h, w) of the ``b = N / frames`` videos. The video
    kernels are temporal-only, ``[kt, 1, 1]`` with padding ``[kt // 2, 0, 0]``: on the device that is
    one implicit-GEMM MFMA conv over the image ``[b, t + 2p, h*w, C]`` with a ``(kt, 1)`` filter (the
    frames are zero-padded along t once, never an im2col). Other kernel shapes run ``F.conv3d``.
    """

    def __init__(self, in_channels, out_channels, kernel_size, padding=0, bias=True, dtype=None, device=None):
        super().__init__()
        ks = tuple(kernel_size) if isinstance(kernel_size, (list, tuple)) else (kernel_size,) * 3
        pd = tuple(padding) if isinstance(padding, (list, tuple)) else (padding,) * 3
        self.in_channels, self.out_channels, self.kernel_size, self.padding = in_channels, out_channels, ks, pd
        self.weight = nn.Parameter(torch.empty((out_channels, in_channels) + ks, dtype=dtype, device=device),
                                   requires_grad=False)
        if bias:
            self.bias = nn.Parameter(torch.empty(out_channels, dtype=dtype, device=device), requires_grad=False)
        else:
            self.register_parameter("bias", None)

    def forward(self, x, frames):
        n, c, h, w = x.shape
        b = n // frames
        kt, kh, kw = self.kernel_size
        wgt, bias = self.weight, self.bias
        if wgt.dtype != x.dtype or wgt.device != x.device:
            wgt = wgt.to(device=x.device, dtype=x.dtype)
            bias = None if bias is None else bias.to(device=x.device, dtype=x.dtype)
        temporal = kh == 1 and kw == 1 and self.padding[1] == 0 and self.padding[2] == 0
        if x.is_cuda and temporal and x.dtype == torch.bfloat16 and c % 32 == 0 and wgt is self.weight:
            p = self.padding[0]
            xf = x.contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1).reshape(b, frames, h * w, c)
            if p:
                xp = torch.empty((b, frames + 2 * p, h * w, c), device=x.device, dtype=x.dtype)
                xp[:, :p].zero_()
                xp[:, frames + p:].zero_()
                xp[:, p:frames + p] = xf
            else:
                xp = xf
            img = xp.permute(0, 3, 1, 2)                      # [b, C, t+2p, h*w], channels_last storage
            w2 = self._derived_get("w2d", lambda: self.weight.reshape(self.out_channels, self.in_channels, kt, 1))
            wn = self._derived_get("w2d_nhwc", lambda: w2.permute(0, 2, 3, 1).contiguous())
            y = ops.conv2d(img, w2, bias, 1, 0, weight_nhwc=wn)  # [b, Cout, t, h*w]
            y = y.permute(0, 2, 3, 1).reshape(n, h, w, self.out_channels)
            return y.permute(0, 3, 1, 2)
        x5 = x.reshape(b, frames, c, h, w).permute(0, 2, 1, 3, 4).float()
        y = torch.nn.functional.conv3d(x5, wgt.float(), None if bias is None else bias.float(), 1, self.padding)
        y = y.permute(0, 2, 1, 3, 4).reshape(n, self.out_channels, h, w).to(x.dtype)
        return y.contiguous(memory_format=torch.channels_last) if x.is_cuda else y


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

    def forward(self, x, silu=False, x2=None):
        w, b = self.weight, self.bias
        if w is not None and (w.dtype != x.dtype or w.device != x.device):
            w = w.to(device=x.device, dtype=x.dtype)
            b = b.to(device=x.device, dtype=x.dtype)
        return ops.group_norm(x, self.num_groups, w, b, self.eps, silu=silu, x2=x2)


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
