"""ControlNet model (parity: ``comfy/cldm/cldm.py:22-312``).

A trainable copy of the UNet encoder + middle block (built by ``UNetModel(build_decoder=False)`` so
keys and kernels are shared with the denoiser), a hint encoder (8 convs, /8 spatial) added after
the first input block, and 1x1 zero convs that turn every input-block output and the middle output
into residuals for the UNet (returned outermost-first; ``runtime.controlnet`` maps them onto the
UNet's input/middle/output injection points).

Device path: everything runs on the same HIP ops as the UNet (NHWC implicit-GEMM convs, fused GN,
flash attention); the hint encoder's first conv (3 input channels) is the only vendor-library conv.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops
from .attention import _Seq
from .layers import Conv2d
from .unet import UNetModel


class ControlNet(UNetModel):
    def __init__(self, hint_channels=3, model_channels=320, dtype=torch.float32, device=None, **unet_config):
        unet_config.pop("out_channels", None)
        super().__init__(model_channels=model_channels, dtype=dtype, device=device, build_decoder=False,
                         **unet_config)
        kw = dict(dtype=dtype, device=device)
        chs = [(hint_channels, 16, 1), (16, 16, 1), (16, 32, 2), (32, 32, 1), (32, 96, 2), (96, 96, 1),
               (96, 256, 2)]
        layers = []
        for cin, cout, stride in chs:
            layers += [Conv2d(cin, cout, 3, stride=stride, padding=1, **kw), nn.SiLU()]
        layers.append(Conv2d(256, model_channels, 3, padding=1, **kw))
        self.input_hint_block = _Seq(*layers)
        self.zero_convs = nn.ModuleList([_Seq(Conv2d(c, c, 1, **kw)) for c in self._encoder_channels])
        self.middle_block_out = _Seq(Conv2d(self._mid_channels, self._mid_channels, 1, **kw))

    def _hint(self, hint):
        h = hint
        mods = list(self.input_hint_block)
        for i, m in enumerate(mods):
            if isinstance(m, nn.SiLU):
                continue
            h = m(h)
            if i + 1 < len(mods) and isinstance(mods[i + 1], nn.SiLU):
                h = ops.silu(h)
        return h

    def _zero(self, conv, h, scale, res):
        """One zero conv with the ControlNet merge fused into its epilogue (K15):
        ``scale * conv(h) + res`` -- ``res`` is the chained previous ControlNet's residual for the same
        injection point (controlnet.py:92-138 control_merge). On the device the strength is folded into
        a scaled copy of the 1x1 weights/bias (one slot, recomputed when the strength changes) and
        ``res`` is the conv kernel's residual epilogue, so the residual leaves the kernel merged."""
        if res is not None:
            res = res.to(h.dtype)
        if scale == 1.0:
            return conv(h, residual=res)
        if h.is_cuda and conv.weight.dtype == h.dtype and conv.weight.device == h.device:
            d = conv.__dict__.setdefault("_derived", {})
            ent = d.get("w_scaled")
            if ent is None or ent[0] != scale:
                w = (conv.weight.float() * scale).to(h.dtype)
                b = None if conv.bias is None else (conv.bias.float() * scale).to(h.dtype)
                ent = d["w_scaled"] = (scale, w, b, w.permute(0, 2, 3, 1).contiguous())
            return ops.conv2d(h, ent[1], ent[2], conv.stride, conv.padding, residual=res, weight_nhwc=ent[3])
        y = conv(h) * scale
        return y if res is None else y + res

    def forward(self, x, hint, timesteps, context, y=None, transformer_options=None, zero_scale=None,
                zero_residuals=None, **kwargs):
        """Returns the zero-conv residuals (input blocks in order, then the middle block). With
        ``zero_scale`` / ``zero_residuals`` set, each is already ``strength * out + previous``."""
        to = dict(transformer_options or {})
        to.pop("patches", None)
        to.pop("patches_replace", None)
        dt = self.dtype
        if x.is_cuda:
            x = x.to(dt).contiguous(memory_format=torch.channels_last)
            hint = hint.to(dt).contiguous(memory_format=torch.channels_last)
        else:
            x, hint = x.to(dt), hint.to(dt)
        context = context.to(dt) if context is not None else None
        t_emb = ops.timestep_embedding(timesteps, self.model_channels).to(dt)
        emb = self.time_embed[2](ops.silu(self.time_embed[0](t_emb)))
        guided = self._hint(hint)
        if self.num_classes is not None:
            assert y is not None and y.shape[0] == x.shape[0]
            le = self.label_emb[0]
            emb = le[2](ops.silu(le[0](y.to(dt))), residual=emb)
        emb_silu = ops.silu(emb)
        outs = []
        h = x
        for i, (mod, zc) in enumerate(zip(self.input_blocks, self.zero_convs)):
            to["block"] = ("input", i)
            h = mod(h, emb_silu, context, to)
            if guided is not None:
                h = h + guided
                guided = None
            outs.append(self._emit(zc[0], h, len(outs), zero_scale, zero_residuals))
        to["block"] = ("middle", 0)
        h = self.middle_block(h, emb_silu, context, to)
        outs.append(self._emit(self.middle_block_out[0], h, len(outs), zero_scale, zero_residuals))
        return outs

    def _emit(self, conv, h, i, scale, residuals):
        if scale is None and residuals is None:
            return conv(h)
        return self._zero(conv, h, 1.0 if scale is None else float(scale),
                          None if residuals is None else residuals[i])
