"""Latent-diffusion UNet for SD1.x / SD2.x / SDXL (+ refiner, SSD-1B, Vega, KOALA, IP2P, x4).

Behavioural parity with ``comfy/ldm/modules/diffusionmodules/openaimodel.py:366-890``
(UNetModel: time/label embeddings, input/middle/output blocks with skip concat, ControlNet
residual injection ``apply_control`` at :356-364, patch hooks input_block_patch /
input_block_patch_after_skip / output_block_patch at :852-877, transformer_options block
addressing at :828-870). State-dict keys are identical to ldm checkpoints.

MI355X design choices:
  * activations stay NHWC (channels_last) for the whole forward on the device;
  * ResBlock: GroupNorm+SiLU is one kernel; the timestep-embedding add ``h + emb[..., None, None]``
    is folded into the second GroupNorm (per-(n, c) pre-add), and the skip connection add is
    fused into the last conv's epilogue;
  * SiLU(emb) is computed once per forward and shared by every ResBlock;
  * all embedding projections (time/label/ResBlock emb layers) are host-launch-bound at
    M = batch, so the forward is meant to be replayed from a hipGraph (``runtime/graphs.py``).
"""
from __future__ import annotations

import logging
import os

import torch
import torch.nn as nn

from .. import ops
from .attention import BasicTransformerBlock, SpatialTransformer, _Seq
from .layers import Conv2d, Conv3d, DerivedMixin, GroupNorm, Linear, _hooked, module_epoch


def _SKIPCAT():
    import os
    return os.environ.get("CGS_SKIPCAT", "1") != "0"


class SkipCat:
    """``torch.cat([h, skip], 1)`` of the UNet decoder kept as its two halves (K14): the output
    ResBlock's GroupNorm and 1x1 skip conv read the channel concat straight from both tensors, so the
    concat (openaimodel.py:879) is never written. Anything else materialises it."""
    __slots__ = ("a", "b")

    def __init__(self, a, b):
        self.a, self.b = a, b

    @property
    def shape(self):
        return torch.Size((self.a.shape[0], self.a.shape[1] + self.b.shape[1]) + tuple(self.a.shape[2:]))

    def materialize(self):
        h = torch.cat([self.a, self.b], dim=1)
        return h.contiguous(memory_format=torch.channels_last) if h.is_cuda else h


class ResBlock(nn.Module):
    def __init__(self, channels, emb_channels, out_channels=None, dtype=None, device=None,
                 kernel_size=3, skip_t_emb=False):
        super().__init__()
        out_channels = out_channels or channels
        self.channels = channels
        self.out_channels = out_channels
        self.skip_t_emb = skip_t_emb
        pad = kernel_size // 2
        self.in_layers = _Seq(GroupNorm(32, channels, dtype=dtype, device=device), nn.SiLU(),
                              Conv2d(channels, out_channels, kernel_size, padding=pad, dtype=dtype, device=device))
        if not skip_t_emb:
            self.emb_layers = _Seq(nn.SiLU(), Linear(emb_channels, out_channels, dtype=dtype, device=device))
        self.out_layers = _Seq(GroupNorm(32, out_channels, dtype=dtype, device=device), nn.SiLU(), nn.Dropout(0.0),
                               Conv2d(out_channels, out_channels, kernel_size, padding=pad, dtype=dtype, device=device))
        if out_channels == channels:
            self.skip_connection = nn.Identity()
        else:
            self.skip_connection = Conv2d(channels, out_channels, 1, dtype=dtype, device=device)

    def forward(self, x, emb_silu, transformer_options=None):
        if isinstance(x, SkipCat):
            if isinstance(self.skip_connection, nn.Identity):
                x = x.materialize()
            else:
                h = self.in_layers[2](self.in_layers[0](x.a, silu=True, x2=x.b), gn_stats=True)
                return self._out(h, emb_silu, self.skip_connection(x.a, x2=x.b))
        h = self.in_layers[0](x, silu=True)
        h = self.in_layers[2](h, gn_stats=True)      # out_layers' GroupNorm statistics from its epilogue
        skip = x if isinstance(self.skip_connection, nn.Identity) else None
        return self._out(h, emb_silu, skip if skip is not None else self.skip_connection(x))

    def _out(self, h, emb_silu, skip):
        pre = None
        if not self.skip_t_emb and emb_silu is not None:
            pj, off = getattr(emb_silu, "_cgs_emb_proj", None), self.__dict__.get("_cgs_emb_off")
            if pj is not None and off is not None:     # this block's columns of the batched projection (a view)
                pre = pj[:, off:off + self.out_channels]
            else:
                pre = self.emb_layers[1](emb_silu).to(h.dtype)          # [B, C]
        h = ops.group_norm(h, 32, self.out_layers[0].weight, self.out_layers[0].bias,
                           self.out_layers[0].eps, silu=True, pre_add=pre)
        return self.out_layers[3](h, residual=skip)


class Downsample(nn.Module):
    def __init__(self, channels, out_channels=None, dtype=None, device=None):
        super().__init__()
        self.op = Conv2d(channels, out_channels or channels, 3, stride=2, padding=1, dtype=dtype, device=device)

    def forward(self, x, *a, **k):
        return self.op(x)


class Upsample(nn.Module):
    def __init__(self, channels, out_channels=None, dtype=None, device=None):
        super().__init__()
        self.conv = Conv2d(channels, out_channels or channels, 3, padding=1, dtype=dtype, device=device)

    def forward(self, x, *a, output_shape=None, **k):
        if output_shape is not None and (output_shape[2] != 2 * x.shape[2] or output_shape[3] != 2 * x.shape[3]):
            x = torch.nn.functional.interpolate(x, size=output_shape[2:], mode="nearest")
        else:
            return self.conv(x, upsample2x=True)
        return self.conv(x)


# ------------------------------------------------------------------------------------------------
# Video (SVD / SV3D) blocks: openaimodel.py:267-345 (VideoResBlock), attention.py:642-800
# (SpatialVideoTransformer), util.py:20-86 (AlphaBlender). Activations keep the 2-D frame layout
# [(b t), C, H, W]; temporal mixing reshapes NHWC frames, never materialises b c t h w.
# ------------------------------------------------------------------------------------------------
class AlphaBlender(nn.Module):
    def __init__(self, alpha, merge_strategy="learned_with_images"):
        super().__init__()
        self.merge_strategy = merge_strategy
        if merge_strategy == "fixed":
            self.register_buffer("mix_factor", torch.tensor([float(alpha)]))
        elif merge_strategy in ("learned", "learned_with_images"):
            self.mix_factor = nn.Parameter(torch.tensor([float(alpha)]), requires_grad=False)
        else:
            raise ValueError(f"unknown merge strategy {merge_strategy}")

    def get_alpha(self, image_only_indicator, device):
        m = self.mix_factor.to(device=device, dtype=torch.float32)
        if self.merge_strategy == "fixed":
            return m
        a = torch.sigmoid(m)
        if self.merge_strategy == "learned_with_images" and image_only_indicator is not None:
            a = torch.where(image_only_indicator.bool().to(device), torch.ones_like(a), a).reshape(-1)
        return a

    def forward(self, x_spatial, x_temporal, image_only_indicator=None):
        a = self.get_alpha(image_only_indicator, x_spatial.device)
        if a.numel() > 1:          # per-frame: frames are the leading dim of both operands
            a = a.view((-1,) + (1,) * (x_spatial.dim() - 1))
        a = a.to(x_spatial.dtype)
        return a * x_spatial + (1.0 - a) * x_temporal


def group_norm_frames(gn, x, frames, silu=False):
    """GroupNorm of a 5-D video tensor (statistics over C/G x t x h x w per video) given as frames."""
    n, c, h, w = x.shape
    b = n // frames
    if x.is_cuda:
        x4 = x.contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1).reshape(b, frames * h, w, c)
        y = gn(x4.permute(0, 3, 1, 2), silu=silu)
        return y.permute(0, 2, 3, 1).reshape(n, h, w, c).permute(0, 3, 1, 2)
    x5 = x.reshape(b, frames, c, h, w).transpose(1, 2).float()
    y = torch.nn.functional.group_norm(x5, gn.num_groups, None if gn.weight is None else gn.weight.float(),
                                       None if gn.bias is None else gn.bias.float(), gn.eps)
    if silu:
        y = torch.nn.functional.silu(y)
    return y.transpose(1, 2).reshape(n, c, h, w).to(x.dtype)


class TimeStackResBlock(nn.Module):
    """ResBlock(dims=3) of the video blocks: GN over the whole clip, temporal [kt,1,1] convs, optional
    per-frame timestep embedding (``exchange_temb_dims``), identity skip."""

    def __init__(self, channels, emb_channels, kernel_size=(3, 1, 1), skip_t_emb=False, dtype=None, device=None):
        super().__init__()
        ks = list(kernel_size) if isinstance(kernel_size, (list, tuple)) else [kernel_size] * 3
        pad = [k // 2 for k in ks]
        kw = dict(dtype=dtype, device=device)
        self.skip_t_emb = skip_t_emb
        self.in_layers = _Seq(GroupNorm(32, channels, **kw), nn.SiLU(), Conv3d(channels, channels, ks, pad, **kw))
        if not skip_t_emb:
            self.emb_layers = _Seq(nn.SiLU(), Linear(emb_channels, channels, **kw))
        self.out_layers = _Seq(GroupNorm(32, channels, **kw), nn.SiLU(), nn.Dropout(0.0),
                               Conv3d(channels, channels, ks, pad, **kw))

    def forward(self, x, emb_silu, frames):
        h = self.in_layers[2](group_norm_frames(self.in_layers[0], x, frames, silu=True), frames)
        if not self.skip_t_emb and emb_silu is not None:
            e = self.emb_layers[1](emb_silu).to(h.dtype)          # [(b t), C]: per-frame embedding
            h = h + e[:, :, None, None]
        h = group_norm_frames(self.out_layers[0], h, frames, silu=True)
        return self.out_layers[3](h, frames) + x


class TimestepEmbedSequential(nn.ModuleList):
    def forward(self, x, emb_silu, context, transformer_options, output_shape=None, time_context=None,
                num_video_frames=None, image_only_indicator=None):
        for layer in self:
            if isinstance(x, SkipCat) and not (isinstance(layer, ResBlock) and not isinstance(layer, VideoResBlock)):
                x = x.materialize()
            if isinstance(layer, VideoResBlock):
                x = layer(x, emb_silu, transformer_options, num_video_frames, image_only_indicator)
            elif isinstance(layer, ResBlock):
                x = layer(x, emb_silu, transformer_options)
            elif isinstance(layer, SpatialVideoTransformer):
                x = layer(x, context, transformer_options, time_context=time_context, frames=num_video_frames,
                          image_only_indicator=image_only_indicator)
                if "transformer_index" in transformer_options:
                    transformer_options["transformer_index"] += 1
            elif isinstance(layer, SpatialTransformer):
                x = layer(x, context, transformer_options)
                if "transformer_index" in transformer_options:
                    transformer_options["transformer_index"] += 1
            elif isinstance(layer, Upsample):
                x = layer(x, output_shape=output_shape)
            else:
                x = layer(x)
        return x


class VideoResBlock(ResBlock):
    def __init__(self, channels, emb_channels, out_channels=None, video_kernel_size=(3, 1, 1),
                 merge_strategy="fixed", merge_factor=0.5, dtype=None, device=None):
        super().__init__(channels, emb_channels, out_channels, dtype=dtype, device=device)
        self.time_stack = TimeStackResBlock(self.out_channels, emb_channels, video_kernel_size, dtype=dtype,
                                            device=device)
        self.time_mixer = AlphaBlender(merge_factor, merge_strategy)

    def forward(self, x, emb_silu, transformer_options=None, num_video_frames=None, image_only_indicator=None):
        x = super().forward(x, emb_silu, transformer_options)
        xt = self.time_stack(x, emb_silu, num_video_frames)
        return self.time_mixer(x_spatial=x, x_temporal=xt, image_only_indicator=image_only_indicator)


class SpatialVideoTransformer(SpatialTransformer):
    def __init__(self, in_channels, n_heads, d_head, depth=1, context_dim=None, use_linear=False,
                 time_context_dim=None, ff_in=False, use_spatial_context=False, merge_strategy="fixed",
                 merge_factor=0.5, disable_self_attn=False, disable_temporal_crossattention=False,
                 max_time_embed_period=10000, dtype=None, device=None):
        super().__init__(in_channels, n_heads, d_head, depth=depth, context_dim=context_dim,
                         disable_self_attn=disable_self_attn, use_linear=use_linear, dtype=dtype, device=device)
        inner = n_heads * d_head
        if use_spatial_context:
            time_context_dim = context_dim
        kw = dict(dtype=dtype, device=device)
        self.time_stack = nn.ModuleList([
            BasicTransformerBlock(inner, n_heads, d_head, context_dim=time_context_dim, ff_in=ff_in, inner_dim=inner,
                                  disable_self_attn=disable_self_attn,
                                  disable_temporal_crossattention=disable_temporal_crossattention, **kw)
            for _ in range(depth)])
        self.use_spatial_context = use_spatial_context
        self.max_time_embed_period = max_time_embed_period
        self.time_pos_embed = _Seq(Linear(in_channels, in_channels * 4, **kw), nn.SiLU(),
                                   Linear(in_channels * 4, in_channels, **kw))
        self.time_mixer = AlphaBlender(merge_factor, merge_strategy)

    def forward(self, x, context=None, transformer_options=None, time_context=None, frames=None,
                image_only_indicator=None):
        to = transformer_options if transformer_options is not None else {}
        b_t, c, h, w = x.shape
        frames = frames or b_t
        b = b_t // frames
        S = h * w
        if self.use_spatial_context:
            tc = context if time_context is None else time_context
            time_context = tc[::frames].repeat_interleave(S, dim=0)
        elif time_context is not None:
            time_context = time_context.repeat_interleave(S, dim=0)
            if time_context.dim() == 2:
                time_context = time_context[:, None]
        x_in = x
        x = self.norm(x)
        if not self.use_linear:
            x = self.proj_in(x)
        x = x.permute(0, 2, 3, 1).reshape(b_t, S, -1)
        if self.use_linear:
            x = self.proj_in(x)
        C = x.shape[-1]
        fr = torch.arange(frames, device=x.device, dtype=torch.float32).repeat(b)
        t_emb = ops.timestep_embedding(fr, self.in_channels, max_period=self.max_time_embed_period).to(x.dtype)
        emb = self.time_pos_embed[2](ops.silu(self.time_pos_embed[0](t_emb)))[:, None, :]
        for i, (blk, mix) in enumerate(zip(self.transformer_blocks, self.time_stack)):
            to["block_index"] = i
            x = blk(x, context=context, transformer_options=to)
            xm = (x + emb).reshape(b, frames, S, C).transpose(1, 2).reshape(b * S, frames, C)
            xm = mix(xm, context=time_context)
            xm = xm.reshape(b, S, frames, C).transpose(1, 2).reshape(b_t, S, C)
            x = self.time_mixer(x_spatial=x, x_temporal=xm, image_only_indicator=image_only_indicator)
        if self.use_linear:
            x = self.proj_out(x)
        x = x.reshape(b_t, h, w, -1).permute(0, 3, 1, 2)
        if not self.use_linear:
            x = self.proj_out(x)
        return x + x_in


def _apply_control(h, control, name):
    if control is not None and name in control and len(control[name]) > 0:
        ctrl = control[name].pop()
        if ctrl is not None:
            if ctrl.shape == h.shape:
                h = h + ctrl.to(h.dtype)
            else:
                logging.warning("warning control could not be applied %s %s", h.shape, ctrl.shape)
    return h


class UNetModel(nn.Module, DerivedMixin):
    def __init__(self, in_channels=4, model_channels=320, out_channels=4, num_res_blocks=2,
                 channel_mult=(1, 2, 4, 4), transformer_depth=1, transformer_depth_middle=None,
                 transformer_depth_output=None, context_dim=None, num_heads=-1, num_head_channels=-1,
                 use_linear_in_transformer=False, adm_in_channels=None, num_classes=None,
                 disable_self_attentions=None, use_temporal_attention=False, use_temporal_resblock=False,
                 time_context_dim=None, extra_ff_mix_layer=False, use_spatial_context=False, merge_strategy=None,
                 merge_factor=0.0, video_kernel_size=None, disable_temporal_crossattention=False,
                 max_ddpm_temb_period=10000, disable_middle_self_attn=False, dtype=torch.float32,
                 device=None, build_decoder=True, **unused):
        super().__init__()
        self.default_num_video_frames = None
        # latency mode may cut this network into row bands (parallel/latency.py): every layer is
        # band-aware (halo convs, group-summed GroupNorm, sequence-parallel attention) unless temporal
        # layers mix frames through the band-local ops
        self.row_shardable = not (use_temporal_attention or use_temporal_resblock)
        vks = video_kernel_size if video_kernel_size is not None else [3, 1, 1]

        def resblock(ch_in, emb_ch, ch_out, **kw2):
            if use_temporal_resblock:
                return VideoResBlock(ch_in, emb_ch, ch_out, video_kernel_size=vks, merge_strategy=merge_strategy,
                                     merge_factor=merge_factor, **kw2)
            return ResBlock(ch_in, emb_ch, ch_out, **kw2)

        def attn_layer(ch, nh, dh, depth, dsa, **kw2):
            if use_temporal_attention:
                return SpatialVideoTransformer(ch, nh, dh, depth=depth, context_dim=context_dim,
                                               use_linear=use_linear_in_transformer, time_context_dim=time_context_dim,
                                               ff_in=extra_ff_mix_layer, use_spatial_context=use_spatial_context,
                                               merge_strategy=merge_strategy, merge_factor=merge_factor,
                                               disable_self_attn=dsa,
                                               disable_temporal_crossattention=disable_temporal_crossattention,
                                               max_time_embed_period=max_ddpm_temb_period, **kw2)
            return SpatialTransformer(ch, nh, dh, depth=depth, context_dim=context_dim, disable_self_attn=dsa,
                                      use_linear=use_linear_in_transformer, **kw2)
        nl = len(channel_mult)
        if isinstance(num_res_blocks, int):
            num_res_blocks = [num_res_blocks] * nl
        if isinstance(transformer_depth, int):
            transformer_depth = [transformer_depth] * (nl * max(num_res_blocks))
        transformer_depth = list(transformer_depth)
        if transformer_depth_output is None:
            transformer_depth_output = []
            for lvl in range(nl):
                d = transformer_depth[lvl * num_res_blocks[lvl]] if lvl * num_res_blocks[lvl] < len(transformer_depth) else 0
                transformer_depth_output += [d] * (num_res_blocks[lvl] + 1)
        transformer_depth_output = list(transformer_depth_output)
        if transformer_depth_middle is None:
            transformer_depth_middle = transformer_depth[-1]
        self.dtype = dtype
        self.in_channels = in_channels
        self.model_channels = model_channels
        self.out_channels = out_channels
        self.num_classes = num_classes
        ted = model_channels * 4

        def heads_for(ch):
            if num_head_channels == -1:
                return num_heads, ch // num_heads
            return ch // num_head_channels, num_head_channels

        def dsa(i):
            return bool(disable_self_attentions[i]) if disable_self_attentions is not None else False

        kw = dict(dtype=dtype, device=device)
        self.time_embed = _Seq(Linear(model_channels, ted, **kw), nn.SiLU(), Linear(ted, ted, **kw))
        if num_classes is not None:
            if num_classes == "sequential":
                self.label_emb = _Seq(_Seq(Linear(adm_in_channels, ted, **kw), nn.SiLU(), Linear(ted, ted, **kw)))
            elif num_classes == "continuous":
                self.label_emb = nn.Linear(1, ted)
            else:
                self.label_emb = nn.Embedding(num_classes, ted)

        self.input_blocks = nn.ModuleList([TimestepEmbedSequential([Conv2d(in_channels, model_channels, 3, padding=1, **kw)])])
        chans = [model_channels]
        ch = model_channels
        td = list(transformer_depth)
        for level, mult in enumerate(channel_mult):
            for _ in range(num_res_blocks[level]):
                layers = [resblock(ch, ted, mult * model_channels, **kw)]
                ch = mult * model_channels
                nt = td.pop(0) if td else 0
                if nt > 0:
                    h, dh = heads_for(ch)
                    layers.append(attn_layer(ch, h, dh, nt, dsa(level), **kw))
                self.input_blocks.append(TimestepEmbedSequential(layers))
                chans.append(ch)
            if level != nl - 1:
                self.input_blocks.append(TimestepEmbedSequential([Downsample(ch, ch, **kw)]))
                chans.append(ch)

        self.middle_block = None
        if transformer_depth_middle >= -1:
            mid = [resblock(ch, ted, ch, **kw)]
            if transformer_depth_middle >= 0:
                h, dh = heads_for(ch)
                mid += [attn_layer(ch, h, dh, transformer_depth_middle, disable_middle_self_attn, **kw),
                        resblock(ch, ted, ch, **kw)]
            self.middle_block = TimestepEmbedSequential(mid)

        self._encoder_channels = list(chans)
        self._mid_channels = ch
        if not build_decoder:          # ControlNet: encoder + middle only (models/cldm.py)
            return
        self.output_blocks = nn.ModuleList([])
        tdo = list(transformer_depth_output)
        for level, mult in list(enumerate(channel_mult))[::-1]:
            for i in range(num_res_blocks[level] + 1):
                ich = chans.pop()
                layers = [resblock(ch + ich, ted, model_channels * mult, **kw)]
                ch = model_channels * mult
                nt = tdo.pop() if tdo else 0
                if nt > 0:
                    h, dh = heads_for(ch)
                    layers.append(attn_layer(ch, h, dh, nt, dsa(level), **kw))
                if level and i == num_res_blocks[level]:
                    layers.append(Upsample(ch, ch, **kw))
                self.output_blocks.append(TimestepEmbedSequential(layers))
        self.out = _Seq(GroupNorm(32, ch, **kw), nn.SiLU(), Conv2d(model_channels, out_channels, 3, padding=1, **kw))

    # ------------------------------------------------------------------------------------------
    def _emb_proj(self, emb_silu):
        """Every ResBlock's time-embedding projection (reference openaimodel.py:245-264, one Linear per block) as
        ONE GEMM per forward: [N, sum of the blocks' channels]. Each block's GroupNorm then reads its column slice
        in place (``ops.group_norm`` pre_add with a row stride) -- ~22 skinny launches per SDXL step become one.
        None (per-block projections) off the device, with hooked / cast-on-the-fly layers or CGS_EMB_BATCH=0."""
        if not emb_silu.is_cuda or os.environ.get("CGS_EMB_BATCH", "1") == "0":
            return None
        blocks = self.__dict__.get("_cgs_emb_blocks")
        if blocks is None:
            blocks, off = [], 0
            for m in self.modules():
                if isinstance(m, ResBlock) and not m.skip_t_emb:
                    m.__dict__["_cgs_emb_off"] = off
                    off += m.out_channels
                    blocks.append(m)
            self.__dict__["_cgs_emb_blocks"] = blocks
        lins = [b.emb_layers[1] for b in blocks]
        if not lins or any(_hooked(ln) or ln.bias is None or ln.weight.dtype != emb_silu.dtype
                           or ln.weight.device != emb_silu.device for ln in lins):
            return None
        key = (module_epoch(self), lins[0].weight.data_ptr(), lins[-1].weight.data_ptr())
        wb = self._derived_get("emb_proj", lambda: None)
        if wb is None or wb[0] != key:
            wb = (key, torch.cat([ln.weight for ln in lins]).contiguous(), torch.cat([ln.bias for ln in lins]))
            self.__dict__["_derived"]["emb_proj"] = wb
        return ops.linear(emb_silu, wb[1], wb[2])

    def forward(self, x, timesteps=None, context=None, y=None, control=None, transformer_options=None, **kwargs):
        to = transformer_options if transformer_options is not None else {}
        num_video_frames = kwargs.get("num_video_frames", self.default_num_video_frames)
        image_only_indicator = kwargs.get("image_only_indicator")
        time_context = kwargs.get("time_context")
        vk = dict(time_context=time_context, num_video_frames=num_video_frames,
                  image_only_indicator=image_only_indicator)
        to["original_shape"] = list(x.shape)
        to["transformer_index"] = 0
        patches = to.get("patches", {})
        if control is not None:  # never mutate the caller's lists
            control = {k: list(v) for k, v in control.items()}
        dt = self.dtype
        if x.is_cuda:
            x = x.to(dt).contiguous(memory_format=torch.channels_last)
        else:
            x = x.to(dt)
        if context is not None:
            context = context.to(dt)
        if time_context is not None:
            vk["time_context"] = time_context.to(dt)
        t_emb = ops.timestep_embedding(timesteps, self.model_channels).to(dt)
        emb = self.time_embed[2](ops.silu(self.time_embed[0](t_emb)))
        if self.num_classes is not None:
            assert y is not None and y.shape[0] == x.shape[0]
            le = self.label_emb[0]
            emb = le[2](ops.silu(le[0](y.to(dt))), residual=emb)
        emb_silu = ops.silu(emb)
        proj = self._emb_proj(emb_silu)
        if proj is not None:
            emb_silu._cgs_emb_proj = proj

        hs = []
        h = x
        for i, mod in enumerate(self.input_blocks):
            to["block"] = ("input", i)
            h = mod(h, emb_silu, context, to, **vk)
            h = _apply_control(h, control, "input")
            for p in patches.get("input_block_patch", []):
                h = p(h, to)
            hs.append(h)
            for p in patches.get("input_block_patch_after_skip", []):
                h = p(h, to)

        to["block"] = ("middle", 0)
        if self.middle_block is not None:
            h = self.middle_block(h, emb_silu, context, to, **vk)
        h = _apply_control(h, control, "middle")

        for i, mod in enumerate(self.output_blocks):
            to["block"] = ("output", i)
            hsp = hs.pop()
            hsp = _apply_control(hsp, control, "output")
            for p in patches.get("output_block_patch", []):
                h, hsp = p(h, hsp, to)
            if (x.is_cuda and _SKIPCAT() and h.shape[1] % 64 == 0 and hsp.shape[1] % 64 == 0
                    and h.dtype == hsp.dtype == torch.bfloat16):
                h = SkipCat(h, hsp)          # consumed by the block's ResBlock without a concat
            else:
                h = torch.cat([h, hsp], dim=1)
                if x.is_cuda:
                    h = h.contiguous(memory_format=torch.channels_last)
            out_shape = hs[-1].shape if hs else None
            h = mod(h, emb_silu, context, to, output_shape=out_shape, **vk)
        h = self.out[0](h, silu=True)
        return self.out[2](h)
