"""Transformer blocks of the latent-diffusion UNet.

Behavioural parity with ``comfy/ldm/modules/attention.py:386-640`` (CrossAttention,
BasicTransformerBlock incl. every ``transformer_options`` patch point, SpatialTransformer).
MI355X design:
  * self-attention q/k/v come from ONE fused GEMM (weight rows [Wq;Wk;Wv]); the flash kernel
    reads q, k, v as strided views of that buffer — no head split/permute copies;
  * cross-attention k/v are one fused GEMM over the context; within a sampling run the context
    is constant, so its k/v are cached per (context tensor, block) (``ctx_cache``);
  * residual adds ``x + attn(...)``/``x + ff(...)`` are fused into the out-projection GEMM epilogue;
  * GEGLU's gate is fused into the projection GEMM epilogue (interleaved weight rows).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops
from .layers import DerivedMixin, GroupNorm, LayerNorm, Linear, Conv2d


class _Seq(nn.Module):
    """nn.Sequential-compatible container whose forward forwards extra kwargs to element 0."""

    def __init__(self, *mods):
        super().__init__()
        for i, m in enumerate(mods):
            if m is not None:
                self.add_module(str(i), m)

    def __getitem__(self, i):
        return self._modules[str(i)]

    def __iter__(self):
        return iter(self._modules.values())

    def __len__(self):
        return len(self._modules)


class CrossAttention(nn.Module, DerivedMixin):
    def __init__(self, query_dim, context_dim=None, heads=8, dim_head=64, dtype=None, device=None):
        super().__init__()
        inner = heads * dim_head
        context_dim = query_dim if context_dim is None else context_dim
        self.heads = heads
        self.dim_head = dim_head
        self.is_cross = context_dim != query_dim
        self.to_q = Linear(query_dim, inner, bias=False, dtype=dtype, device=device)
        self.to_k = Linear(context_dim, inner, bias=False, dtype=dtype, device=device)
        self.to_v = Linear(context_dim, inner, bias=False, dtype=dtype, device=device)
        self.to_out = _Seq(Linear(inner, query_dim, dtype=dtype, device=device))

    def _w_qkv(self):
        return self._derived_get("w_qkv", lambda: torch.cat(
            [self.to_q.weight, self.to_k.weight, self.to_v.weight], 0).contiguous())

    def _w_kv(self):
        return self._derived_get("w_kv", lambda: torch.cat([self.to_k.weight, self.to_v.weight], 0).contiguous())

    def project_kv(self, context, value=None, ctx_cache=None, cache_key=None):
        """k, v for ``context`` (and optional separate ``value`` source)."""
        if value is not None and value is not context:
            return self.to_k(context), self.to_v(value)
        if ctx_cache is not None and cache_key is not None:
            hit = ctx_cache.get(cache_key)
            if hit is not None and hit[0] is context:
                return hit[1], hit[2]
        inner = self.heads * self.dim_head
        if context.dtype == self.to_k.weight.dtype and context.device == self.to_k.weight.device:
            kv = ops.linear(context, self._w_kv())
            k, v = kv[..., :inner], kv[..., inner:]
        else:
            k, v = self.to_k(context), self.to_v(context)
        if ctx_cache is not None and cache_key is not None:
            ctx_cache[cache_key] = (context, k, v)
        return k, v

    def forward_lnfold(self, x, rs, norm, residual=None, sp=None, row_stats=False):
        """Self-attention on LN(x) with the LayerNorm folded into the fused QKV GEMM (K07): ``x`` raw
        rows, ``rs`` their (mean, rstd) from ``ops.layernorm_stats``; ``row_stats``: the output feeds a
        LayerNorm (the out-projection's epilogue writes its statistics partials)."""
        inner = self.heads * self.dim_head
        w2, cs, b2 = self._derived_get(("lnfold_qkv", id(norm)), lambda: ops.lnfold_weights(
            self._w_qkv(), None, norm.weight, norm.bias))
        qkv = ops.linear_lnfold(x, rs, w2, cs, b2)
        q, k, v = qkv[..., :inner], qkv[..., inner:2 * inner], qkv[..., 2 * inner:]
        if sp is not None:
            o = sp.attention(q.contiguous(), k.contiguous(), v.contiguous(), self.heads)
        else:
            o = ops.attention(q, k, v, self.heads)
        return self.to_out[0](o, residual=residual, row_stats=row_stats)

    def forward_lnfold_cross(self, x, rs, norm, context, residual=None, ctx_cache=None, cache_key=None, kv=None,
                             row_stats=False):
        """Cross-attention on LN(x) with the LayerNorm folded into the query GEMM."""
        w2, cs, b2 = self._derived_get(("lnfold_q", id(norm)), lambda: ops.lnfold_weights(
            self.to_q.weight, None, norm.weight, norm.bias))
        q = ops.linear_lnfold(x, rs, w2, cs, b2)
        kvs = None
        if kv is not None and context.is_cuda and context.dtype == self.to_k.weight.dtype:
            kvs = self.static_kv(context, kv)
        k, v = kvs if kvs is not None else self.project_kv(context, None, ctx_cache, cache_key)
        o = ops.attention(q, k, v, self.heads)
        return self.to_out[0](o, residual=residual, row_stats=row_stats)

    def static_kv(self, context, kv):
        """Cross-attention K/V of a sampling run's constant context, kept in a per-context buffer
        (``kv`` = (mode, ids of the step plan's static context tensors), sampling/step_graph.py): in
        "fill" mode the fused K/V GEMM runs and its result is stored; in "use" mode (the captured
        step graph) the buffer is read, so the replayed steps carry no K/V GEMM -- the run's prologue
        (``refresh_static_kv``) recomputes it once per job instead of once per step."""
        mode, sources = kv
        if id(context) not in sources:
            return None
        inner = self.heads * self.dim_head
        store = self.__dict__.setdefault("_kv_static", {})
        ent = store.get(id(context))
        if mode == "fill" or ent is None or ent[0] is not context:
            kvt = ops.linear(context, self._w_kv())
            if ent is None or ent[0] is not context or ent[1].shape != kvt.shape:
                ent = (context, torch.empty_like(kvt))
                store[id(context)] = ent
            ent[1].copy_(kvt)
        buf = ent[1]
        return buf[..., :inner], buf[..., inner:]

    def refresh_static_kv(self, sources) -> int:
        n = 0
        for key, (ctx, buf) in self.__dict__.get("_kv_static", {}).items():
            if key in sources:
                buf.copy_(ops.linear(ctx, self._w_kv()))
                n += 1
        return n

    def forward(self, x, context=None, value=None, mask=None, residual=None, ctx_cache=None, cache_key=None,
                sp=None, kv=None):
        """``sp`` (parallel.sp.SeqParallel): x is this rank's token shard; self-attention runs over
        the whole sequence through ``sp.attention`` (cross-attention needs no exchange). ``kv``:
        step-graph static K/V mode (``static_kv``)."""
        inner = self.heads * self.dim_head
        if context is None and value is None and x.dtype == self.to_q.weight.dtype \
                and x.device == self.to_q.weight.device:
            qkv = ops.linear(x, self._w_qkv())
            q, k, v = qkv[..., :inner], qkv[..., inner:2 * inner], qkv[..., 2 * inner:]
        else:
            q = self.to_q(x)
            ctx = x if context is None else context
            kvs = None
            if kv is not None and value is None and context is not None and context.is_cuda \
                    and context.dtype == self.to_k.weight.dtype:
                kvs = self.static_kv(context, kv)
            k, v = kvs if kvs is not None else self.project_kv(ctx, value, ctx_cache, cache_key)
        if sp is not None and context is None and value is None and mask is None:
            o = sp.attention(q.contiguous(), k.contiguous(), v.contiguous(), self.heads)
        else:
            o = ops.attention(q, k, v, self.heads, mask=mask)
        return self.to_out[0](o, residual=residual)


class GEGLU(nn.Module, DerivedMixin):
    def __init__(self, dim_in, dim_out, dtype=None, device=None):
        super().__init__()
        self.proj = Linear(dim_in, dim_out * 2, dtype=dtype, device=device)

    def forward(self, x):
        if x.is_cuda and x.dtype == self.proj.weight.dtype and \
                ops.dispatch.backend_for("gemm", x, "cgs_gemm_bf16") == "hip":
            w = self._derived_get("w_il", lambda: ops.core.geglu_interleave(self.proj.weight))
            b = self._derived_get("b_il", lambda: ops.core.geglu_interleave(self.proj.bias))
            return ops.linear_geglu(x, w, b)
        h = self.proj(x)
        a, g = h.chunk(2, dim=-1)
        return a * torch.nn.functional.gelu(g)


class GELUProj(_Seq):
    """Non-gated projection ``Sequential(Linear, GELU)`` (keys ``net.0.0.*``, attention.py:71-74)."""

    def __init__(self, dim_in, dim_out, dtype=None, device=None):
        super().__init__(Linear(dim_in, dim_out, dtype=dtype, device=device))

    def forward(self, x):
        return torch.nn.functional.gelu(self[0](x))


class FeedForward(nn.Module):
    def __init__(self, dim, dim_out=None, mult=4, glu=True, dtype=None, device=None):
        super().__init__()
        inner = int(dim * mult)
        dim_out = dim if dim_out is None else dim_out
        proj = GEGLU(dim, inner, dtype=dtype, device=device) if glu else GELUProj(dim, inner, dtype=dtype, device=device)
        self.net = _Seq(proj, nn.Identity(), Linear(inner, dim_out, dtype=dtype, device=device))

    def forward(self, x, residual=None):
        return self.net[2](self.net[0](x), residual=residual)

    def lnfold_ok(self) -> bool:
        return isinstance(self.net[0], GEGLU)

    def forward_lnfold(self, x, rs, norm, residual=None, row_stats=False):
        """FF on LN(x) with the LayerNorm folded into the GEGLU GEMM (interleaved a/g rows)."""
        g = self.net[0]
        w2, cs, b2 = g._derived_get(("lnfold_geglu", id(norm)), lambda: ops.lnfold_weights(
            ops.core.geglu_interleave(g.proj.weight), ops.core.geglu_interleave(g.proj.bias), norm.weight, norm.bias))
        return self.net[2](ops.linear_lnfold(x, rs, w2, cs, b2, geglu=True), residual=residual, row_stats=row_stats)


class BasicTransformerBlock(nn.Module):
    def __init__(self, dim, n_heads, d_head, context_dim=None, gated_ff=True, disable_self_attn=False,
                 dtype=None, device=None, ff_in=False, inner_dim=None, disable_temporal_crossattention=False,
                 switch_temporal_ca_to_sa=False):
        super().__init__()
        kw = dict(dtype=dtype, device=device)
        # video (SVD time-mixing) options of attention.py:419-457: an input FF (dim -> inner_dim), a
        # residual only when inner_dim == dim, optional temporal cross-attention
        self.has_ff_in = bool(ff_in or inner_dim is not None)
        inner_dim = dim if inner_dim is None else inner_dim
        self.is_res = inner_dim == dim
        if self.has_ff_in:
            self.norm_in = LayerNorm(dim, **kw)
            self.ff_in = FeedForward(dim, dim_out=inner_dim, glu=gated_ff, **kw)
        self.disable_self_attn = disable_self_attn
        self.switch_temporal_ca_to_sa = switch_temporal_ca_to_sa
        self.n_heads = n_heads
        self.d_head = d_head
        self.attn1 = CrossAttention(inner_dim, context_dim if disable_self_attn else None, n_heads, d_head, **kw)
        self.ff = FeedForward(inner_dim, dim_out=dim, glu=gated_ff, **kw)
        if disable_temporal_crossattention:
            if switch_temporal_ca_to_sa:
                raise ValueError("switch_temporal_ca_to_sa needs the temporal cross-attention")
            self.attn2 = None
        else:
            self.attn2 = CrossAttention(inner_dim, None if switch_temporal_ca_to_sa else context_dim, n_heads, d_head,
                                        **kw)
            self.norm2 = LayerNorm(inner_dim, **kw)
        self.norm1 = LayerNorm(inner_dim, **kw)
        self.norm3 = LayerNorm(inner_dim, **kw)
        self._plain = not self.has_ff_in and self.attn2 is not None and self.is_res and not switch_temporal_ca_to_sa

    def forward(self, x, context=None, transformer_options=None):
        to = transformer_options or {}
        patches = to.get("patches", {})
        replace = to.get("patches_replace", {})
        if not self._plain:
            return self._forward_video(x, context)
        if not patches and not replace:
            return self._forward_fast(x, context, to)
        return self._forward_patched(x, context, to, patches, replace)

    def _forward_video(self, x, context):
        """Time-mixing block (SVD): ff_in, self-attention, optional temporal cross-attention, FF."""
        if self.has_ff_in:
            x = self.ff_in(self.norm_in(x), residual=x if self.is_res else None)
        ctx1 = context if self.disable_self_attn else None
        x = self.attn1(self.norm1(x), context=ctx1, residual=x)
        if self.attn2 is not None:
            n = self.norm2(x)
            x = self.attn2(n, context=n if self.switch_temporal_ca_to_sa else context, residual=x)
        return self.ff(self.norm3(x), residual=x if self.is_res else None)

    def _lnfold_ok(self, x) -> bool:
        n1, n3 = self.norm1, self.norm3
        return (n1.weight is not None and n3.weight is not None and n1.weight.dtype == x.dtype
                and n3.weight.dtype == x.dtype and self.attn1.to_q.weight.dtype == x.dtype
                and self.ff.lnfold_ok() and ops.lnfold_available(x, x.shape[-1]))

    def _forward_fast(self, x, context, to):
        """Hook-free path: residual adds fused into the out-projection / FF-out GEMM epilogues; on
        the device the LayerNorms before the fused QKV GEMM and the GEGLU GEMM are folded into those
        GEMMs (only per-row statistics are computed; LN(x) never materialises)."""
        cache = to.get("ctx_cache")
        key = id(self)
        if self._lnfold_ok(x):
            if self.disable_self_attn:
                x = self.attn1(self.norm1(x), context=context, residual=x, ctx_cache=cache, cache_key=(key, 1))
            else:
                # (the LayerNorm statistics come from the producing GEMM's epilogue where it wrote them:
                # ops.layernorm_stats_for)
                x = self.attn1.forward_lnfold(x, ops.layernorm_stats_for(x, self.norm1.eps), self.norm1, residual=x,
                                              sp=to.get("sp"), row_stats=True)
            if self.attn2.is_cross and self.norm2.weight is not None and self.norm2.weight.dtype == x.dtype:
                x = self.attn2.forward_lnfold_cross(x, ops.layernorm_stats_for(x, self.norm2.eps), self.norm2,
                                                    context, residual=x, ctx_cache=cache, cache_key=(key, 2),
                                                    kv=to.get("kv_static"), row_stats=True)
            else:
                x = self.attn2(self.norm2(x), context=context, residual=x, ctx_cache=cache, cache_key=(key, 2),
                               kv=to.get("kv_static"))
            return self.ff.forward_lnfold(x, ops.layernorm_stats_for(x, self.norm3.eps), self.norm3, residual=x,
                                          row_stats=True)
        n = self.norm1(x)
        if self.disable_self_attn:
            x = self.attn1(n, context=context, residual=x, ctx_cache=cache, cache_key=(key, 1))
        else:
            x = self.attn1(n, residual=x, sp=to.get("sp"))
        n = self.norm2(x)
        x = self.attn2(n, context=context, residual=x, ctx_cache=cache, cache_key=(key, 2), kv=to.get("kv_static"))
        return self.ff(self.norm3(x), residual=x)

    def _forward_patched(self, x, context, to, patches, replace):
        extra = {k: v for k, v in to.items() if k not in ("patches", "patches_replace")}
        extra["n_heads"] = self.n_heads
        extra["dim_head"] = self.d_head
        block = to.get("block")
        block_index = to.get("block_index", 0)
        tblock = (block[0], block[1], block_index) if block is not None else None

        n = self.norm1(x)
        ctx1 = context if self.disable_self_attn else None
        val1 = None
        if "attn1_patch" in patches:
            if ctx1 is None:
                ctx1 = n
            val1 = ctx1
            for p in patches["attn1_patch"]:
                n, ctx1, val1 = p(n, ctx1, val1, extra)
        r1 = replace.get("attn1", {})
        key1 = tblock if tblock in r1 else block
        if key1 in r1:
            if ctx1 is None:
                ctx1 = n
                val1 = n
            q = self.attn1.to_q(n)
            k = self.attn1.to_k(ctx1)
            v = self.attn1.to_v(val1)
            n = self.attn1.to_out[0](r1[key1](q, k, v, extra))
        else:
            n = self.attn1(n, context=ctx1, value=val1)
        for p in patches.get("attn1_output_patch", []):
            n = p(n, extra)
        x = x + n
        for p in patches.get("middle_patch", []):
            x = p(x, extra)

        n = self.norm2(x)
        ctx2 = context
        val2 = None
        if "attn2_patch" in patches:
            val2 = ctx2
            for p in patches["attn2_patch"]:
                n, ctx2, val2 = p(n, ctx2, val2, extra)
        r2 = replace.get("attn2", {})
        key2 = tblock if tblock in r2 else block
        if key2 in r2:
            if val2 is None:
                val2 = ctx2
            q = self.attn2.to_q(n)
            k = self.attn2.to_k(ctx2)
            v = self.attn2.to_v(val2)
            n = self.attn2.to_out[0](r2[key2](q, k, v, extra))
        else:
            n = self.attn2(n, context=ctx2, value=val2)
        for p in patches.get("attn2_output_patch", []):
            n = p(n, extra)
        x = x + n
        return self.ff(self.norm3(x), residual=x)


class SpatialTransformer(nn.Module):
    def __init__(self, in_channels, n_heads, d_head, depth=1, context_dim=None, disable_self_attn=False,
                 use_linear=False, dtype=None, device=None):
        super().__init__()
        if not isinstance(context_dim, (list, tuple)):
            context_dim = [context_dim] * depth
        inner = n_heads * d_head
        self.in_channels = in_channels
        self.use_linear = use_linear
        self.norm = GroupNorm(32, in_channels, eps=1e-6, dtype=dtype, device=device)
        if use_linear:
            self.proj_in = Linear(in_channels, inner, dtype=dtype, device=device)
            self.proj_out = Linear(inner, in_channels, dtype=dtype, device=device)
        else:
            self.proj_in = Conv2d(in_channels, inner, 1, dtype=dtype, device=device)
            self.proj_out = Conv2d(inner, in_channels, 1, dtype=dtype, device=device)
        self.transformer_blocks = nn.ModuleList([
            BasicTransformerBlock(inner, n_heads, d_head, context_dim=context_dim[d],
                                  disable_self_attn=disable_self_attn, dtype=dtype, device=device)
            for d in range(depth)])

    def forward(self, x, context=None, transformer_options=None):
        to = transformer_options if transformer_options is not None else {}
        if not isinstance(context, list):
            context = [context] * len(self.transformer_blocks)
        sp = to.get("sp")
        from ..parallel import spatial
        if spatial.current() is not None:
            pass     # row-sharded UNet: x is already this rank's token band; sp does the self-attention
        elif sp is not None and sp.P > 1 and not to.get("patches") and not to.get("patches_replace") \
                and (x.shape[2] * x.shape[3]) % sp.P == 0 and all(bk._plain for bk in self.transformer_blocks):
            return self._forward_sp(x, context, to, sp)
        else:
            to = dict(to, sp=None) if sp is not None else to
        b, c, h, w = x.shape
        x_in = x
        x = self.norm(x)
        if not self.use_linear:
            x = self.proj_in(x)
        # NHWC storage makes this a view on the device
        x = x.permute(0, 2, 3, 1).reshape(b, h * w, -1)
        if self.use_linear:
            x = self.proj_in(x, row_stats=True)       # the first block's LayerNorm reads its statistics partials
        for i, blk in enumerate(self.transformer_blocks):
            to["block_index"] = i
            x = blk(x, context=context[i], transformer_options=to)
        if self.use_linear:
            res = x_in.permute(0, 2, 3, 1).reshape(b, h * w, c)
            if res.is_contiguous():
                x = self.proj_out(x, residual=res)   # fused "+ x_in"
                return x.reshape(b, h, w, c).permute(0, 3, 1, 2)
            x = self.proj_out(x)
            return x.reshape(b, h, w, c).permute(0, 3, 1, 2) + x_in
        x = x.reshape(b, h, w, -1).permute(0, 3, 1, 2)
        return self.proj_out(x, residual=x_in)

    def _forward_sp(self, x, context, to, sp):
        """Token-parallel stack (latency mode): GroupNorm on the full image (replicated), then only
        this rank's contiguous token shard through proj_in, the blocks and proj_out (+ the fused
        residual), then one all-gather of the tokens back into the image."""
        b, c, h, w = x.shape
        T = h * w
        lo, hi = sp.rank * (T // sp.P), (sp.rank + 1) * (T // sp.P)
        x_tok = x.permute(0, 2, 3, 1).reshape(b, T, c)
        n = self.norm(x)
        if not self.use_linear:
            n = self.proj_in(n)
        t = n.permute(0, 2, 3, 1).reshape(b, T, -1)[:, lo:hi].contiguous()
        if self.use_linear:
            t = self.proj_in(t)
        for i, blk in enumerate(self.transformer_blocks):
            to["block_index"] = i
            t = blk(t, context=context[i], transformer_options=to)
        res = x_tok[:, lo:hi].contiguous()
        if self.use_linear:
            t = self.proj_out(t, residual=res)
        else:
            # the 1x1 conv on tokens is the same GEMM
            wgt = self.proj_out.weight.reshape(c, -1).to(device=t.device, dtype=t.dtype)
            bias = None if self.proj_out.bias is None else self.proj_out.bias.to(device=t.device, dtype=t.dtype)
            t = ops.linear(t, wgt, bias, residual=res)
        full = sp.gather(t, dim=1)                          # [b, T, c]
        return full.reshape(b, h, w, c).permute(0, 3, 1, 2)


def refresh_static_kv(model: nn.Module, sources) -> int:
    """Recompute every cross-attention's static K/V buffer of the contexts in ``sources`` (ids of the
    step plan's static context tensors, just refreshed with a new job's conditioning)."""
    n = 0
    for m in model.modules():
        fn = getattr(m, "refresh_static_kv", None)     # CrossAttention; Stable Cascade's stages
        if fn is not None:
            n += fn(sources)
    return n
