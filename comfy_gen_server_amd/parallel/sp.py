"""Sequence-parallel attention across the GPUs of a node (SURVEY §2.5 SP / Ulysses / ring rows,
§5.7, §5.8 R4-R5). The reference has no multi-device sequence parallelism; these are the optional
latency-mode building blocks for one very large image (B = 1, >= 2048² latents, VAE mid attention
at 64 k tokens) where data parallelism has nothing to split.

Both take the *local* sequence shard of q / k / v — [B, S / P, H * D] on each of the P ranks of
``group``, shards in rank order — and return the local shard of the attention output.

* ``ulysses_attention`` (R4): one all-to-all turns sequence shards into head shards
  ([B, S, H / P * D]), every rank runs the single-GPU flash kernel (``ops.attention``) on its
  heads over the whole sequence, a second all-to-all turns the result back. Two all-to-alls of
  the activations per attention; needs H % P == 0. On xGMI every pair of GPUs has its own link,
  so the all-to-all runs at full per-link bandwidth (no ring hops).
* ``ring_attention`` (R5): K/V shards travel around the ring (send to rank + 1, receive from
  rank - 1, overlapped with the partial attention of the block in hand); partial results are
  merged with their log-sum-exp. Works for any head count including the single-head VAE
  attention; memory per rank stays O(S / P).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from .. import ops
from . import coll


def _world(group):
    return dist.get_world_size(group), dist.get_rank(group)


def _all_to_all(chunks, group):
    """chunks: list of P same-shape tensors (chunk p goes to rank p) -> list received (from rank p).
    One ``all_to_all_single`` over the stacked chunks (supported by RCCL and Gloo alike)."""
    inp = torch.stack(chunks).contiguous()
    out = torch.empty_like(inp)
    coll.all_to_all_single(out, inp, group=group)
    return list(out.unbind(0))


def ulysses_attention(q, k, v, heads: int, group=None):
    P, _ = _world(group)
    if P == 1:
        return ops.attention(q, k, v, heads)
    if heads % P:
        raise ValueError(f"ulysses_attention: {heads} heads not divisible by {P} ranks")
    B, Sl, HD = q.shape
    D = HD // heads
    hp = heads // P

    def seq_to_heads(t):
        # [B, Sl, H*D] -> send head block p to rank p -> [B, P*Sl, hp*D] (sequence in rank order)
        parts = [c.contiguous() for c in t.view(B, Sl, P, hp * D).unbind(2)]
        got = _all_to_all(parts, group)
        return torch.cat(got, dim=1)

    qh, kh, vh = seq_to_heads(q), seq_to_heads(k), seq_to_heads(v)
    o = ops.attention(qh, kh, vh, hp)                      # [B, S, hp*D]
    back = _all_to_all([c.contiguous() for c in o.split(Sl, dim=1)], group)   # from rank p: its heads
    return torch.stack(back, dim=2).reshape(B, Sl, HD)


def _partial_attention(q, k, v, heads):
    """Partial attention of q against one K/V block: (o fp32 [B, Sq, H, D], lse fp32 [B, Sq, H, 1]).
    The HIP flash kernels produce both in one pass (``ops.attention_lse``); the scores never exist."""
    B, Sq, HD = q.shape
    o, lse = ops.attention_lse(q, k, v, heads)
    return o.float().view(B, Sq, heads, HD // heads), lse.transpose(1, 2).unsqueeze(-1)


def ring_attention(q, k, v, heads: int, group=None):
    P, r = _world(group)
    if P == 1:
        return ops.attention(q, k, v, heads)
    B, Sl, HD = q.shape
    ranks = dist.get_process_group_ranks(group) if group is not None else list(range(P))
    nxt, prv = ranks[(r + 1) % P], ranks[(r - 1) % P]
    kv = torch.cat([k, v], dim=-1).contiguous()
    o_acc, lse_acc = None, None
    for step in range(P):
        reqs = []
        if step < P - 1:                                    # overlap: ship the block while computing on it
            recv = torch.empty_like(kv)
            reqs = coll.exchange([(kv, nxt)], [(recv, prv)], group)
        o, lse = _partial_attention(q, kv[..., :HD], kv[..., HD:], heads)
        if o_acc is None:
            o_acc, lse_acc = o, lse
        else:                                               # log-sum-exp merge of the two partials
            m = torch.maximum(lse_acc, lse)
            wa, wb = torch.exp(lse_acc - m), torch.exp(lse - m)
            o_acc = (o_acc * wa + o * wb) / (wa + wb)
            lse_acc = m + torch.log(wa + wb)
        for req in reqs:
            req.wait()
        if step < P - 1:
            kv = recv
    return o_acc.reshape(B, Sl, HD).to(q.dtype)


def shard_sequence(x, group=None, dim=1):
    """This rank's contiguous shard of ``x`` along ``dim`` (sequence length divisible by P)."""
    P, r = _world(group)
    return x.chunk(P, dim=dim)[r].contiguous()


def gather_sequence(x, group=None, dim=1):
    """Inverse of ``shard_sequence``: all-gather the shards back into the full sequence."""
    P, _ = _world(group)
    if P == 1:
        return x
    parts = [torch.empty_like(x) for _ in range(P)]
    coll.all_gather(parts, x.contiguous(), group=group)
    return torch.cat(parts, dim=dim)


def kv_gather_attention(q, k, v, heads: int, group=None):
    """Local query shard against the all-gathered keys/values (one all-gather of K and V, then the
    single-GPU flash kernel on [B, S/P] x [B, S] -- any head count; the choice when heads % P != 0,
    e.g. SDXL's 10-head level-1 blocks on 4 ranks)."""
    P, _ = _world(group)
    if P == 1:
        return ops.attention(q, k, v, heads)
    kv = gather_sequence(torch.cat([k, v], dim=-1), group)
    HD = q.shape[-1]
    return ops.attention(q, kv[..., :HD], kv[..., HD:], heads)


class SeqParallel:
    """Token (sequence) parallelism of the UNet's transformer stacks over ``group`` (latency mode,
    ``parallel/latency.py``): a SpatialTransformer keeps only its rank's contiguous token shard
    through LayerNorm / QKV / FF / projections; self-attention exchanges through ``attention``
    (Ulysses all-to-all when the heads divide over the ranks, else the K/V all-gather form);
    cross-attention needs nothing (the text context is replicated); the stack output is
    all-gathered back to the full image for the (replicated) ResBlocks."""

    def __init__(self, group=None):
        self.group = group
        self.P, self.rank = _world(group)
        self.mode = os.environ.get("CGS_SP_ATTN", "auto")   # auto | ulysses | kvgather | ring
        self.stats = {"ulysses": 0, "kvgather": 0, "ring": 0}

    def attention(self, q, k, v, heads: int):
        if self.mode == "ring":
            self.stats["ring"] += 1
            return ring_attention(q, k, v, heads, self.group)
        if self.mode != "kvgather" and heads % self.P == 0:
            self.stats["ulysses"] += 1
            return ulysses_attention(q, k, v, heads, self.group)
        self.stats["kvgather"] += 1
        return kv_gather_attention(q, k, v, heads, self.group)

    def shard(self, x, dim=1):
        return shard_sequence(x, self.group, dim)

    def gather(self, x, dim=1):
        return gather_sequence(x, self.group, dim)
