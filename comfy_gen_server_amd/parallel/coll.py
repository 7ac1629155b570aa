"""The collectives the model-parallel paths issue inside a UNet call (latency mode: parallel/spatial.py,
parallel/sp.py, parallel/latency.py), with one extra case: device tensors on a Gloo group.

On a node every rank owns a GPU and the group is RCCL: the calls go straight to ``torch.distributed``.
Gloo has no device send / recv / all-to-all, so when a group is Gloo and the tensors live on the GPU --
the shared-GPU rehearsal (``CGS_SHARED_GPU=1``: several ranks on ONE card, e.g. the 1-GPU development
box) -- the payload is staged through host memory (16-bit floats travel as fp32, exactly). The
model code is the same in both cases, so a multi-rank latency-mode run on one GPU exercises the exact
halo / statistics / sequence-parallel call sequence the 8-GPU node runs over RCCL.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def _staged(t: torch.Tensor, group) -> bool:
    return t.is_cuda and dist.get_backend(group) == "gloo"


def _host(t: torch.Tensor) -> torch.Tensor:
    h = t.detach().contiguous().cpu()
    return h.float() if h.dtype in (torch.bfloat16, torch.float16) else h    # exact; Gloo lacks 16-bit types


def _host_empty(t: torch.Tensor) -> torch.Tensor:
    dt = torch.float32 if t.dtype in (torch.bfloat16, torch.float16) else t.dtype
    return torch.empty(t.shape, dtype=dt)


def _back(dst: torch.Tensor, h: torch.Tensor):
    dst.copy_(h)


def all_gather(parts, t: torch.Tensor, group=None):
    if not _staged(t, group):
        dist.all_gather(parts, t, group=group)
        return
    hp = [_host_empty(p) for p in parts]
    dist.all_gather(hp, _host(t), group=group)
    for p, h in zip(parts, hp):
        _back(p, h)


def all_to_all_single(out: torch.Tensor, inp: torch.Tensor, group=None):
    if not _staged(inp, group):
        dist.all_to_all_single(out, inp, group=group)
        return
    ho = _host_empty(out)
    dist.all_to_all_single(ho, _host(inp), group=group)
    _back(out, ho)


class _Done:
    def wait(self):
        return True


def exchange(sends, recvs, group=None):
    """Point-to-point round: ``sends`` [(tensor, global peer rank)], ``recvs`` [(buffer, peer)]. Returns
    the requests to wait on (the receive buffers are filled once they completed)."""
    if not sends and not recvs:
        return []
    probe = (sends or recvs)[0][0]
    if not _staged(probe, group):
        ops = [dist.P2POp(dist.isend, t, p, group) for t, p in sends] + \
              [dist.P2POp(dist.irecv, b, p, group) for b, p in recvs]
        return dist.batch_isend_irecv(ops)
    hs = [(_host(t), p) for t, p in sends]
    hr = [(_host_empty(b), b, p) for b, p in recvs]
    ops = [dist.P2POp(dist.isend, h, p, group) for h, p in hs] + [dist.P2POp(dist.irecv, h, p, group) for h, _, p in hr]
    for req in dist.batch_isend_irecv(ops):
        req.wait()
    for h, b, _ in hr:
        _back(b, h)
    return [_Done()]
