"""hipGraph capture / replay of the denoiser forward (SURVEY §7.1 'static batch/shape plans').

The reference re-dispatches every UNet op from Python on every sampler step
(``comfy/model_base.py:74-98`` -> ``openaimodel.py:819-890``). Here the diffusion model's forward
for a fixed (shapes, dtypes, weights) plan is captured once into a ``torch.cuda.CUDAGraph`` (a
hipGraph on ROCm) and replayed for every later step and job with the same plan: ~1.5k kernel
launches collapse into one graph launch, so the host never limits the GPU, even at batch 1.

Plan lifecycle:
  * 1st call of a plan: eager (per-shape kernel autotuning, lazy kernel attributes and the derived
    weight layouts -- fused QKV, interleaved GEGLU, NHWC conv weights -- all happen here);
  * 2nd call: capture into a private memory pool, then replay;
  * later calls: copy the inputs into the static buffers, replay, clone the output.
A plan is only graphed when nothing dynamic can reach the forward: no ControlNet residuals, no
``transformer_options`` patches / replacements (their Python hooks run per step), CUDA tensors.
Weight patching (LoRA merge / unpatch) or a device move stamps a new epoch on that model's module
tree (``models.layers.stamp_epoch``), which retires the plans captured over it (the graph holds raw
pointers to the old weight buffers); other models' plans stay (Cascade Stage C / B alternate).
Disable with ``CGS_GRAPHS=0``.
"""
from __future__ import annotations

import logging
import os
import threading

import torch

_lock = threading.Lock()


def enabled() -> bool:
    return os.environ.get("CGS_GRAPHS", "1") != "0"


def _sig(t):
    if t is None:
        return None
    if isinstance(t, torch.Tensor):
        return (tuple(t.shape), t.dtype, t.device)
    return ("const", t)


class _Plan:
    __slots__ = ("graph", "inputs", "out", "kw_static")


class GraphedForward:
    """Wraps ``module.forward(x, timesteps, context=, y=, control=, transformer_options=, **kw)``."""

    MAX_PLANS = 8

    def __init__(self, module):
        self.module = module
        self.plans: dict = {}
        self.seen: dict = {}
        self.failed: set = set()
        self.pool = None
        self.stats = {"eager": 0, "capture": 0, "replay": 0}

    # ------------------------------------------------------------------------------------------
    def _eligible(self, x, control, to, kw):
        if not enabled() or not x.is_cuda or control is not None:
            return False
        if to and (to.get("patches") or to.get("patches_replace") or to.get("sp") is not None):
            return False            # Python hooks / latency-mode collectives run eagerly
        for v in kw.values():
            if isinstance(v, torch.Tensor) and not v.is_cuda:
                return False
        try:
            if torch.cuda.is_current_stream_capturing():
                return False
        except Exception:
            return False
        return True

    def _key(self, x, timesteps, context, y, kw):
        from ..models import layers
        return (layers.module_epoch(self.module), _sig(x), _sig(timesteps), _sig(context), _sig(y),
                tuple(sorted((k, _sig(v)) for k, v in kw.items())))

    def _eager(self, x, timesteps, context, y, control, to, kw):
        self.stats["eager"] += 1
        return self.module(x, timesteps, context=context, y=y, control=control,
                           transformer_options=to if to is not None else {}, **kw)

    def __call__(self, x, timesteps=None, context=None, y=None, control=None, transformer_options=None, **kw):
        if not self._eligible(x, control, transformer_options, kw):
            return self._eager(x, timesteps, context, y, control, transformer_options, kw)
        key = self._key(x, timesteps, context, y, kw)
        plan = self.plans.get(key)
        if plan is None:
            if key in self.failed:
                return self._eager(x, timesteps, context, y, control, transformer_options, kw)
            n = self.seen.get(key, 0) + 1
            self.seen[key] = n
            if n < 2:
                return self._eager(x, timesteps, context, y, control, transformer_options, kw)
            plan = self._capture(key, x, timesteps, context, y, transformer_options, kw)
            if plan is None:
                return self._eager(x, timesteps, context, y, control, transformer_options, kw)
        for dst, src in zip(plan.inputs, (x, timesteps, context, y)):
            if dst is not None:
                dst.copy_(src, non_blocking=True)
        for k, dst in plan.kw_static.items():
            if isinstance(dst, torch.Tensor):
                dst.copy_(kw[k], non_blocking=True)
        plan.graph.replay()
        self.stats["replay"] += 1
        return plan.out.clone()

    # ------------------------------------------------------------------------------------------
    def _capture(self, key, x, timesteps, context, y, to, kw):
        from ..models import layers
        with _lock:
            # plans captured under an older weight epoch hold stale pointers: drop them
            for k in [k for k in self.plans if k[0] != layers.module_epoch(self.module)]:
                del self.plans[k]
            if len(self.plans) >= self.MAX_PLANS:
                self.plans.pop(next(iter(self.plans)))
            if self.pool is None:
                self.pool = torch.cuda.graph_pool_handle()
            plan = _Plan()
            clone = (lambda t: None if t is None else t.detach().clone())
            plan.inputs = (clone(x), clone(timesteps), clone(context), clone(y))
            plan.kw_static = {k: (v.detach().clone() if isinstance(v, torch.Tensor) else v) for k, v in kw.items()}
            sx, st, sc, sy = plan.inputs
            to_static = {k: v for k, v in (to or {}).items() if k not in ("sigmas",)}
            g = torch.cuda.CUDAGraph()
            try:
                # warm-up on the capture stream (library workspaces are per stream), then capture
                side = torch.cuda.Stream()
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    self.module(sx, st, context=sc, y=sy, control=None,
                                transformer_options=dict(to_static), **plan.kw_static)
                torch.cuda.current_stream().wait_stream(side)
                torch.cuda.synchronize()
                with torch.cuda.graph(g, pool=self.pool, stream=side):
                    out = self.module(sx, st, context=sc, y=sy, control=None,
                                      transformer_options=dict(to_static), **plan.kw_static)
                torch.cuda.synchronize()
            except Exception as e:  # capture-unsafe op somewhere in the forward: stay eager for this plan
                logging.warning("hipGraph capture failed (%s); plan stays eager", e)
                self.failed.add(key)
                try:
                    torch.cuda.synchronize()
                except Exception:
                    pass
                return None
            plan.graph = g
            plan.out = out
            self.plans[key] = plan
            self.stats["capture"] += 1
            return plan

    def reset(self):
        with _lock:
            self.plans.clear()
            self.seen.clear()
            self.failed.clear()
