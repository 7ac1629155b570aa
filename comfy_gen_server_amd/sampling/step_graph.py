"""One hipGraph per sampler step: UNet(cond ‖ uncond) + CFG combine + Euler(-a) update + noise.

The reference runs the k-diffusion loop in Python, one op at a time
(``comfy/k_diffusion/sampling.py:148-164`` -> ``comfy/samplers.py:234-255`` -> ``model_base.py:74-98``).
Here the whole step body is captured ONCE per plan into a ``torch.cuda.CUDAGraph`` and replayed
for every step of every job with that plan:

  * every per-step scalar lives on the device: a host-built table ``params[step] = (sigma,
    sigma_down, sigma_up, s_noise)`` and ``meta = (step, seed, index0)``; the graph's first kernel
    broadcasts ``sigma`` into the model's sigma vector, its last kernel advances ``meta[0]``;
  * the model sees sigma as a device tensor (c_in scaling, sigma -> timestep, calculate_denoised
    are device ops), so nothing in the forward depends on host values;
  * CFG combine, the Euler / Euler-ancestral update and the ancestral noise (counter-based, keyed
    by (seed, global image index, step) — ``rng.py``) are ONE kernel (``cgs_sampler_step_dev``).

A job then costs: copy x and the conditioning into the plan's static buffers, one 16-B-per-step
parameter upload, and ``steps`` graph launches — no per-step Python op dispatch, no host gaps.

ControlNet (``comfy/controlnet.py:152``, chains included) runs inside the same captured step: its
timestep window is evaluated on the host per step (one graph per distinct on/off pattern of the
chain, usually one), the strength is part of the plan key, and the prepared hint is a static input
refreshed per job.

Eligible (else the eager loop runs): device tensors, Euler / Euler-a (no churn), a seed and
contiguous global image indices, a plain ``CFGGuider`` with one full-frame cond and uncond entry
sharing one ControlNet chain (or none) — no areas / masks / gligen / timestep ranges / T2I adapters,
no denoise mask, no sampler cfg hooks or model wrappers, no transformer patches. ``CGS_GRAPHS=0``
disables it.
"""
from __future__ import annotations

import logging
import math
import os
import threading

import torch

from .. import ops
from ..runtime import graphs
from . import rng

_lock = threading.Lock()
CAPACITY = 1024          # steps per parameter table
stats = {"capture": 0, "replay": 0, "jobs": 0}


class _Plan:
    __slots__ = ("graphs", "x", "params", "meta", "sig", "den", "cond", "hints", "pool", "kv_sources", "kind",
                 "old", "w")


def _ancestral(s0, s1, eta):
    from .k_samplers import get_ancestral_step
    return get_ancestral_step(s0, s1, eta=eta)


def _no(reason):
    """Record why the fused step graph declined a run (bench JSON / ``/metrics``: ``ineligible``); the
    run then goes to the per-step run capture (run_graph.py) or the eager loop."""
    d = stats.setdefault("ineligible", {})
    d[reason] = d.get(reason, 0) + 1
    return None


def _eligible(mk, x, extra_args, record=False):
    from .samplers import CFGGuider, KSamplerX0Inpaint, _simple_conds
    no = _no if record else (lambda reason: None)
    if not graphs.enabled():
        return no("hip graphs disabled")
    if not x.is_cuda or x.dtype != torch.float32 or not x.is_contiguous():
        return no("latent not a contiguous fp32 device tensor")
    try:
        if torch.cuda.is_current_stream_capturing():      # inside a sampler-run capture (run_graph.py)
            return None
    except Exception:
        return None
    if x[0].numel() % 4 or not isinstance(mk, KSamplerX0Inpaint):
        return no("latent shape")
    if extra_args.get("denoise_mask") is not None:
        return no("denoise mask (inpaint)")
    if extra_args.get("seed") is None:
        return no("no seed")
    inds = extra_args.get("noise_inds") or list(range(x.shape[0]))
    index0, contiguous = rng.contiguous_inds(inds)
    if not contiguous or len(inds) != x.shape[0]:
        return no("non-contiguous noise indices")
    guider = mk.inner_model
    if type(guider) is not CFGGuider:
        return no("custom guider")
    mo = extra_args.get("model_options") or {}
    if any(k in mo for k in ("sampler_cfg_function", "sampler_post_cfg_function", "model_function_wrapper",
                             "denoise_mask_function")):
        return no("sampler cfg / post-cfg / wrapper hook")
    to = mo.get("transformer_options", {})
    if to.get("patches") or to.get("patches_replace"):
        return no("transformer patches")
    pos, neg = guider.conds.get("positive"), guider.conds.get("negative")
    use_uncond = not (abs(guider.cfg - 1.0) < 1e-9 and not mo.get("disable_cfg1_optimization", False))
    lists = [pos, neg] if use_uncond else [pos]
    if any(cl is None or len(cl) != 1 for cl in lists) or not _simple_conds(lists):
        return no("area / mask / timestep-range / multi-entry conds")
    if any(cl[0].get("gligen") is not None for cl in lists):
        return no("gligen")
    ctrls = [cl[0].get("control") for cl in lists]
    ctrl = ctrls[0]
    if any(c is not ctrl for c in ctrls):       # cond and uncond must share the control (one batch)
        return no("different controlnets on cond / uncond")
    if ctrl is not None:
        from ..runtime.controlnet import ControlNet
        if any(type(cn) is not ControlNet and not issubclass(type(cn), ControlNet) for cn in _chain(ctrl)):
            return no("t2i adapter / non-controlnet control")   # T2I adapters / others: eager
    return guider, lists, use_uncond, index0, mo, ctrl


def _chain(ctrl):
    out = []
    while ctrl is not None:
        out.append(ctrl)
        ctrl = ctrl.previous_controlnet
    return out


def _conditioning(guider, lists, x, sigma0):
    from .samplers import can_concat_cond, cond_cat, get_area_and_mult
    sig = torch.full((x.shape[0],), sigma0, device=x.device, dtype=torch.float32)
    runs = [get_area_and_mult(cl[0], x, sig, need_mult=False) for cl in lists]
    if len(runs) == 2 and not can_concat_cond(runs[0], runs[1]):
        return None
    return cond_cat([r.conditioning for r in runs])


def try_sample(mk, x, sigmas, extra_args, callback, kind: str, eta: float = 1.0, s_noise: float = 1.0):
    """Run the whole sampling loop from graph replays; None when not eligible (caller runs eager)."""
    el = _eligible(mk, x, extra_args, record=True)
    if el is None:
        return None
    guider, lists, use_uncond, index0, mo, ctrl = el
    s = [float(v) for v in sigmas.detach().cpu()]
    n = len(s) - 1
    if n < 1 or n >= CAPACITY:      # meta[0] counts up to n: keep every read inside the table
        return None
    cond = _conditioning(guider, lists, x, s[0])
    # device tensors, or host scalars that are constant over the run (SVD's num_video_frames): those are
    # part of the plan key and baked into the captured graph
    if cond is None or any(not (isinstance(v, torch.Tensor) and v.is_cuda) and
                           not (isinstance(v, (int, float, bool)) and not isinstance(v, torch.Tensor))
                           for v in cond.values()):
        return None
    model = guider.inner_model
    # floating conds in the model's compute dtype up front: apply_model's .to(dtype) is then the
    # identity, so the UNet sees the plan's static tensors themselves (static K/V keys on them)
    try:
        mdt = model.manual_cast_dtype or model.get_dtype()
        cond = {k: (v.to(mdt) if torch.is_tensor(v) and v.is_floating_point() and k in _STATIC_CAST else v)
                for k, v in cond.items()}
    except Exception:
        pass
    chain = _chain(ctrl)
    batched = 2 if use_uncond else 1
    # ControlNet: the per-step on/off window is decided on the HOST (one captured graph per distinct
    # on/off pattern of the chain), the hint is a static input, strength is part of the plan key
    patterns = [tuple(not cn.outside_window_at(s[i]) for cn in chain) for i in range(n)]
    hints = []
    if chain:
        xin = torch.empty((x.shape[0] * batched,) + tuple(x.shape[1:]), device=x.device, dtype=x.dtype)
        hints = [cn.prepare_hint(xin, batched) for cn in chain]
    from ..models import layers
    epoch = layers.module_epoch(model)
    key = (epoch, kind == "dpmpp_2m", tuple(x.shape), use_uncond, float(guider.cfg),
           tuple(sorted((k, tuple(v.shape), v.dtype) if torch.is_tensor(v) else (k, "scalar", v)
                        for k, v in cond.items())),
           tuple((id(cn.control_model), layers.module_epoch(cn.control_model), float(cn.strength),
                  bool(cn.global_average_pooling), tuple(h.shape), h.dtype) for cn, h in zip(chain, hints)))
    plans = model.__dict__.setdefault("_step_graph_plans", {})
    plan = plans.get(key)
    if plan is None:
        plan = _new_plan(x, cond, hints)
        plan.kind = "dpmpp_2m" if kind == "dpmpp_2m" else "euler"
        with _lock:
            for k in [k for k in plans if k[0] != epoch]:
                del plans[k]
            plans[key] = plan
    for pat in sorted(set(patterns)):
        if pat not in plan.graphs:
            rep = s[patterns.index(pat)]
            g = _capture(plan, model, chain, pat, rep, use_uncond, float(guider.cfg), mo)
            if g is None:
                return None
            plan.graphs[pat] = g
    # per-job inputs
    rows = []
    for i in range(n):
        if kind == "dpmpp_2m":
            # DPM++ 2M (k_samplers.sample_dpmpp_2m) is the Euler update x' = (s'/s) x + (1 - s'/s) d applied
            # to d = den + w (den - den_prev), w = 1 / (2 r) with r = h_last / h (0 on the first and last
            # steps); column 3 carries w (no noise: sigma_up = 0)
            w = 0.0
            if i > 0 and s[i + 1] > 0:
                h = math.log(s[i]) - math.log(s[i + 1])
                h_last = math.log(s[i - 1]) - math.log(s[i])
                w = 1.0 / (2.0 * (h_last / h))
            rows.append((s[i], s[i + 1], 0.0, w))
            continue
        if kind == "lcm":
            # LCM (k_samplers.sample_lcm): x' = den + s' * noise == the Euler-a kernel with sigma_down = 0,
            # sigma_up = s', s_noise = 1 (same per-step noise stream as the eager loop)
            rows.append((s[i], 0.0, s[i + 1], 1.0))
            continue
        if kind == "euler_ancestral":
            down, up = _ancestral(s[i], s[i + 1], eta)
            if s[i + 1] <= 0:
                up = 0.0
        else:
            down, up = s[i + 1], 0.0
        rows.append((s[i], down, up, s_noise))
    plan.params[:n].copy_(torch.tensor(rows, dtype=torch.float32))
    plan.meta.copy_(torch.tensor([0, int(extra_args["seed"]) & 0x7FFFFFFFFFFFFFFF, index0], dtype=torch.int64))
    plan.x.copy_(x)
    if plan.old is not None:
        plan.old.zero_()
    for k, v in cond.items():
        if torch.is_tensor(v):
            plan.cond[k].copy_(v)
    if plan.kv_sources:
        # the run's constant context -> every cross-attention K/V once per job (the captured steps
        # read the buffers instead of recomputing them each step)
        from ..models.attention import refresh_static_kv
        stats["kv_refresh"] = stats.get("kv_refresh", 0) + refresh_static_kv(model.diffusion_model, plan.kv_sources)
    for dst, src in zip(plan.hints, hints):
        if dst is not src:
            dst.copy_(src)
    stats["jobs"] += 1
    for i in range(n):
        x_pre = plan.x.clone() if callback is not None else None   # the eager loops report x before the update
        plan.graphs[patterns[i]].replay()
        stats["replay"] += 1
        if callback is not None:
            callback({"x": x_pre, "i": i, "sigma": s[i], "sigma_hat": s[i], "denoised": plan.den.clone()})
    return plan.x.clone()


# conds apply_model casts to the compute dtype anyway (not c_concat: that one follows x's dtype)
_STATIC_CAST = ("c_crossattn", "y", "clip_text", "clip_text_pooled", "clip_img", "clip", "effnet")


def _new_plan(x, cond, hints):
    p = _Plan()
    dev = x.device
    p.x = x.detach().clone()
    p.params = torch.zeros((CAPACITY, 4), device=dev, dtype=torch.float32)
    p.params[:, 0] = 1.0
    p.meta = torch.zeros(3, device=dev, dtype=torch.int64)
    p.sig = torch.empty(x.shape[0], device=dev, dtype=torch.float32)
    p.den = torch.empty_like(p.x)
    p.cond = {k: (v.detach().clone() if torch.is_tensor(v) else v) for k, v in cond.items()}
    # static cross-attention K/V over the plan's context buffers (CGS_STATIC_KV=0 disables)
    p.kv_sources = frozenset(id(v) for v in p.cond.values() if torch.is_tensor(v)) \
        if os.environ.get("CGS_STATIC_KV", "1") != "0" \
        else frozenset()
    p.hints = list(hints)           # the first job's prepared hint tensors become the static inputs
    p.graphs = {}
    p.pool = None
    p.kind = "euler"
    p.old = torch.zeros_like(p.x)          # DPM++ 2M: previous step's denoised
    p.w = torch.zeros(1, device=dev, dtype=torch.float32)
    return p


def _capture(p, model, chain, pattern, rep_sigma, use_uncond, cfg, mo):
    """Capture the step body for one ControlNet on/off pattern (``rep_sigma``: a step's sigma with
    that pattern, published as the host sigma while the body records)."""
    from .samplers import current_sigma
    to = dict(mo.get("transformer_options", {}))
    to["cond_or_uncond"] = [0, 1] if use_uncond else [0]
    for cn, h in zip(chain, p.hints):
        cn.cond_hint = h            # get_control() then reads the plan's static hint

    def body(kv_mode):
        ops.step_param(p.sig, p.params, p.meta, 0)
        if use_uncond:
            xin, tin = torch.cat([p.x, p.x]), torch.cat([p.sig, p.sig])
        else:
            xin, tin = p.x, p.sig
        t = dict(to)
        t["sigmas"] = p.sig
        if p.kv_sources:
            t["kv_static"] = (kv_mode, p.kv_sources)
        control = None
        if chain:
            control = chain[0].get_control(xin, tin, p.cond, 2 if use_uncond else 1)
        out = model.apply_model(xin, tin, control=control, transformer_options=t, **p.cond)
        if p.kind == "dpmpp_2m":
            if use_uncond:
                oc, ou = out.chunk(2)
                p.den.copy_(ops.cfg_combine(oc.float().contiguous(), ou.float().contiguous(), cfg))
            else:
                p.den.copy_(out)
            ops.step_param(p.w, p.params, p.meta, 3)
            d = torch.addcmul(p.den, p.w, p.den - p.old)
            ops.sampler_step_dev(p.x, d, None, None, 1.0, p.params, p.meta)
            p.old.copy_(p.den)
        elif use_uncond:
            oc, ou = out.chunk(2)
            ops.sampler_step_dev(p.x, oc.contiguous(), ou.contiguous(), p.den, cfg, p.params, p.meta)
        else:
            ops.sampler_step_dev(p.x, out.contiguous(), None, p.den, 1.0, p.params, p.meta)
        ops.step_advance(p.meta)

    g = torch.cuda.CUDAGraph()
    tok = current_sigma.set(float(rep_sigma))
    saved_x, saved_meta = p.x.clone(), p.meta.clone()
    p.meta[0] = 0                   # a previous job left meta[0] = its step count: warm-up reads row 0
    try:
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            body("fill")                # warm-up: autotune keys, derived weight layouts, lazy attrs, K/V buffers
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        if p.pool is None:
            p.pool = torch.cuda.graph_pool_handle()
        with torch.cuda.graph(g, pool=p.pool, stream=side):
            body("use")
        torch.cuda.synchronize()
    except Exception as e:  # capture-unsafe op in the step: this plan stays eager
        stats["capture_failed"] = stats.get("capture_failed", 0) + 1
        logging.warning("step hipGraph capture failed (%s); sampling stays eager", e,
                        exc_info=os.environ.get("CGS_GRAPH_DEBUG", "0") == "1")
        try:
            torch.cuda.synchronize()
        except Exception:
            pass
        return None
    finally:
        current_sigma.reset(tok)
        p.x.copy_(saved_x)
        p.meta.copy_(saved_meta)
    stats["capture"] += 1
    return g
