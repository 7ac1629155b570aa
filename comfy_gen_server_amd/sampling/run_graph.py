"""Whole sampler runs replayed from hipGraphs: any k-diffusion / UniPC sampler, CFG batching, area / mask /
timestep-range conds and model patches (FreeU, SAG, PAG, HyperTile, ToMe, Kohya deep-shrink, ...).

The reference runs its sampler loops in Python (``comfy/k_diffusion/sampling.py:127-757``,
``comfy/extra_samplers/uni_pc.py``): per step, hundreds of UNet ops plus the update are dispatched from
the host. ``step_graph.py`` replays ONE graph for every step of the samplers whose update it has as a
device-parameterised kernel (Euler, Euler-a, DPM++ 2M, LCM). This module covers everything else with a
different mechanism: the sampler function itself runs under stream capture, cut into ONE GRAPH PER STEP
at its progress callback; every host-side quantity of the run (sigmas, ancestral steps, multistep
coefficients, timestep-range gates, patch hyper-parameters) is baked into the kernel arguments, so a
plan is keyed by exactly those values (the sigma schedule, the sampler and its options, the cond
structure, the patch callables and the model's weight epoch).

Per job the static inputs are refreshed in place -- the initial latent, the conditioning tensors of
every cond entry, the inpaint latent / noise / mask -- and the per-image noise key: draws keyed by
(seed, global image index) (``rng.py``: Philox ancestral / SDE noise, the virtual Brownian tree) read
the seed and first index from a device tensor while the run is captured (``ops.rng_key_scope``), so a
replay with another seed produces that seed's noise. The graphs then replay back to back; after graph
i the progress callback of the eager loop runs with that step's x / denoised (previews included).

ControlNet chains (any sampler) run inside the captured steps with their original hints as static inputs;
GLIGEN position conditioning is part of the plan key (its per-box tensors are memoised on the eager run).

Plan life cycle: the first run of a key is eager (autotune, lazy layouts), the second captures then
replays, later runs replay. A capture that hits a host sync or an unsupported op marks the key failed
(eager from then on; ``stats["ineligible"]`` counts every reason). ``CGS_RUN_GRAPHS=0`` disables.
"""
from __future__ import annotations

import logging
import os
import threading
from collections import OrderedDict

import torch

from .. import ops
from ..runtime import graphs

_lock = threading.Lock()
stats: dict = {"capture": 0, "replay_runs": 0, "replay_steps": 0, "capture_failed": 0, "ineligible": {}}
MAX_PLANS = 6
_seen: set = set()
_failed: set = set()


def enabled() -> bool:
    return graphs.enabled() and os.environ.get("CGS_RUN_GRAPHS", "1") != "0"


def _ineligible(reason: str):
    d = stats["ineligible"]
    d[reason] = d.get(reason, 0) + 1
    return None


# ------------------------------------------------------------------------------------------------
# static inputs: every tensor a run reads from outside, in a deterministic order, plus a structural key
# ------------------------------------------------------------------------------------------------
def _walk(obj, tensors, sig, depth=0):
    from .conds import CONDRegular
    if depth > 8:
        raise TypeError("cond structure too deep")
    if torch.is_tensor(obj):
        tensors.append(obj)
        sig.append(("T", tuple(obj.shape), obj.dtype, obj.device.type))
    elif isinstance(obj, dict):
        sig.append(("D", len(obj)))
        for k in sorted(obj, key=str):
            sig.append(("k", str(k)))
            _walk(obj[k], tensors, sig, depth + 1)
    elif isinstance(obj, (list, tuple)):
        sig.append(("L", len(obj)))
        for v in obj:
            _walk(v, tensors, sig, depth + 1)
    elif isinstance(obj, CONDRegular):
        sig.append(("C", type(obj).__name__))
        _walk(obj.cond, tensors, sig, depth + 1)
    elif obj is None or isinstance(obj, (bool, int, float, str)):
        sig.append(("V", obj))
    else:
        raise TypeError(f"unsupported cond value {type(obj).__name__}")


def _control_chain(c):
    out = []
    while c is not None:
        out.append(c)
        c = c.previous_controlnet
    return out


def _control_inputs(ctrl, tensors, sig):
    """A ControlNet chain inside a captured run: each net's ORIGINAL hint is a static input (the
    resize / cast / batch broadcast that get_control() does on first use is captured with the step it
    first runs in, reading that static tensor, so every replay rebuilds the hint of its own job); the
    net, its weights, strength, window and pooling are part of the plan key (the window gates per
    step on host sigmas, which the key already fixes)."""
    from ..models import layers
    from ..runtime.controlnet import ControlNet
    for cn in _control_chain(ctrl):
        if type(cn) is not ControlNet or not torch.is_tensor(cn.cond_hint_original):
            raise TypeError(f"control {type(cn).__name__} (only plain ControlNet chains are captured)")
        if cn.cond_hint is not None:   # a cached hint from an earlier run would be read, not rebuilt
            raise TypeError("controlnet hint already prepared")
        sig.append(("CN", id(cn.control_model), layers.module_epoch(cn.control_model), float(cn.strength),
                    tuple(cn.timestep_percent_range), bool(cn.global_average_pooling), cn.upscale_algorithm,
                    cn.compression_ratio))
        _walk(cn.cond_hint_original, tensors, sig)


def _gligen_key(g, sig):
    """GLIGEN position conditioning: the model and its boxes / phrase embeddings are part of the plan key
    (Gligen.set_position memoises its device tensors per key, built on the eager first run)."""
    kind, model, params = g[0], g[1], (g[2] if len(g) > 2 else [])
    sig.append(("G", kind, id(model), tuple((id(p[0]),) + tuple(float(v) for v in p[1:]) for p in params)))


def _static_inputs(guider, mk, x, extra_args):
    tensors, sig = [], []
    _walk(x, tensors, sig)
    _walk(mk.latent_image, tensors, sig)
    _walk(mk.noise if extra_args.get("denoise_mask") is not None else None, tensors, sig)
    _walk(extra_args.get("denoise_mask"), tensors, sig)
    conds = {}
    for name, cl in (guider.conds or {}).items():
        if cl is None:
            continue
        conds[name] = [{k: v for k, v in c.items() if k not in ("control", "gligen")} for c in cl]
    _walk(conds, tensors, sig)
    for name in sorted(guider.conds or {}, key=str):
        for c in guider.conds[name] or []:
            if c.get("control") is not None:
                _control_inputs(c["control"], tensors, sig)
            if c.get("gligen") is not None:
                _gligen_key(c["gligen"], sig)
    return tensors, tuple(sig)


def _options_key(mo):
    """Identity of every hook in model_options (closures hold their own state: same object = same run)."""
    out = []
    for k in sorted(mo, key=str):
        v = mo[k]
        if k == "transformer_options":
            for tk in sorted(v, key=str):
                tv = v[tk]
                if isinstance(tv, dict):
                    out.append((tk, tuple((str(a), tuple(id(f) for f in (b if isinstance(b, list) else [b])))
                                          for a, b in sorted(tv.items(), key=lambda t: str(t[0])))))
                elif callable(tv) or torch.is_tensor(tv):
                    out.append((tk, id(tv)))
                else:
                    out.append((tk, repr(tv)[:200]))
        elif callable(v):
            out.append((k, id(v)))
        elif isinstance(v, list):
            out.append((k, tuple(id(f) for f in v)))
        else:
            out.append((k, repr(v)[:200]))
    return tuple(out)


class _Plan:
    __slots__ = ("graphs", "records", "static", "key_t", "out", "pool", "keepalive")


def _specialised(fn, mk, x, extra_args) -> bool:
    """The fused device-parameterised step graph (step_graph.py) serves this run."""
    from . import k_samplers, step_graph
    if fn not in (k_samplers.sample_euler, k_samplers.sample_euler_ancestral, k_samplers.sample_dpmpp_2m,
                  k_samplers.sample_lcm):
        return False
    return step_graph._eligible(mk, x, extra_args) is not None


def try_run(ksampler, guider, mk, x, sigmas, extra_args, callback):
    """Run ``ksampler.sampler_function`` from per-step hipGraphs; None -> the caller runs it eagerly."""
    from . import k_samplers, rng
    from .samplers import CFGGuider
    if not enabled() or not x.is_cuda or x.dtype != torch.float32:
        return None
    try:
        if torch.cuda.is_current_stream_capturing():
            return None
    except Exception:
        return None
    from ..sched import spmd
    ctx = spmd.active()
    if ctx is not None and ctx.mode == "latency":
        # The UNet call's collectives (CFG all-gather, halo send / recv, GroupNorm statistics) are RCCL ops
        # on the capturing stream, which RCCL records into the graph. Opt-in: every rank of the group must
        # make the same capture / replay decision, and a capture failure on one rank would leave the others
        # inside a captured collective -- CGS_LATENCY_GRAPHS=1 once a node has been validated with it.
        if os.environ.get("CGS_LATENCY_GRAPHS") != "1" or getattr(ctx.comm, "backend", None) != "nccl":
            return _ineligible("latency mode (collectives inside the UNet call; CGS_LATENCY_GRAPHS=1 captures them)")
    fn = ksampler.sampler_function
    if getattr(fn, "__name__", "") in ("sample_dpm_fast", "sample_dpm_adaptive", "fn"):
        return _ineligible("adaptive step size (host-side error control)")
    if _specialised(fn, mk, x, extra_args):
        return None
    if not isinstance(guider, CFGGuider):
        return _ineligible("custom guider")
    seed = extra_args.get("seed")
    if seed is None:
        return _ineligible("no seed")
    inds = extra_args.get("noise_inds") or list(range(x.shape[0]))
    index0, contiguous = rng.contiguous_inds(inds)
    if not contiguous or len(inds) != x.shape[0]:
        return _ineligible("non-contiguous noise indices")
    try:
        tensors, sig = _static_inputs(guider, mk, x, extra_args)
    except TypeError as e:
        return _ineligible(str(e))
    if any(not t.is_cuda for t in tensors):
        return _ineligible("host tensor in the conditioning")
    from ..models import layers
    model = guider.inner_model
    mo = extra_args.get("model_options") or {}
    s = [float(v) for v in sigmas.detach().cpu()]
    key = (id(fn), repr(sorted(ksampler.extra_options.items())), tuple(s), sig, float(guider.cfg),
           _options_key(mo), layers.module_epoch(model), id(model))
    plans: OrderedDict = model.__dict__.setdefault("_run_graph_plans", OrderedDict())
    plan = plans.get(key)
    if plan is None:
        if key in _failed:
            return None
        if key not in _seen:          # first run of this plan: eager (warms autotune / lazy layouts)
            _seen.add(key)
            return None
        plan = _capture(ksampler, mk, x, sigmas, extra_args, tensors, int(seed), index0)
        if plan is None:
            _failed.add(key)
            return None
        with _lock:
            plans[key] = plan
            while len(plans) > MAX_PLANS:
                plans.popitem(last=False)
        stats["capture"] += 1
    else:
        plans.move_to_end(key)
        for dst, src in zip(plan.static, tensors):
            if dst is not src:
                dst.copy_(src)
    plan.key_t.copy_(torch.tensor([int(seed) & 0x7FFFFFFFFFFFFFFF, index0], dtype=torch.int64))
    for g, rec in zip(plan.graphs, plan.records + [None]):
        if g is not None:             # None: a segment that captured no work (nothing to replay)
            g.replay()
        stats["replay_steps"] += 1
        if rec is not None and callback is not None:
            callback(dict(rec))
    stats["replay_runs"] += 1
    return plan.out.clone()


_graveyard: list = []


def _abort_capture(stream):
    """End a capture an exception left open on ``stream`` (native hipStreamEndCapture)."""
    from .. import _native
    lib = _native.load_kernels()
    if lib is not None and _native.has_kernel("cgs_abort_stream_capture"):
        if lib.cgs_abort_stream_capture(stream.cuda_stream) > 0:
            logging.warning("ended a stream capture left open by the failed sampler-run capture")


def _capture(ksampler, mk, x, sigmas, extra_args, tensors, seed, index0):
    """Capture the run with THIS job's tensors as the static inputs (the plan keeps them alive)."""
    p = _Plan()
    p.static = list(tensors)
    p.key_t = torch.tensor([seed & 0x7FFFFFFFFFFFFFFF, index0], dtype=torch.int64, device=x.device)
    p.graphs, p.records = [], []
    p.pool = torch.cuda.graph_pool_handle()
    side = torch.cuda.Stream(device=x.device)
    side.wait_stream(torch.cuda.current_stream())
    torch.cuda.synchronize()
    cur = [torch.cuda.CUDAGraph()]

    def end_segment():
        """capture_end; a segment that recorded no kernels (e.g. after the last progress callback of a
        sampler whose final update ran before it) is kept as None and skipped on replay."""
        import warnings
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            cur[0].capture_end()
        if any("empty" in str(x.message).lower() for x in w):
            stats["empty_segments"] = stats.get("empty_segments", 0) + 1
            _graveyard.append(cur[0])
            return None
        return cur[0]

    def cut(d):                       # the sampler's per-step callback: end this step's graph
        p.graphs.append(end_segment())
        p.records.append({k: v for k, v in d.items()})
        cur[0] = torch.cuda.CUDAGraph()
        cur[0].capture_begin(pool=p.pool)

    sig_cpu = sigmas.detach().cpu()
    capturing = False
    try:
        with torch.cuda.stream(side), ops.rng_key_scope(p.key_t, seed, index0):
            cur[0].capture_begin(pool=p.pool)
            capturing = True
            out = ksampler.sampler_function(mk, x, sig_cpu, extra_args=extra_args, callback=cut, disable=True,
                                            **ksampler.extra_options)
            capturing = False
            p.graphs.append(end_segment())
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
    except Exception as e:
        if capturing:
            try:
                cur[0].capture_end()
            except Exception:
                pass
            _abort_capture(side)
        # the aborted graph objects stay referenced: destroying a graph whose capture was
        # invalidated can itself raise in the destructor (fatal outside Python's control)
        _graveyard.append((cur[0], p.graphs))
        try:
            torch.cuda.synchronize()
        except Exception:
            pass
        stats["capture_failed"] += 1
        _ineligible(f"capture: {type(e).__name__}: {str(e)[:80]}")
        logging.warning("sampler-run hipGraph capture failed (%s); this plan stays eager", e,
                        exc_info=os.environ.get("CGS_GRAPH_DEBUG", "0") == "1")
        return None
    p.out = out
    p.keepalive = (mk, extra_args)   # the captured kernels read the guider's cond tensors
    return p
