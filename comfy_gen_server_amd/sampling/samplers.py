"""CFG guidance, conditioning batching and the KSampler facade.

Parity with ``comfy/samplers.py`` (C20/C21): get_area_and_mult (timestep gating, area crop,
mask / feathered multipliers), calc_cond_batch (cond+uncond packed into one UNet batch, outputs
scatter-added by mult and normalised), cfg_function (+ sampler_cfg_function / post-cfg hooks),
sampling_function (cfg==1 skips uncond), KSamplerX0Inpaint, process_conds (area/mask resolve,
start/end percent, extra_conds, opposite-area fill, control pre_run, apply_empty_x_to_equal_area),
KSAMPLER, ksampler(), sampler_object(), calculate_sigmas, KSampler (denoise / start / last step /
force_full_denoise / discard-penultimate-sigma), CFGGuider and sample().

MI355X differences (same results):
  * the memory-driven sub-batching (``get_free_memory`` every step) is gone: with 288 GB the whole
    cond+uncond batch always runs as one forward;
  * a *fast path* for the common case (one cond + one uncond entry, no areas/masks/gligen) skips
    the scatter/mult/count buffers entirely and can be replayed from a hipGraph
    (``runtime/graphs.py``);
  * timestep gating compares host floats (the sampler publishes the current sigma), no D2H sync.
"""
from __future__ import annotations

import collections
import contextvars
import logging
import math

import torch

from .. import ops

from ..runtime import device as dm
from ..utils import telemetry
from . import k_samplers as kds
from . import uni_pc
from .schedulers import SCHEDULER_NAMES, calculate_sigmas  # noqa: F401
from . import sampler_helpers

current_sigma = contextvars.ContextVar("cgs_current_sigma", default=None)

CondObj = collections.namedtuple("cond_obj", ["input_x", "mult", "conditioning", "area", "control", "patches"])


def _host_sigma(timestep):
    s = current_sigma.get()
    if s is not None:
        return s
    return float(timestep[0])


def get_area_and_mult(conds, x_in, timestep_in, need_mult=True):
    area = (x_in.shape[2], x_in.shape[3], 0, 0)
    strength = 1.0
    if "timestep_start" in conds or "timestep_end" in conds:
        t0 = _host_sigma(timestep_in)
        if "timestep_start" in conds and t0 > conds["timestep_start"]:
            return None
        if "timestep_end" in conds and t0 < conds["timestep_end"]:
            return None
    if "area" in conds:
        area = conds["area"]
    if "strength" in conds:
        strength = conds["strength"]
    input_x = x_in[:, :, area[2]:area[0] + area[2], area[3]:area[1] + area[3]]
    mult = None
    if need_mult:
        if "mask" in conds:
            ms = conds.get("mask_strength", 1.0)
            mask = conds["mask"]
            assert mask.shape[1] == x_in.shape[2] and mask.shape[2] == x_in.shape[3]
            mask = mask[:, area[2]:area[0] + area[2], area[3]:area[1] + area[3]] * ms
            mask = mask.unsqueeze(1).repeat(input_x.shape[0] // mask.shape[0], input_x.shape[1], 1, 1)
        else:
            mask = torch.ones_like(input_x)
        mult = mask * strength
        if "mask" not in conds:
            rr = 8
            H, W = x_in.shape[2], x_in.shape[3]
            ramp = [(1.0 / rr) * (t + 1) for t in range(rr)]
            if area[2] != 0:
                for t in range(rr):
                    mult[:, :, t:1 + t, :] *= ramp[t]
            if (area[0] + area[2]) < H:
                for t in range(rr):
                    mult[:, :, area[0] - 1 - t:area[0] - t, :] *= ramp[t]
            if area[3] != 0:
                for t in range(rr):
                    mult[:, :, :, t:1 + t] *= ramp[t]
            if (area[1] + area[3]) < W:
                for t in range(rr):
                    mult[:, :, :, area[1] - 1 - t:area[1] - t] *= ramp[t]
    conditioning = {k: v.process_cond(batch_size=x_in.shape[0], device=x_in.device, area=area)
                    for k, v in conds["model_conds"].items()}
    control = conds.get("control")
    patches = None
    if "gligen" in conds:
        g = conds["gligen"]
        patches = {}
        if g[0] == "position":
            gp = g[1].model.set_position(input_x.shape, g[2], input_x.device)
        else:
            gp = g[1].model.set_empty(input_x.shape, input_x.device)
        patches["middle_patch"] = [gp]
    return CondObj(input_x, mult, conditioning, area, control, patches)


def cond_equal_size(c1, c2):
    if c1 is c2:
        return True
    if c1.keys() != c2.keys():
        return False
    return all(c1[k].can_concat(c2[k]) for k in c1)


def can_concat_cond(c1, c2):
    if c1.input_x.shape != c2.input_x.shape:
        return False

    def same(a, b):
        if (a is None) != (b is None):
            return False
        return a is None or a is b
    if not same(c1.control, c2.control) or not same(c1.patches, c2.patches):
        return False
    return cond_equal_size(c1.conditioning, c2.conditioning)


def cond_cat(c_list):
    temp = {}
    for x in c_list:
        for k, v in x.items():
            temp.setdefault(k, []).append(v)
    return {k: v[0].concat(v[1:]) for k, v in temp.items()}


def _run_batch(model, batch, timestep, model_options):
    """batch: list of (CondObj, cond_index). Returns (outputs per chunk)."""
    input_x = torch.cat([p.input_x for p, _ in batch])
    c = cond_cat([p.conditioning for p, _ in batch])
    cond_or_uncond = [i for _, i in batch]
    control = batch[-1][0].control
    patches = batch[-1][0].patches
    n = len(batch)
    timestep_ = torch.cat([timestep] * n)
    if control is not None:
        c["control"] = control.get_control(input_x, timestep_, c, n)
    to = dict(model_options.get("transformer_options", {}))
    if patches is not None:
        cur = dict(to.get("patches", {}))
        for k, v in patches.items():
            cur[k] = cur.get(k, []) + v
        to["patches"] = cur
    to["cond_or_uncond"] = cond_or_uncond[:]
    to["sigmas"] = timestep
    c["transformer_options"] = to
    if "model_function_wrapper" in model_options:
        out = model_options["model_function_wrapper"](model.apply_model, {"input": input_x, "timestep": timestep_, "c": c,
                                                                          "cond_or_uncond": cond_or_uncond})
    else:
        out = model.apply_model(input_x, timestep_, **c)
    return out.chunk(n), cond_or_uncond


def _simple_conds(conds):
    for cl in conds:
        if cl is None:
            continue
        if len(cl) != 1:
            return False
        x = cl[0]
        if "area" in x or "mask" in x or "gligen" in x or "timestep_start" in x or "timestep_end" in x:
            return False
        if x.get("strength", 1.0) != 1.0:
            return False
    return True


def calc_cond_batch(model, conds, x_in, timestep, model_options):
    # ---- fast path: one entry per cond list, full-frame -> one batched forward, no scatter
    if _simple_conds(conds):
        runs = []
        for i, cl in enumerate(conds):
            if cl is not None:
                runs.append((get_area_and_mult(cl[0], x_in, timestep, need_mult=False), i))
        if len(runs) == 2 and not can_concat_cond(runs[0][0], runs[1][0]):
            outs = [_run_batch(model, [r], timestep, model_options) for r in runs]
            res = [None] * len(conds)
            for (o, idx) in outs:
                res[idx[0]] = o[0]
            return res
        if runs:
            outs, order = _run_batch(model, runs, timestep, model_options)
            res = [None] * len(conds)
            for o, idx in zip(outs, order):
                res[idx] = o
            return res

    # ---- general path (areas / masks / gligen / timestep ranges)
    out_conds, out_counts, to_run = [], [], []
    for i, cond in enumerate(conds):
        out_conds.append(torch.zeros_like(x_in))
        out_counts.append(torch.ones_like(x_in) * 1e-37)
        if cond is not None:
            for x in cond:
                p = get_area_and_mult(x, x_in, timestep)
                if p is not None:
                    to_run.append((p, i))
    while to_run:
        first = to_run[0]
        idx = [j for j in range(len(to_run)) if can_concat_cond(to_run[j][0], first[0])]
        batch = [to_run[j] for j in idx]
        for j in reversed(idx):
            to_run.pop(j)
        outs, order = _run_batch(model, batch, timestep, model_options)
        for o, (p, ci) in zip(outs, batch):
            a = p.area
            # out[area] += o * mult ; count[area] += mult (one HIP kernel on the device, K17)
            ops.region_accumulate(out_conds[ci], out_counts[ci], o, a[2], a[3], mult=p.mult)
    return [ops.region_normalize(oc, cnt) for oc, cnt in zip(out_conds, out_counts)]


def calc_cond_uncond_batch(model, cond, uncond, x_in, timestep, model_options):
    return tuple(calc_cond_batch(model, [cond, uncond], x_in, timestep, model_options))


def cfg_function(model, cond_pred, uncond_pred, cond_scale, x, timestep, model_options=None, cond=None, uncond=None):
    model_options = model_options or {}
    if "sampler_cfg_function" in model_options:
        args = {"cond": x - cond_pred, "uncond": x - uncond_pred, "cond_scale": cond_scale, "timestep": timestep,
                "input": x, "sigma": timestep, "cond_denoised": cond_pred, "uncond_denoised": uncond_pred,
                "model": model, "model_options": model_options}
        res = x - model_options["sampler_cfg_function"](args)
    elif uncond_pred is None:
        res = cond_pred
    else:
        from .. import ops
        res = ops.cfg_combine(cond_pred.contiguous(), uncond_pred.contiguous(), cond_scale)
    for fn in model_options.get("sampler_post_cfg_function", []):
        args = {"denoised": res, "cond": cond, "uncond": uncond, "model": model, "uncond_denoised": uncond_pred,
                "cond_denoised": cond_pred, "sigma": timestep, "model_options": model_options, "input": x}
        res = fn(args)
    return res


def sampling_function(model, x, timestep, uncond, cond, cond_scale, model_options=None, seed=None):
    model_options = model_options or {}
    if math.isclose(cond_scale, 1.0) and not model_options.get("disable_cfg1_optimization", False):
        uncond_ = None
    else:
        uncond_ = uncond
    out = calc_cond_batch(model, [cond, uncond_], x, timestep, model_options)
    return cfg_function(model, out[0], out[1], cond_scale, x, timestep, model_options=model_options, cond=cond,
                        uncond=uncond_)


class KSamplerX0Inpaint:
    def __init__(self, model, sigmas):
        self.inner_model = model
        self.sigmas = sigmas
        self.noise = None
        self.latent_image = None

    def __call__(self, x, sigma, denoise_mask=None, model_options=None, seed=None, noise_inds=None):
        model_options = model_options or {}
        if denoise_mask is not None:
            if "denoise_mask_function" in model_options:
                denoise_mask = model_options["denoise_mask_function"](
                    sigma, denoise_mask, extra_options={"model": self.inner_model, "sigmas": self.sigmas})
            latent_mask = 1.0 - denoise_mask
            ms = self.inner_model.inner_model.model_sampling
            x = x * denoise_mask + ms.noise_scaling(sigma.reshape([sigma.shape[0]] + [1] * (self.noise.ndim - 1)),
                                                    self.noise, self.latent_image) * latent_mask
        out = self.inner_model(x, sigma, model_options=model_options, seed=seed)
        if denoise_mask is not None:
            out = out * denoise_mask + self.latent_image * latent_mask
        return out


# ------------------------------------------------------------------------------------------------
# cond processing (pre-loop, host side)
# ------------------------------------------------------------------------------------------------
def get_mask_aabb(masks):
    b = masks.shape[0]
    boxes = torch.zeros((b, 4), dtype=torch.int)
    empty = torch.zeros((b,), dtype=torch.bool)
    for i in range(b):
        m = masks[i]
        if m.numel() == 0:
            continue
        if not bool((m != 0).any()):
            empty[i] = True
            continue
        y, x = torch.where(m)
        boxes[i] = torch.tensor([int(x.min()), int(y.min()), int(x.max()), int(y.max())])
    return boxes, empty


def resolve_areas_and_cond_masks(conditions, h, w, device):
    for i, c in enumerate(conditions):
        if "area" in c:
            a = c["area"]
            if a[0] == "percentage":
                c = dict(c)
                c["area"] = (max(1, round(a[1] * h)), max(1, round(a[2] * w)), round(a[3] * h), round(a[4] * w))
                conditions[i] = c
        if "mask" in c:
            mask = c["mask"].to(device=device)
            mod = dict(c)
            if mask.ndim == 2:
                mask = mask.unsqueeze(0)
            if mask.shape[1] != h or mask.shape[2] != w:
                mask = torch.nn.functional.interpolate(mask.unsqueeze(1), size=(h, w), mode="bilinear",
                                                       align_corners=False).squeeze(1)
            if mod.get("set_area_to_bounds", False):
                bounds = torch.max(torch.abs(mask), dim=0).values.unsqueeze(0)
                boxes, empty = get_mask_aabb(bounds.cpu())
                if empty[0]:
                    mod["area"] = (8, 8, 0, 0)
                else:
                    bx = boxes[0]
                    H, W, Y, X = (int(bx[3] - bx[1] + 1), int(bx[2] - bx[0] + 1), int(bx[1]), int(bx[0]))
                    mod["area"] = (max(8, H), max(8, W), Y, X)
            mod["mask"] = mask
            conditions[i] = mod


def create_cond_with_same_area_if_none(conds, c):
    if "area" not in c:
        return
    ca = c["area"]
    smallest = None
    for x in conds:
        if "area" in x:
            a = x["area"]
            if ca[2] >= a[2] and ca[3] >= a[3] and a[0] + a[2] >= ca[0] + ca[2] and a[1] + a[3] >= ca[1] + ca[3]:
                if smallest is None or "area" not in smallest or smallest["area"][0] * smallest["area"][1] > a[0] * a[1]:
                    smallest = x
        elif smallest is None:
            smallest = x
    if smallest is None:
        return
    if "area" in smallest and smallest["area"] == ca:
        return
    out = dict(c)
    out["model_conds"] = dict(smallest["model_conds"])
    conds.append(out)


def calculate_start_end_timesteps(model, conds):
    s = model.model_sampling
    for t, x in enumerate(conds):
        ts = s.percent_to_sigma(x["start_percent"]) if "start_percent" in x else None
        te = s.percent_to_sigma(x["end_percent"]) if "end_percent" in x else None
        if ts is not None or te is not None:
            n = dict(x)
            if ts is not None:
                n["timestep_start"] = ts
            if te is not None:
                n["timestep_end"] = te
            conds[t] = n


def pre_run_control(model, conds):
    s = model.model_sampling
    for x in conds:
        if "control" in x:
            x["control"].pre_run(model, lambda a: s.percent_to_sigma(a))


def apply_empty_x_to_equal_area(conds, uncond, name, fill):
    cond_cnets, uncond_cnets, uncond_other = [], [], []
    for x in conds:
        if "area" not in x and name in x and x[name] is not None:
            cond_cnets.append(x[name])
    for t, x in enumerate(uncond):
        if "area" not in x:
            if name in x and x[name] is not None:
                uncond_cnets.append(x[name])
            else:
                uncond_other.append((x, t))
    if uncond_cnets or not uncond_other:
        return
    for i in range(len(cond_cnets)):
        o, idx = uncond_other[i % len(uncond_other)]
        n = dict(o)
        n[name] = fill(cond_cnets, i)
        if name in o and o[name] is not None:
            uncond.append(n)
        else:
            uncond[idx] = n


def encode_model_conds(model_function, conds, noise, device, prompt_type, **kwargs):
    for t, x in enumerate(conds):
        params = dict(x)
        params["device"] = device
        params["noise"] = noise
        params.setdefault("width", noise.shape[3] * 8)
        params.setdefault("height", noise.shape[2] * 8)
        params.setdefault("prompt_type", prompt_type)
        for k, v in kwargs.items():
            params.setdefault(k, v)
        out = model_function(**params)
        x = dict(x)
        mc = dict(x["model_conds"])
        mc.update(out)
        x["model_conds"] = mc
        conds[t] = x
    return conds


def process_conds(model, noise, conds, device, latent_image=None, denoise_mask=None, seed=None):
    for k in conds:
        conds[k] = conds[k][:]
        resolve_areas_and_cond_masks(conds[k], noise.shape[2], noise.shape[3], device)
    for k in conds:
        calculate_start_end_timesteps(model, conds[k])
    if hasattr(model, "extra_conds"):
        for k in conds:
            conds[k] = encode_model_conds(model.extra_conds, conds[k], noise, device, k,
                                          latent_image=latent_image, denoise_mask=denoise_mask, seed=seed)
    for k in conds:
        for c in conds[k]:
            for kk in conds:
                if k != kk:
                    create_cond_with_same_area_if_none(conds[kk], c)
    for k in conds:
        pre_run_control(model, conds[k])
    if "positive" in conds:
        pos = conds["positive"]
        for k in conds:
            if k != "positive":
                apply_empty_x_to_equal_area([c for c in pos if c.get("control_apply_to_uncond", False)], conds[k],
                                            "control", lambda cn, x: cn[x])
                apply_empty_x_to_equal_area(pos, conds[k], "gligen", lambda cn, x: cn[x])
    return conds


# ------------------------------------------------------------------------------------------------
class Sampler:
    def sample(self, *a, **k):
        raise NotImplementedError

    def max_denoise(self, model_wrap, sigmas):
        max_sigma = float(model_wrap.inner_model.model_sampling.sigma_max)
        sigma = float(sigmas[0])
        return math.isclose(max_sigma, sigma, rel_tol=1e-05) or sigma > max_sigma


KSAMPLER_NAMES = ["euler", "euler_ancestral", "heun", "heunpp2", "dpm_2", "dpm_2_ancestral", "lms", "dpm_fast",
                  "dpm_adaptive", "dpmpp_2s_ancestral", "dpmpp_sde", "dpmpp_sde_gpu", "dpmpp_2m", "dpmpp_2m_sde",
                  "dpmpp_2m_sde_gpu", "dpmpp_3m_sde", "dpmpp_3m_sde_gpu", "ddpm", "lcm"]
SAMPLER_NAMES = KSAMPLER_NAMES + ["ddim", "uni_pc", "uni_pc_bh2"]


class KSAMPLER(Sampler):
    def __init__(self, sampler_function, extra_options=None, inpaint_options=None):
        self.sampler_function = sampler_function
        self.extra_options = extra_options or {}
        self.inpaint_options = inpaint_options or {}

    def sample(self, model_wrap, sigmas, extra_args, callback, noise, latent_image=None, denoise_mask=None,
               disable_pbar=False):
        extra_args["denoise_mask"] = denoise_mask
        mk = KSamplerX0Inpaint(model_wrap, sigmas)
        mk.latent_image = latent_image
        if self.inpaint_options.get("random", False):
            g = torch.manual_seed(extra_args.get("seed", 41) + 1)
            mk.noise = torch.randn(noise.shape, generator=g, device="cpu").to(noise.dtype).to(noise.device)
        else:
            mk.noise = noise
        ms = model_wrap.inner_model.model_sampling
        noise = ms.noise_scaling(sigmas[0], noise, latent_image, self.max_denoise(model_wrap, sigmas))
        total = len(sigmas) - 1
        timed = telemetry.step_timer(callback)        # per-step wall clock + fault site
        k_cb = lambda x: timed(x["i"], x["denoised"], x["x"], total)  # noqa: E731
        from . import run_graph
        samples = run_graph.try_run(self, model_wrap, mk, noise, sigmas, extra_args, k_cb)   # one hipGraph per step
        if samples is None:
            samples = self.sampler_function(mk, noise, sigmas, extra_args=extra_args, callback=k_cb,
                                            disable=disable_pbar, **self.extra_options)
        return ms.inverse_noise_scaling(sigmas[-1], samples)


def ksampler(sampler_name, extra_options=None, inpaint_options=None):
    if sampler_name == "dpm_fast":
        def fn(model, noise, sigmas, extra_args, callback, disable):
            smin = float(sigmas[-1]) or float(sigmas[-2])
            return kds.sample_dpm_fast(model, noise, smin, float(sigmas[0]), len(sigmas) - 1, extra_args=extra_args,
                                       callback=callback, disable=disable)
    elif sampler_name == "dpm_adaptive":
        def fn(model, noise, sigmas, extra_args, callback, disable, **eo):
            smin = float(sigmas[-1]) or float(sigmas[-2])
            return kds.sample_dpm_adaptive(model, noise, smin, float(sigmas[0]), extra_args=extra_args,
                                           callback=callback, disable=disable, **eo)
    else:
        fn = getattr(kds, f"sample_{sampler_name}")
    return KSAMPLER(fn, extra_options, inpaint_options)


def sampler_object(name):
    if name == "uni_pc":
        return KSAMPLER(uni_pc.sample_unipc)
    if name == "uni_pc_bh2":
        return KSAMPLER(uni_pc.sample_unipc_bh2)
    if name == "ddim":
        return ksampler("euler", inpaint_options={"random": True})
    return ksampler(name)


class CFGGuider:
    def __init__(self, model_patcher):
        self.model_patcher = model_patcher
        self.model_options = model_patcher.model_options
        self.original_conds = {}
        self.cfg = 1.0

    def set_conds(self, positive, negative):
        self.inner_set_conds({"positive": positive, "negative": negative})

    def set_cfg(self, cfg):
        self.cfg = cfg

    def inner_set_conds(self, conds):
        for k, v in conds.items():
            self.original_conds[k] = sampler_helpers.convert_cond(v)

    def __call__(self, *args, **kwargs):
        return self.predict_noise(*args, **kwargs)

    def predict_noise(self, x, timestep, model_options=None, seed=None):
        return sampling_function(self.inner_model, x, timestep, self.conds.get("negative"), self.conds.get("positive"),
                                 self.cfg, model_options=model_options or {}, seed=seed)

    def inner_sample(self, noise, latent_image, device, sampler, sigmas, denoise_mask, callback, disable_pbar, seed):
        if latent_image is not None and bool(torch.count_nonzero(latent_image) > 0):
            latent_image = self.inner_model.process_latent_in(latent_image)
        self.conds = process_conds(self.inner_model, noise, self.conds, device, latent_image, denoise_mask, seed)
        extra_args = {"model_options": self.model_options, "seed": seed}
        if getattr(self, "noise_inds", None) is not None:
            extra_args["noise_inds"] = list(self.noise_inds)
        samples = sampler.sample(self, sigmas, extra_args, callback, noise, latent_image, denoise_mask, disable_pbar)
        return self.inner_model.process_latent_out(samples.to(torch.float32))

    def sample(self, noise, latent_image, sampler, sigmas, denoise_mask=None, callback=None, disable_pbar=False,
               seed=None):
        if sigmas.shape[-1] == 0:
            return latent_image
        self.conds = {k: [dict(a) for a in v] for k, v in self.original_conds.items()}
        self.inner_model, self.conds, self.loaded_models = sampler_helpers.prepare_sampling(
            self.model_patcher, noise.shape, self.conds)
        device = self.model_patcher.load_device
        if denoise_mask is not None:
            denoise_mask = sampler_helpers.prepare_mask(denoise_mask, noise.shape, device)
        noise = noise.to(device)
        latent_image = latent_image.to(device)
        sigmas = sigmas.to(device)
        with torch.inference_mode():
            out = self.inner_sample(noise, latent_image, device, sampler, sigmas, denoise_mask, callback,
                                    disable_pbar, seed)
        sampler_helpers.cleanup_models(self.conds, self.loaded_models)
        del self.inner_model, self.conds, self.loaded_models
        return out


def sample(model, noise, positive, negative, cfg, device, sampler, sigmas, model_options=None, latent_image=None,
           denoise_mask=None, callback=None, disable_pbar=False, seed=None, noise_inds=None):
    g = CFGGuider(model)
    g.set_conds(positive, negative)
    g.set_cfg(cfg)
    g.noise_inds = noise_inds
    return g.sample(noise, latent_image, sampler, sigmas, denoise_mask, callback, disable_pbar, seed)


class KSampler:
    SCHEDULERS = SCHEDULER_NAMES
    SAMPLERS = SAMPLER_NAMES
    DISCARD_PENULTIMATE_SIGMA_SAMPLERS = {"dpm_2", "dpm_2_ancestral", "uni_pc", "uni_pc_bh2"}

    def __init__(self, model, steps, device, sampler=None, scheduler=None, denoise=None, model_options=None):
        self.model = model
        self.device = device
        self.scheduler = scheduler if scheduler in self.SCHEDULERS else self.SCHEDULERS[0]
        self.sampler = sampler if sampler in self.SAMPLERS else self.SAMPLERS[0]
        self.set_steps(steps, denoise)
        self.denoise = denoise
        self.model_options = model_options or {}

    def calculate_sigmas(self, steps):
        discard = self.sampler in self.DISCARD_PENULTIMATE_SIGMA_SAMPLERS
        if discard:
            steps += 1
        sigmas = calculate_sigmas(self.model.get_model_object("model_sampling"), self.scheduler, steps)
        if discard:
            sigmas = torch.cat([sigmas[:-2], sigmas[-1:]])
        return sigmas

    def set_steps(self, steps, denoise=None):
        self.steps = steps
        if denoise is None or denoise > 0.9999:
            self.sigmas = self.calculate_sigmas(steps).to(self.device)
        elif denoise <= 0.0:
            self.sigmas = torch.FloatTensor([])
        else:
            new_steps = int(steps / denoise)
            self.sigmas = self.calculate_sigmas(new_steps).to(self.device)[-(steps + 1):]

    def sample(self, noise, positive, negative, cfg, latent_image=None, start_step=None, last_step=None,
               force_full_denoise=False, denoise_mask=None, sigmas=None, callback=None, disable_pbar=False, seed=None,
               noise_inds=None):
        if sigmas is None:
            sigmas = self.sigmas
        if last_step is not None and last_step < len(sigmas) - 1:
            sigmas = sigmas[:last_step + 1].clone()
            if force_full_denoise:
                sigmas[-1] = 0
        if start_step is not None:
            if start_step < len(sigmas) - 1:
                sigmas = sigmas[start_step:]
            else:
                return latent_image if latent_image is not None else torch.zeros_like(noise)
        return sample(self.model, noise, positive, negative, cfg, self.device, sampler_object(self.sampler), sigmas,
                      self.model_options, latent_image=latent_image, denoise_mask=denoise_mask, callback=callback,
                      disable_pbar=disable_pbar, seed=seed, noise_inds=noise_inds)
