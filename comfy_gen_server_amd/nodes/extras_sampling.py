"""Custom-sampling node API (parity: ``comfy_extras/nodes_custom_sampler.py``, ``nodes_align_your_steps.py``,
``nodes_perpneg.py`` guider; SURVEY §2.2 'Sampling').

Schedulers return SIGMAS (1-D float tensors on the host), samplers return SAMPLER objects
(``sampling.samplers.KSAMPLER`` with extra options), guiders return GUIDER objects (a CFGGuider
subclass), noise nodes return NOISE objects with ``generate_noise(latent)`` + ``seed``.
"""
from __future__ import annotations

import torch

from ..runtime import device as dm
from ..sampling import k_samplers as kds
from ..sampling import sample as S
from ..sampling import samplers as SM
from ..sampling import schedulers as SCH
from ..utils import progress
from . import helpers as NH

_FLOAT = lambda d, lo=0.0, hi=1000.0, st=0.01: ("FLOAT", {"default": d, "min": lo, "max": hi, "step": st,  # noqa: E731
                                                          "round": False})


# ---------------------------------------------------------------- schedulers
class BasicScheduler:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model": ("MODEL",), "scheduler": (SCH.SCHEDULER_NAMES,),
                             "steps": ("INT", {"default": 20, "min": 1, "max": 10000}),
                             "denoise": ("FLOAT", {"default": 1.0, "min": 0.0, "max": 1.0, "step": 0.01})}}
    RETURN_TYPES = ("SIGMAS",)
    CATEGORY = "sampling/custom_sampling/schedulers"
    FUNCTION = "get_sigmas"

    def get_sigmas(self, model, scheduler, steps, denoise):
        total = steps
        if denoise < 1.0:
            if denoise <= 0.0:
                return (torch.FloatTensor([]),)
            total = int(steps / denoise)
        sigmas = SCH.calculate_sigmas(model.get_model_object("model_sampling"), scheduler, total).cpu()
        return (sigmas[-(steps + 1):],)


class KarrasScheduler:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"steps": ("INT", {"default": 20, "min": 1, "max": 10000}),
                             "sigma_max": _FLOAT(14.614642), "sigma_min": _FLOAT(0.0291675),
                             "rho": _FLOAT(7.0, 0.0, 100.0)}}
    RETURN_TYPES = ("SIGMAS",)
    CATEGORY = "sampling/custom_sampling/schedulers"
    FUNCTION = "get_sigmas"

    def get_sigmas(self, steps, sigma_max, sigma_min, rho):
        return (SCH.get_sigmas_karras(n=steps, sigma_min=sigma_min, sigma_max=sigma_max, rho=rho),)


class ExponentialScheduler:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"steps": ("INT", {"default": 20, "min": 1, "max": 10000}),
                             "sigma_max": _FLOAT(14.614642), "sigma_min": _FLOAT(0.0291675)}}
    RETURN_TYPES = ("SIGMAS",)
    CATEGORY = "sampling/custom_sampling/schedulers"
    FUNCTION = "get_sigmas"

    def get_sigmas(self, steps, sigma_max, sigma_min):
        return (SCH.get_sigmas_exponential(n=steps, sigma_min=sigma_min, sigma_max=sigma_max),)


class PolyexponentialScheduler:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"steps": ("INT", {"default": 20, "min": 1, "max": 10000}),
                             "sigma_max": _FLOAT(14.614642), "sigma_min": _FLOAT(0.0291675),
                             "rho": _FLOAT(1.0, 0.0, 100.0)}}
    RETURN_TYPES = ("SIGMAS",)
    CATEGORY = "sampling/custom_sampling/schedulers"
    FUNCTION = "get_sigmas"

    def get_sigmas(self, steps, sigma_max, sigma_min, rho):
        return (SCH.get_sigmas_polyexponential(n=steps, sigma_min=sigma_min, sigma_max=sigma_max, rho=rho),)


class SDTurboScheduler:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model": ("MODEL",), "steps": ("INT", {"default": 1, "min": 1, "max": 10}),
                             "denoise": ("FLOAT", {"default": 1.0, "min": 0, "max": 1.0, "step": 0.01})}}
    RETURN_TYPES = ("SIGMAS",)
    CATEGORY = "sampling/custom_sampling/schedulers"
    FUNCTION = "get_sigmas"

    def get_sigmas(self, model, steps, denoise):
        return (SCH.sd_turbo_sigmas(model.get_model_object("model_sampling"), steps, denoise),)


class VPScheduler:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"steps": ("INT", {"default": 20, "min": 1, "max": 10000}),
                             "beta_d": _FLOAT(19.9), "beta_min": _FLOAT(0.1),
                             "eps_s": ("FLOAT", {"default": 0.001, "min": 0.0, "max": 1.0, "step": 0.0001,
                                                 "round": False})}}
    RETURN_TYPES = ("SIGMAS",)
    CATEGORY = "sampling/custom_sampling/schedulers"
    FUNCTION = "get_sigmas"

    def get_sigmas(self, steps, beta_d, beta_min, eps_s):
        return (SCH.get_sigmas_vp(n=steps, beta_d=beta_d, beta_min=beta_min, eps_s=eps_s),)


class AlignYourStepsScheduler:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model_type": (["SD1", "SDXL", "SVD"],),
                             "steps": ("INT", {"default": 10, "min": 10, "max": 10000}),
                             "denoise": ("FLOAT", {"default": 1.0, "min": 0.0, "max": 1.0, "step": 0.01})}}
    RETURN_TYPES = ("SIGMAS",)
    CATEGORY = "sampling/custom_sampling/schedulers"
    FUNCTION = "get_sigmas"

    def get_sigmas(self, model_type, steps, denoise):
        return (SCH.ays_sigmas(model_type, steps, denoise),)


class SplitSigmas:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"sigmas": ("SIGMAS",), "step": ("INT", {"default": 0, "min": 0, "max": 10000})}}
    RETURN_TYPES = ("SIGMAS", "SIGMAS")
    CATEGORY = "sampling/custom_sampling/sigmas"
    FUNCTION = "get_sigmas"

    def get_sigmas(self, sigmas, step):
        return (sigmas[:step + 1], sigmas[step:])


class FlipSigmas:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"sigmas": ("SIGMAS",)}}
    RETURN_TYPES = ("SIGMAS",)
    CATEGORY = "sampling/custom_sampling/sigmas"
    FUNCTION = "get_sigmas"

    def get_sigmas(self, sigmas):
        if len(sigmas) == 0:
            return (sigmas,)
        sigmas = sigmas.flip(0)
        if sigmas[0] == 0:
            sigmas = sigmas.clone()
            sigmas[0] = 0.0001
        return (sigmas,)


# ---------------------------------------------------------------- samplers
class KSamplerSelect:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"sampler_name": (SM.SAMPLER_NAMES,)}}
    RETURN_TYPES = ("SAMPLER",)
    CATEGORY = "sampling/custom_sampling/samplers"
    FUNCTION = "get_sampler"

    def get_sampler(self, sampler_name):
        return (SM.sampler_object(sampler_name),)


class SamplerDPMPP_3M_SDE:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"eta": _FLOAT(1.0, 0.0, 100.0), "s_noise": _FLOAT(1.0, 0.0, 100.0),
                             "noise_device": (["gpu", "cpu"],)}}
    RETURN_TYPES = ("SAMPLER",)
    CATEGORY = "sampling/custom_sampling/samplers"
    FUNCTION = "get_sampler"

    def get_sampler(self, eta, s_noise, noise_device):
        name = "dpmpp_3m_sde" if noise_device == "cpu" else "dpmpp_3m_sde_gpu"
        return (SM.ksampler(name, {"eta": eta, "s_noise": s_noise}),)


class SamplerDPMPP_2M_SDE:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"solver_type": (["midpoint", "heun"],), "eta": _FLOAT(1.0, 0.0, 100.0),
                             "s_noise": _FLOAT(1.0, 0.0, 100.0), "noise_device": (["gpu", "cpu"],)}}
    RETURN_TYPES = ("SAMPLER",)
    CATEGORY = "sampling/custom_sampling/samplers"
    FUNCTION = "get_sampler"

    def get_sampler(self, solver_type, eta, s_noise, noise_device):
        name = "dpmpp_2m_sde" if noise_device == "cpu" else "dpmpp_2m_sde_gpu"
        return (SM.ksampler(name, {"eta": eta, "s_noise": s_noise, "solver_type": solver_type}),)


class SamplerDPMPP_SDE:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"eta": _FLOAT(1.0, 0.0, 100.0), "s_noise": _FLOAT(1.0, 0.0, 100.0),
                             "r": _FLOAT(0.5, 0.0, 100.0), "noise_device": (["gpu", "cpu"],)}}
    RETURN_TYPES = ("SAMPLER",)
    CATEGORY = "sampling/custom_sampling/samplers"
    FUNCTION = "get_sampler"

    def get_sampler(self, eta, s_noise, r, noise_device):
        name = "dpmpp_sde" if noise_device == "cpu" else "dpmpp_sde_gpu"
        return (SM.ksampler(name, {"eta": eta, "s_noise": s_noise, "r": r}),)


class SamplerEulerAncestral:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"eta": _FLOAT(1.0, 0.0, 100.0), "s_noise": _FLOAT(1.0, 0.0, 100.0)}}
    RETURN_TYPES = ("SAMPLER",)
    CATEGORY = "sampling/custom_sampling/samplers"
    FUNCTION = "get_sampler"

    def get_sampler(self, eta, s_noise):
        return (SM.ksampler("euler_ancestral", {"eta": eta, "s_noise": s_noise}),)


class SamplerLMS:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"order": ("INT", {"default": 4, "min": 1, "max": 100})}}
    RETURN_TYPES = ("SAMPLER",)
    CATEGORY = "sampling/custom_sampling/samplers"
    FUNCTION = "get_sampler"

    def get_sampler(self, order):
        return (SM.ksampler("lms", {"order": order}),)


class SamplerDPMAdaptative:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"order": ("INT", {"default": 3, "min": 2, "max": 3}),
                             "rtol": _FLOAT(0.05, 0.0, 100.0), "atol": _FLOAT(0.0078, 0.0, 100.0),
                             "h_init": _FLOAT(0.05, 0.0, 100.0), "pcoeff": _FLOAT(0.0, 0.0, 100.0),
                             "icoeff": _FLOAT(1.0, 0.0, 100.0), "dcoeff": _FLOAT(0.0, 0.0, 100.0),
                             "accept_safety": _FLOAT(0.81, 0.0, 100.0), "eta": _FLOAT(0.0, 0.0, 100.0),
                             "s_noise": _FLOAT(1.0, 0.0, 100.0)}}
    RETURN_TYPES = ("SAMPLER",)
    CATEGORY = "sampling/custom_sampling/samplers"
    FUNCTION = "get_sampler"

    def get_sampler(self, order, rtol, atol, h_init, pcoeff, icoeff, dcoeff, accept_safety, eta, s_noise):
        return (SM.ksampler("dpm_adaptive", {"order": order, "rtol": rtol, "atol": atol, "h_init": h_init,
                                             "pcoeff": pcoeff, "icoeff": icoeff, "dcoeff": dcoeff,
                                             "accept_safety": accept_safety, "eta": eta, "s_noise": s_noise}),)


# ---------------------------------------------------------------- noise
class Noise_EmptyNoise:
    def __init__(self):
        self.seed = 0

    def generate_noise(self, input_latent):
        li = input_latent["samples"]
        return torch.zeros(li.shape, dtype=li.dtype, layout=li.layout, device="cpu")


class Noise_RandomNoise:
    def __init__(self, seed):
        self.seed = seed

    def generate_noise(self, input_latent):
        return S.prepare_noise(input_latent["samples"], self.seed, input_latent.get("batch_index"))


class DisableNoise:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {}}
    RETURN_TYPES = ("NOISE",)
    FUNCTION = "get_noise"
    CATEGORY = "sampling/custom_sampling/noise"

    def get_noise(self):
        return (Noise_EmptyNoise(),)


class RandomNoise(DisableNoise):
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"noise_seed": ("INT", {"default": 0, "min": 0, "max": 0xffffffffffffffff})}}

    def get_noise(self, noise_seed):
        return (Noise_RandomNoise(noise_seed),)


class AddNoise:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model": ("MODEL",), "noise": ("NOISE",), "sigmas": ("SIGMAS",),
                             "latent_image": ("LATENT",)}}
    RETURN_TYPES = ("LATENT",)
    FUNCTION = "add_noise"
    CATEGORY = "_for_testing/custom_sampling/noise"

    def add_noise(self, model, noise, sigmas, latent_image):
        if len(sigmas) == 0:
            return (latent_image,)
        latent = latent_image
        li = latent["samples"]
        noisy = noise.generate_noise(latent)
        ms = model.get_model_object("model_sampling")
        scale = torch.abs(sigmas[0] - sigmas[-1]) if len(sigmas) > 1 else sigmas[0]
        if torch.count_nonzero(li) > 0:     # the empty latent is not shifted
            li = model.get_model_object("process_latent_in")(li)
        noisy = ms.noise_scaling(scale, noisy, li)
        noisy = model.get_model_object("process_latent_out")(noisy)
        out = latent.copy()
        out["samples"] = torch.nan_to_num(noisy, nan=0.0, posinf=0.0, neginf=0.0)
        return (out,)


# ---------------------------------------------------------------- guiders
class Guider_Basic(SM.CFGGuider):
    def set_conds(self, positive):
        self.inner_set_conds({"positive": positive})


class Guider_DualCFG(SM.CFGGuider):
    def set_cfg(self, cfg1, cfg2):
        self.cfg1 = cfg1
        self.cfg2 = cfg2

    def set_conds(self, positive, middle, negative):
        middle = NH.conditioning_set_values(middle, {"prompt_type": "negative"})
        self.inner_set_conds({"positive": positive, "middle": middle, "negative": negative})

    def predict_noise(self, x, timestep, model_options=None, seed=None):
        model_options = model_options or {}
        neg = self.conds.get("negative")
        mid = self.conds.get("middle")
        out = SM.calc_cond_batch(self.inner_model, [neg, mid, self.conds.get("positive")], x, timestep,
                                 model_options)
        return SM.cfg_function(self.inner_model, out[1], out[0], self.cfg2, x, timestep,
                               model_options=model_options, cond=mid, uncond=neg) + (out[2] - out[1]) * self.cfg1


class Guider_PerpNeg(SM.CFGGuider):
    """Perp-Neg (nodes_perpneg.py): remove from the positive direction the component along the
    negative prompt, relative to an empty-prompt prediction."""

    def set_conds(self, positive, negative, empty_negative_prompt):
        empty = NH.conditioning_set_values(empty_negative_prompt, {"prompt_type": "negative"})
        self.inner_set_conds({"positive": positive, "empty_negative_prompt": empty, "negative": negative})

    def set_cfg(self, cfg, neg_scale):
        self.cfg = cfg
        self.neg_scale = neg_scale

    def predict_noise(self, x, timestep, model_options=None, seed=None):
        model_options = model_options or {}
        pos = self.conds.get("positive")
        neg = self.conds.get("negative")
        empty = self.conds.get("empty_negative_prompt")
        pos_out, neg_out, empty_out = SM.calc_cond_batch(self.inner_model, [pos, neg, empty], x, timestep,
                                                         model_options)
        cfg = perp_neg_combine(x, pos_out, neg_out, empty_out, self.neg_scale, self.cfg)
        for fn in model_options.get("sampler_post_cfg_function", []):
            cfg = fn({"denoised": cfg, "cond": pos, "uncond": neg, "model": self.inner_model,
                      "uncond_denoised": neg_out, "cond_denoised": pos_out, "sigma": timestep,
                      "model_options": model_options, "input": x, "empty_cond": empty,
                      "empty_cond_denoised": empty_out})
        return cfg


def perp_neg_combine(x, pos_out, neg_out, empty_out, neg_scale, cond_scale):
    from .extras_model import perp_neg
    return perp_neg(x, pos_out, neg_out, empty_out, neg_scale, cond_scale)


class BasicGuider:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model": ("MODEL",), "conditioning": ("CONDITIONING",)}}
    RETURN_TYPES = ("GUIDER",)
    FUNCTION = "get_guider"
    CATEGORY = "sampling/custom_sampling/guiders"

    def get_guider(self, model, conditioning):
        g = Guider_Basic(model)
        g.set_conds(conditioning)
        return (g,)


class CFGGuider:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model": ("MODEL",), "positive": ("CONDITIONING",), "negative": ("CONDITIONING",),
                             "cfg": ("FLOAT", {"default": 8.0, "min": 0.0, "max": 100.0, "step": 0.1, "round": 0.01})}}
    RETURN_TYPES = ("GUIDER",)
    FUNCTION = "get_guider"
    CATEGORY = "sampling/custom_sampling/guiders"

    def get_guider(self, model, positive, negative, cfg):
        g = SM.CFGGuider(model)
        g.set_conds(positive, negative)
        g.set_cfg(cfg)
        return (g,)


class DualCFGGuider:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model": ("MODEL",), "cond1": ("CONDITIONING",), "cond2": ("CONDITIONING",),
                             "negative": ("CONDITIONING",),
                             "cfg_conds": ("FLOAT", {"default": 8.0, "min": 0.0, "max": 100.0, "step": 0.1, "round": 0.01}),
                             "cfg_cond2_negative": ("FLOAT", {"default": 8.0, "min": 0.0, "max": 100.0, "step": 0.1,
                                                              "round": 0.01})}}
    RETURN_TYPES = ("GUIDER",)
    FUNCTION = "get_guider"
    CATEGORY = "sampling/custom_sampling/guiders"

    def get_guider(self, model, cond1, cond2, negative, cfg_conds, cfg_cond2_negative):
        g = Guider_DualCFG(model)
        g.set_conds(cond1, cond2, negative)
        g.set_cfg(cfg_conds, cfg_cond2_negative)
        return (g,)


class PerpNegGuider:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model": ("MODEL",), "positive": ("CONDITIONING",), "negative": ("CONDITIONING",),
                             "empty_conditioning": ("CONDITIONING",),
                             "cfg": ("FLOAT", {"default": 8.0, "min": 0.0, "max": 100.0, "step": 0.1, "round": 0.01}),
                             "neg_scale": ("FLOAT", {"default": 1.0, "min": 0.0, "max": 100.0, "step": 0.01})}}
    RETURN_TYPES = ("GUIDER",)
    FUNCTION = "get_guider"
    CATEGORY = "_for_testing"

    def get_guider(self, model, positive, negative, empty_conditioning, cfg, neg_scale):
        g = Guider_PerpNeg(model)
        g.set_conds(positive, negative, empty_conditioning)
        g.set_cfg(cfg, neg_scale)
        return (g,)


# ---------------------------------------------------------------- sampling nodes
def _finish(latent, samples, x0_output, process_latent_out):
    out = latent.copy()
    out["samples"] = samples
    if "x0" in x0_output:
        den = latent.copy()
        den["samples"] = process_latent_out(x0_output["x0"].cpu())
    else:
        den = out
    return (out, den)


class SamplerCustom:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model": ("MODEL",), "add_noise": ("BOOLEAN", {"default": True}),
                             "noise_seed": ("INT", {"default": 0, "min": 0, "max": 0xffffffffffffffff}),
                             "cfg": ("FLOAT", {"default": 8.0, "min": 0.0, "max": 100.0, "step": 0.1, "round": 0.01}),
                             "positive": ("CONDITIONING",), "negative": ("CONDITIONING",),
                             "sampler": ("SAMPLER",), "sigmas": ("SIGMAS",), "latent_image": ("LATENT",)}}
    RETURN_TYPES = ("LATENT", "LATENT")
    RETURN_NAMES = ("output", "denoised_output")
    FUNCTION = "sample"
    CATEGORY = "sampling/custom_sampling"

    def sample(self, model, add_noise, noise_seed, cfg, positive, negative, sampler, sigmas, latent_image):
        latent = latent_image
        noise = (Noise_RandomNoise(noise_seed) if add_noise else Noise_EmptyNoise()).generate_noise(latent)
        x0_output = {}
        cb = NH.prepare_callback(model, sigmas.shape[-1] - 1, x0_output)
        samples = S.sample_custom(model, noise, cfg, sampler, sigmas, positive, negative, latent["samples"],
                                  noise_mask=latent.get("noise_mask"), callback=cb,
                                  disable_pbar=not progress.PROGRESS_BAR_ENABLED, seed=noise_seed,
                                  noise_inds=latent.get("batch_index"))
        return _finish(latent, samples, x0_output, model.model.process_latent_out)


class SamplerCustomAdvanced:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"noise": ("NOISE",), "guider": ("GUIDER",), "sampler": ("SAMPLER",),
                             "sigmas": ("SIGMAS",), "latent_image": ("LATENT",)}}
    RETURN_TYPES = ("LATENT", "LATENT")
    RETURN_NAMES = ("output", "denoised_output")
    FUNCTION = "sample"
    CATEGORY = "sampling/custom_sampling"

    def sample(self, noise, guider, sampler, sigmas, latent_image):
        latent = latent_image
        x0_output = {}
        cb = NH.prepare_callback(guider.model_patcher, sigmas.shape[-1] - 1, x0_output)
        samples = guider.sample(noise.generate_noise(latent), latent["samples"], sampler, sigmas,
                                denoise_mask=latent.get("noise_mask"), callback=cb,
                                disable_pbar=not progress.PROGRESS_BAR_ENABLED, seed=noise.seed)
        samples = samples.to(dm.intermediate_device())
        return _finish(latent, samples, x0_output, guider.model_patcher.model.process_latent_out)


NODE_CLASS_MAPPINGS = {
    "SamplerCustom": SamplerCustom, "BasicScheduler": BasicScheduler, "KarrasScheduler": KarrasScheduler,
    "ExponentialScheduler": ExponentialScheduler, "PolyexponentialScheduler": PolyexponentialScheduler,
    "VPScheduler": VPScheduler, "SDTurboScheduler": SDTurboScheduler, "KSamplerSelect": KSamplerSelect,
    "SamplerEulerAncestral": SamplerEulerAncestral, "SamplerLMS": SamplerLMS,
    "SamplerDPMPP_3M_SDE": SamplerDPMPP_3M_SDE, "SamplerDPMPP_2M_SDE": SamplerDPMPP_2M_SDE,
    "SamplerDPMPP_SDE": SamplerDPMPP_SDE, "SamplerDPMAdaptative": SamplerDPMAdaptative,
    "SplitSigmas": SplitSigmas, "FlipSigmas": FlipSigmas, "CFGGuider": CFGGuider, "DualCFGGuider": DualCFGGuider,
    "BasicGuider": BasicGuider, "PerpNegGuider": PerpNegGuider, "RandomNoise": RandomNoise,
    "DisableNoise": DisableNoise, "AddNoise": AddNoise, "SamplerCustomAdvanced": SamplerCustomAdvanced,
    "AlignYourStepsScheduler": AlignYourStepsScheduler,
}
NODE_DISPLAY_NAME_MAPPINGS = {"SamplerDPMAdaptative": "SamplerDPMAdaptative"}
_ = kds   # k-diffusion functions are reached through SM.ksampler
