"""Model parameterisations and noise schedules.

Parity with ``comfy/model_sampling.py:1-203``: EPS / V_PREDICTION / EDM / X0 / LCM prediction
types (calculate_input = c_in scaling, calculate_denoised, noise_scaling, inverse_noise_scaling),
ModelSamplingDiscrete (1000-step beta schedule, log-sigma nearest timestep, interpolated sigma,
percent_to_sigma), ModelSamplingContinuousEDM, StableCascadeSampling (cosine schedule + shift),
ModelSamplingDiscreteDistilled (LCM).

Everything a sampler needs per step is host-computable, so a sampling run precomputes its
sigma -> timestep table once (``timestep_table``) and the per-step hipGraph sees only constants.
"""
from __future__ import annotations

import math

import numpy as np
import torch


def make_beta_schedule(schedule, n_timestep, linear_start=1e-4, linear_end=2e-2, cosine_s=8e-3):
    if schedule == "linear":
        betas = torch.linspace(linear_start ** 0.5, linear_end ** 0.5, n_timestep, dtype=torch.float64) ** 2
    elif schedule == "cosine":
        ts = torch.arange(n_timestep + 1, dtype=torch.float64) / n_timestep + cosine_s
        alphas = torch.cos(ts / (1 + cosine_s) * math.pi / 2).pow(2)
        alphas = alphas / alphas[0]
        betas = (1 - alphas[1:] / alphas[:-1]).clamp(0, 0.999)
    elif schedule == "squaredcos_cap_v2":
        def abar(t):
            return math.cos((t + 0.008) / 1.008 * math.pi / 2) ** 2
        betas = torch.tensor([min(1 - abar((i + 1) / n_timestep) / abar(i / n_timestep), 0.999)
                              for i in range(n_timestep)], dtype=torch.float64)
    elif schedule == "sqrt_linear":
        betas = torch.linspace(linear_start, linear_end, n_timestep, dtype=torch.float64)
    elif schedule == "sqrt":
        betas = torch.linspace(linear_start, linear_end, n_timestep, dtype=torch.float64) ** 0.5
    else:
        raise ValueError(f"schedule '{schedule}' unknown.")
    return betas


def _bview(sigma, ref):
    return sigma.reshape(sigma.shape[:1] + (1,) * (ref.ndim - 1))


class EPS:
    sigma_data = 1.0

    def calculate_input(self, sigma, noise):
        s = _bview(sigma, noise)
        return noise / (s * s + self.sigma_data ** 2) ** 0.5

    def calculate_denoised(self, sigma, model_output, model_input):
        return model_input - model_output * _bview(sigma, model_output)

    def noise_scaling(self, sigma, noise, latent_image, max_denoise=False):
        if max_denoise:
            noise = noise * torch.sqrt(1.0 + sigma ** 2.0)
        else:
            noise = noise * sigma
        return noise + latent_image

    def inverse_noise_scaling(self, sigma, latent):
        return latent


class V_PREDICTION(EPS):
    def calculate_denoised(self, sigma, model_output, model_input):
        s = _bview(sigma, model_output)
        sd2 = self.sigma_data ** 2
        return model_input * sd2 / (s * s + sd2) - model_output * s * self.sigma_data / (s * s + sd2) ** 0.5


class EDM(V_PREDICTION):
    def calculate_denoised(self, sigma, model_output, model_input):
        s = _bview(sigma, model_output)
        sd2 = self.sigma_data ** 2
        return model_input * sd2 / (s * s + sd2) + model_output * s * self.sigma_data / (s * s + sd2) ** 0.5


class X0(EPS):
    def calculate_denoised(self, sigma, model_output, model_input):
        return model_output


class ModelSamplingDiscrete(torch.nn.Module):
    def __init__(self, model_config=None):
        super().__init__()
        ss = getattr(model_config, "sampling_settings", None) or {}
        self._register_schedule(beta_schedule=ss.get("beta_schedule", "linear"), timesteps=1000,
                                linear_start=ss.get("linear_start", 0.00085), linear_end=ss.get("linear_end", 0.012))
        self.sigma_data = 1.0

    def _register_schedule(self, given_betas=None, beta_schedule="linear", timesteps=1000,
                           linear_start=1e-4, linear_end=2e-2, cosine_s=8e-3):
        betas = given_betas if given_betas is not None else make_beta_schedule(
            beta_schedule, timesteps, linear_start, linear_end, cosine_s)
        alphas_cumprod = torch.cumprod(1.0 - betas, dim=0)
        self.num_timesteps = int(betas.shape[0])
        self.linear_start = linear_start
        self.linear_end = linear_end
        sigmas = ((1 - alphas_cumprod) / alphas_cumprod) ** 0.5
        self.set_sigmas(sigmas)

    def set_sigmas(self, sigmas):
        self.register_buffer("sigmas", sigmas.float())
        self.register_buffer("log_sigmas", sigmas.log().float())

    @property
    def sigma_min(self):
        return self.sigmas[0]

    @property
    def sigma_max(self):
        return self.sigmas[-1]

    def timestep(self, sigma):
        log_sigma = sigma.log()
        dists = log_sigma.to(self.log_sigmas.device) - self.log_sigmas[:, None]
        return dists.abs().argmin(dim=0).view(sigma.shape).to(sigma.device)

    def sigma(self, timestep):
        t = torch.clamp(timestep.float().to(self.log_sigmas.device), min=0, max=len(self.sigmas) - 1)
        lo = t.floor().long()
        hi = t.ceil().long()
        w = t.frac()
        ls = (1 - w) * self.log_sigmas[lo] + w * self.log_sigmas[hi]
        return ls.exp().to(timestep.device)

    def percent_to_sigma(self, percent):
        if percent <= 0.0:
            return 999999999.9
        if percent >= 1.0:
            return 0.0
        return self.sigma(torch.tensor((1.0 - percent) * 999.0)).item()


class ModelSamplingDiscreteDistilled(ModelSamplingDiscrete):
    original_timesteps = 50

    def __init__(self, model_config=None):
        super().__init__(model_config)
        self.skip_steps = self.num_timesteps // self.original_timesteps
        full = self.sigmas
        idx = torch.arange(1, self.original_timesteps + 1) * self.skip_steps - 1
        self.set_sigmas(full[idx])

    def timestep(self, sigma):
        t = super().timestep(sigma)
        return (t * self.skip_steps + (self.skip_steps - 1)).to(sigma.device)

    def sigma(self, timestep):
        t = torch.clamp(((timestep.float() - (self.skip_steps - 1)) / self.skip_steps), min=0,
                        max=len(self.sigmas) - 1)
        lo = t.floor().long()
        hi = t.ceil().long()
        w = t.frac()
        ls = (1 - w) * self.log_sigmas[lo] + w * self.log_sigmas[hi]
        return ls.exp().to(timestep.device)


class LCM(EPS):
    """LCM boundary-condition scalings (c_skip/c_out) on top of an eps model."""

    def calculate_denoised(self, sigma, model_output, model_input):
        timestep = self.timestep(sigma).view(sigma.shape[:1] + (1,) * (model_output.ndim - 1))
        s = _bview(sigma, model_output)
        x0 = model_input - model_output * s
        sigma_data = 0.5
        scaled_t = timestep * 10.0
        c_skip = sigma_data ** 2 / (scaled_t ** 2 + sigma_data ** 2)
        c_out = scaled_t / (scaled_t ** 2 + sigma_data ** 2) ** 0.5
        return c_out * x0 + c_skip * model_input


class ModelSamplingContinuousEDM(torch.nn.Module):
    def __init__(self, model_config=None):
        super().__init__()
        ss = getattr(model_config, "sampling_settings", None) or {}
        self.set_parameters(ss.get("sigma_min", 0.002), ss.get("sigma_max", 120.0), ss.get("sigma_data", 1.0))

    def set_parameters(self, sigma_min, sigma_max, sigma_data):
        self.sigma_data = sigma_data
        sigmas = torch.linspace(math.log(sigma_min), math.log(sigma_max), 1000).exp()
        self.register_buffer("sigmas", sigmas)
        self.register_buffer("log_sigmas", sigmas.log())

    @property
    def sigma_min(self):
        return self.sigmas[0]

    @property
    def sigma_max(self):
        return self.sigmas[-1]

    def timestep(self, sigma):
        return 0.25 * sigma.log()

    def sigma(self, timestep):
        return (timestep / 0.25).exp()

    def percent_to_sigma(self, percent):
        if percent <= 0.0:
            return 999999999.9
        if percent >= 1.0:
            return 0.0
        percent = 1.0 - percent
        lmin = math.log(self.sigma_min)
        return math.exp((math.log(self.sigma_max) - lmin) * percent + lmin)


class StableCascadeSampling(ModelSamplingDiscrete):
    def __init__(self, model_config=None):
        torch.nn.Module.__init__(self)
        ss = getattr(model_config, "sampling_settings", None) or {}
        self.set_parameters(ss.get("shift", 1.0))

    def set_parameters(self, shift=1.0, cosine_s=8e-3):
        self.shift = shift
        self.cosine_s = torch.tensor(cosine_s)
        self._init_alpha_cumprod = torch.cos(self.cosine_s / (1 + self.cosine_s) * torch.pi * 0.5) ** 2
        self.num_timesteps = 10000
        sigmas = torch.empty(self.num_timesteps, dtype=torch.float32)
        for x in range(self.num_timesteps):
            t = (x + 1) / self.num_timesteps
            sigmas[x] = self.sigma(t)
        self.set_sigmas(sigmas)

    def sigma(self, timestep):
        t = timestep if torch.is_tensor(timestep) else torch.tensor(float(timestep))
        ac = (torch.cos((t + self.cosine_s) / (1 + self.cosine_s) * torch.pi * 0.5) ** 2 / self._init_alpha_cumprod)
        if self.shift != 1.0:
            var = ac
            logSNR = (var / (1 - var)).log()
            logSNR += 2 * torch.log(1.0 / torch.tensor(self.shift))
            ac = logSNR.sigmoid()
        ac = ac.clamp(0.0001, 0.9999)
        return ((1 - ac) / ac) ** 0.5

    def timestep(self, sigma):
        var = 1 / ((sigma * sigma) + 1)
        var = var.clamp(0, 1.0)
        # host scalars (fp32 values, applied in var's dtype): no H2D copy, so a captured step graph
        # (sampling/step_graph.py) can hold this -- a .to(device) here made every Cascade capture fail
        s, min_var = float(self.cosine_s), float(self._init_alpha_cumprod)
        t = (((var * min_var) ** 0.5).acos() / (torch.pi * 0.5)) * (1 + s) - s
        return t

    def percent_to_sigma(self, percent):
        if percent <= 0.0:
            return 999999999.9
        if percent >= 1.0:
            return 0.0
        percent = 1.0 - percent
        return float(self.sigma(torch.tensor(percent)))


def model_sampling(model_config, model_type):
    """Build the ModelSampling object for (family config, ModelType) — model_base.py:14-45."""
    from ..runtime.model_base import ModelType
    s = ModelSamplingDiscrete
    c = EPS
    if model_type == ModelType.EPS:
        c = EPS
    elif model_type == ModelType.V_PREDICTION:
        c = V_PREDICTION
    elif model_type == ModelType.V_PREDICTION_EDM:
        c = V_PREDICTION
        s = ModelSamplingContinuousEDM
    elif model_type == ModelType.EDM:
        c = EDM
        s = ModelSamplingContinuousEDM
    elif model_type == ModelType.STABLE_CASCADE:
        c = EPS
        s = StableCascadeSampling
    elif model_type == ModelType.X0:
        c = X0

    class ModelSamplingImpl(s, c):
        pass

    return ModelSamplingImpl(model_config)


def timestep_table(ms, sigmas: torch.Tensor) -> torch.Tensor:
    """Host precompute of model timesteps for every sigma of a schedule (capture-safe)."""
    return ms.timestep(sigmas.float().cpu())


def np_sigmas(sigmas) -> np.ndarray:
    return np.asarray(sigmas.detach().cpu().double().numpy())
