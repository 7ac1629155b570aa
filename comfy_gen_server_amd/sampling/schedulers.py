"""Noise schedules (parity: ``comfy/samplers.py:277-313, 660-678`` and
``comfy/k_diffusion/sampling.py:16-42``; AYS/SDTurbo from ``comfy_extras``).

All schedules are computed on the host in fp32 (the sampler loop then has every per-step scalar
as a Python float — capture-safe, no device syncs).
"""
from __future__ import annotations

import math

import numpy as np
import torch


def append_zero(x):
    return torch.cat([x, x.new_zeros([1])])


def get_sigmas_karras(n, sigma_min, sigma_max, rho=7.0, device="cpu"):
    ramp = torch.linspace(0, 1, n)
    lo, hi = sigma_min ** (1 / rho), sigma_max ** (1 / rho)
    return append_zero((hi + ramp * (lo - hi)) ** rho).to(device)


def get_sigmas_exponential(n, sigma_min, sigma_max, device="cpu"):
    return append_zero(torch.linspace(math.log(sigma_max), math.log(sigma_min), n).exp()).to(device)


def get_sigmas_polyexponential(n, sigma_min, sigma_max, rho=1.0, device="cpu"):
    ramp = torch.linspace(1, 0, n) ** rho
    return append_zero(torch.exp(ramp * (math.log(sigma_max) - math.log(sigma_min)) + math.log(sigma_min))).to(device)


def get_sigmas_vp(n, beta_d=19.9, beta_min=0.1, eps_s=1e-3, device="cpu"):
    t = torch.linspace(1, eps_s, n)
    return append_zero(torch.sqrt(torch.exp(beta_d * t ** 2 / 2 + beta_min * t) - 1)).to(device)


def simple_scheduler(ms, steps):
    n = len(ms.sigmas)
    stride = n / steps
    s = [float(ms.sigmas[-(1 + int(i * stride))]) for i in range(steps)]
    return torch.FloatTensor(s + [0.0])


def ddim_scheduler(ms, steps):
    n = len(ms.sigmas)
    stride = max(n // steps, 1)
    s = [float(ms.sigmas[i]) for i in range(1, n, stride)]
    return torch.FloatTensor(s[::-1] + [0.0])


def normal_scheduler(ms, steps, sgm=False):
    start = ms.timestep(ms.sigma_max)
    end = ms.timestep(ms.sigma_min)
    ts = torch.linspace(float(start), float(end), steps + 1)[:-1] if sgm else torch.linspace(float(start), float(end), steps)
    s = [float(ms.sigma(t)) for t in ts]
    return torch.FloatTensor(s + [0.0])


SCHEDULER_NAMES = ["normal", "karras", "exponential", "sgm_uniform", "simple", "ddim_uniform"]


def calculate_sigmas(ms, scheduler_name, steps):
    if scheduler_name == "karras":
        return get_sigmas_karras(steps, float(ms.sigma_min), float(ms.sigma_max))
    if scheduler_name == "exponential":
        return get_sigmas_exponential(steps, float(ms.sigma_min), float(ms.sigma_max))
    if scheduler_name == "normal":
        return normal_scheduler(ms, steps)
    if scheduler_name == "simple":
        return simple_scheduler(ms, steps)
    if scheduler_name == "ddim_uniform":
        return ddim_scheduler(ms, steps)
    if scheduler_name == "sgm_uniform":
        return normal_scheduler(ms, steps, sgm=True)
    raise ValueError(f"invalid scheduler {scheduler_name}")


# Align Your Steps (comfy_extras/nodes_align_your_steps.py) ---------------------------------------
AYS_NOISE_LEVELS = {
    "SD1": [14.6146412293, 6.4745760956, 3.8636745985, 2.6946151520, 1.8841921177, 1.3943805092,
            0.9642583904, 0.6523686016, 0.3977456272, 0.1515232662, 0.0291671582],
    "SDXL": [14.6146412293, 6.3184485287, 3.7681790315, 2.1811480769, 1.3405244945, 0.8620721141,
             0.5550693289, 0.3798540708, 0.2332364134, 0.1114188177, 0.0291671582],
    "SVD": [700.00, 54.5, 15.886, 7.977, 4.248, 1.789, 0.981, 0.403, 0.173, 0.034, 0.002],
}


def loglinear_interp(t_steps, num_steps):
    xs = np.linspace(0, 1, len(t_steps))
    ys = np.log(t_steps[::-1])
    new_xs = np.linspace(0, 1, num_steps)
    new_ys = np.interp(new_xs, xs, ys)
    return np.exp(new_ys)[::-1].copy()


def ays_sigmas(model_type, steps, denoise=1.0):
    total = steps
    if denoise < 1.0:
        if denoise <= 0.0:
            return torch.FloatTensor([])
        total = round(steps * denoise)
    sig = AYS_NOISE_LEVELS[model_type][:]
    if (steps + 1) != len(sig):
        sig = loglinear_interp(sig, steps + 1)
    sig = list(sig[-(total + 1):])
    sig[-1] = 0
    return torch.FloatTensor(sig)


def sd_turbo_sigmas(ms, steps, denoise=1.0):
    start = 10 - int(10 * denoise)
    ts = torch.flip(torch.arange(1, 11) * 100 - 1, (0,))[start:start + steps]
    return torch.cat([ms.sigma(ts).float(), ts.new_zeros([1]).float()])
