"""k-diffusion sampler zoo (parity: ``comfy/k_diffusion/sampling.py:1-810``; C24).

Every sampler keeps the reference calling convention
``sample_x(model, x, sigmas, extra_args=None, callback=None, disable=None, **opts)`` so custom
sampler nodes keep working, but the per-step scalars (sigma, sigma_next, ancestral sigma_up /
sigma_down, log-sigma steps h) are computed on the HOST from a float copy of ``sigmas`` — the
reference evaluates them on device tensors (``get_ancestral_step`` min on tensors, ``sigmas[i+1] > 0``)
which costs a device sync per step and breaks hipGraph capture. The element-wise updates of
Euler / Euler-a run as one fused HIP kernel on the device (``ops.euler_step``).

Noise: ancestral / SDE noise is counter-based (``rng.py`` / ``csrc/kernels/rng.hip``): the value
for image b at sampler call k is a function of (``extra_args['seed']``, the image's GLOBAL batch
index ``extra_args['noise_inds'][b]``, k) only, so a data-parallel split of a batch reproduces the
one-GPU run exactly (the reference draws ``randn_like`` from the global RNG,
``comfy/k_diffusion/sampling.py:60-61``). Euler-a generates its noise inside the update kernel.
SDE samplers use a per-image virtual Brownian tree walked on the device (``brownian.py``) instead of
torchsde.
"""
from __future__ import annotations

import math

import torch

from .. import ops
from .brownian import BrownianTreeNoiseSampler
from .rng import StepNoise
from . import step_graph


def _f(sigmas):
    return [float(s) for s in sigmas.detach().cpu()]


def to_d(x, sigma, denoised):
    return (x - denoised) / sigma


def get_ancestral_step(sigma_from: float, sigma_to: float, eta: float = 1.0):
    if not eta:
        return sigma_to, 0.0
    up = min(sigma_to, eta * math.sqrt(max(0.0, sigma_to ** 2 * (sigma_from ** 2 - sigma_to ** 2) / sigma_from ** 2)))
    down = math.sqrt(max(0.0, sigma_to ** 2 - up ** 2))
    return down, up


def default_noise_sampler(x, seed=None, inds=None):
    if seed is None:
        return lambda sigma, sigma_next: torch.randn_like(x)
    return StepNoise(x, seed, inds)


def _s_in(x):
    return x.new_ones([x.shape[0]])


def _model(model, x, sigma: float, extra_args, s_in):
    from .samplers import current_sigma
    tok = current_sigma.set(float(sigma))    # host copy for timestep gating (no D2H sync)
    try:
        return model(x, s_in * sigma, **extra_args)
    finally:
        current_sigma.reset(tok)


def _cb(callback, i, x, sigma, sigma_hat, denoised):
    if callback is not None:
        callback({"x": x, "i": i, "sigma": sigma, "sigma_hat": sigma_hat, "denoised": denoised})


def _noise_sampler(x, extra_args, noise_sampler):
    if noise_sampler is not None:
        return noise_sampler
    return default_noise_sampler(x, extra_args.get("seed"), extra_args.get("noise_inds"))


def _brownian(x, extra_args, sigma_min, sigma_max, cpu=False):
    return BrownianTreeNoiseSampler(x, sigma_min, sigma_max, seed=extra_args.get("seed"), cpu=cpu,
                                    inds=extra_args.get("noise_inds"))


@torch.no_grad()
def sample_euler(model, x, sigmas, extra_args=None, callback=None, disable=None, s_churn=0.0, s_tmin=0.0,
                 s_tmax=float("inf"), s_noise=1.0):
    extra_args = {} if extra_args is None else extra_args
    if s_churn == 0:
        r = step_graph.try_sample(model, x, sigmas, extra_args, callback, "euler")
        if r is not None:
            return r
    s = _f(sigmas)
    s_in = _s_in(x)
    n = len(s) - 1
    for i in range(n):
        gamma = min(s_churn / n, 2 ** 0.5 - 1) if s_tmin <= s[i] <= s_tmax else 0.0
        sigma_hat = s[i] * (gamma + 1)
        if gamma > 0:
            eps = torch.randn_like(x) * s_noise
            x = x + eps * (sigma_hat ** 2 - s[i] ** 2) ** 0.5
        denoised = _model(model, x, sigma_hat, extra_args, s_in)
        _cb(callback, i, x, s[i], sigma_hat, denoised)
        x = ops.euler_step(x, denoised, None, sigma_hat, s[i + 1], 0.0)
    return x


@torch.no_grad()
def sample_euler_ancestral(model, x, sigmas, extra_args=None, callback=None, disable=None, eta=1.0, s_noise=1.0,
                           noise_sampler=None):
    extra_args = {} if extra_args is None else extra_args
    if noise_sampler is None:
        r = step_graph.try_sample(model, x, sigmas, extra_args, callback, "euler_ancestral", eta, s_noise)
        if r is not None:
            return r
    ns = _noise_sampler(x, extra_args, noise_sampler)
    s = _f(sigmas)
    s_in = _s_in(x)
    for i in range(len(s) - 1):
        denoised = _model(model, x, s[i], extra_args, s_in)
        down, up = get_ancestral_step(s[i], s[i + 1], eta=eta)
        _cb(callback, i, x, s[i], s[i], denoised)
        if s[i + 1] <= 0:
            x = ops.euler_step(x, denoised, None, s[i], down, 0.0)
        elif isinstance(ns, StepNoise) and s_noise == 1.0:
            # noise generated in the update kernel's registers (stream = this sampler's call count)
            x = ops.euler_ancestral_philox(x, denoised, s[i], down, up, ns.seed, ns.inds, ns.calls)
            ns.calls += 1
        else:
            x = ops.euler_step(x, denoised, ns(s[i], s[i + 1]) * s_noise, s[i], down, up)
    return x


@torch.no_grad()
def sample_heun(model, x, sigmas, extra_args=None, callback=None, disable=None, s_churn=0.0, s_tmin=0.0,
                s_tmax=float("inf"), s_noise=1.0):
    extra_args = {} if extra_args is None else extra_args
    s = _f(sigmas)
    s_in = _s_in(x)
    n = len(s) - 1
    for i in range(n):
        gamma = min(s_churn / n, 2 ** 0.5 - 1) if s_tmin <= s[i] <= s_tmax else 0.0
        sigma_hat = s[i] * (gamma + 1)
        if gamma > 0:
            x = x + torch.randn_like(x) * s_noise * (sigma_hat ** 2 - s[i] ** 2) ** 0.5
        denoised = _model(model, x, sigma_hat, extra_args, s_in)
        d = to_d(x, sigma_hat, denoised)
        _cb(callback, i, x, s[i], sigma_hat, denoised)
        dt = s[i + 1] - sigma_hat
        if s[i + 1] == 0:
            x = x + d * dt
        else:
            x2 = x + d * dt
            denoised2 = _model(model, x2, s[i + 1], extra_args, s_in)
            d2 = to_d(x2, s[i + 1], denoised2)
            x = x + (d + d2) / 2 * dt
    return x


@torch.no_grad()
def sample_dpm_2(model, x, sigmas, extra_args=None, callback=None, disable=None, s_churn=0.0, s_tmin=0.0,
                 s_tmax=float("inf"), s_noise=1.0):
    extra_args = {} if extra_args is None else extra_args
    s = _f(sigmas)
    s_in = _s_in(x)
    n = len(s) - 1
    for i in range(n):
        gamma = min(s_churn / n, 2 ** 0.5 - 1) if s_tmin <= s[i] <= s_tmax else 0.0
        sigma_hat = s[i] * (gamma + 1)
        if gamma > 0:
            x = x + torch.randn_like(x) * s_noise * (sigma_hat ** 2 - s[i] ** 2) ** 0.5
        denoised = _model(model, x, sigma_hat, extra_args, s_in)
        d = to_d(x, sigma_hat, denoised)
        _cb(callback, i, x, s[i], sigma_hat, denoised)
        if s[i + 1] == 0:
            x = x + d * (s[i + 1] - sigma_hat)
        else:
            sigma_mid = math.exp(0.5 * (math.log(sigma_hat) + math.log(s[i + 1])))
            x2 = x + d * (sigma_mid - sigma_hat)
            denoised2 = _model(model, x2, sigma_mid, extra_args, s_in)
            d2 = to_d(x2, sigma_mid, denoised2)
            x = x + d2 * (s[i + 1] - sigma_hat)
    return x


@torch.no_grad()
def sample_dpm_2_ancestral(model, x, sigmas, extra_args=None, callback=None, disable=None, eta=1.0, s_noise=1.0,
                           noise_sampler=None):
    extra_args = {} if extra_args is None else extra_args
    ns = _noise_sampler(x, extra_args, noise_sampler)
    s = _f(sigmas)
    s_in = _s_in(x)
    for i in range(len(s) - 1):
        denoised = _model(model, x, s[i], extra_args, s_in)
        down, up = get_ancestral_step(s[i], s[i + 1], eta=eta)
        _cb(callback, i, x, s[i], s[i], denoised)
        d = to_d(x, s[i], denoised)
        if down == 0:
            x = x + d * (down - s[i])
        else:
            sigma_mid = math.exp(0.5 * (math.log(s[i]) + math.log(down)))
            x2 = x + d * (sigma_mid - s[i])
            denoised2 = _model(model, x2, sigma_mid, extra_args, s_in)
            d2 = to_d(x2, sigma_mid, denoised2)
            x = x + d2 * (down - s[i])
            x = x + ns(s[i], s[i + 1]) * s_noise * up
    return x


def linear_multistep_coeff(order, t, i, j):
    if order - 1 > i:
        raise ValueError(f"Order {order} too high for step {i}")
    from scipy import integrate

    def fn(tau):
        prod = 1.0
        for k in range(order):
            if j == k:
                continue
            prod *= (tau - t[i - k]) / (t[i - j] - t[i - k])
        return prod
    return integrate.quad(fn, t[i], t[i + 1], epsrel=1e-4)[0]


@torch.no_grad()
def sample_lms(model, x, sigmas, extra_args=None, callback=None, disable=None, order=4):
    extra_args = {} if extra_args is None else extra_args
    s = _f(sigmas)
    s_in = _s_in(x)
    ds = []
    for i in range(len(s) - 1):
        denoised = _model(model, x, s[i], extra_args, s_in)
        ds.append(to_d(x, s[i], denoised))
        if len(ds) > order:
            ds.pop(0)
        _cb(callback, i, x, s[i], s[i], denoised)
        cur = min(i + 1, order)      # the last step integrates to sigma 0 too (sampling.py:282-284)
        coeffs = [linear_multistep_coeff(cur, s, i, j) for j in range(cur)]
        x = x + sum(c * d for c, d in zip(coeffs, reversed(ds)))
    return x


@torch.no_grad()
def sample_dpmpp_2s_ancestral(model, x, sigmas, extra_args=None, callback=None, disable=None, eta=1.0, s_noise=1.0,
                              noise_sampler=None):
    extra_args = {} if extra_args is None else extra_args
    ns = _noise_sampler(x, extra_args, noise_sampler)
    s = _f(sigmas)
    s_in = _s_in(x)
    for i in range(len(s) - 1):
        denoised = _model(model, x, s[i], extra_args, s_in)
        down, up = get_ancestral_step(s[i], s[i + 1], eta=eta)
        _cb(callback, i, x, s[i], s[i], denoised)
        if down == 0:
            x = x + to_d(x, s[i], denoised) * (down - s[i])
        else:
            t, t_next = -math.log(s[i]), -math.log(down)
            h = t_next - t
            r = 0.5
            s_ = t + r * h
            sig_s = math.exp(-s_)
            x2 = (sig_s / s[i]) * x - math.expm1(-h * r) * denoised
            denoised2 = _model(model, x2, sig_s, extra_args, s_in)
            x = (down / s[i]) * x - math.expm1(-h) * denoised2
        if s[i + 1] > 0:
            x = x + ns(s[i], s[i + 1]) * s_noise * up
    return x


@torch.no_grad()
def sample_dpmpp_sde(model, x, sigmas, extra_args=None, callback=None, disable=None, eta=1.0, s_noise=1.0,
                     noise_sampler=None, r=0.5):
    extra_args = {} if extra_args is None else extra_args
    s = _f(sigmas)
    pos = [v for v in s if v > 0]
    ns = noise_sampler or _brownian(x, extra_args, min(pos), max(s), cpu=True)
    s_in = _s_in(x)
    for i in range(len(s) - 1):
        denoised = _model(model, x, s[i], extra_args, s_in)
        _cb(callback, i, x, s[i], s[i], denoised)
        if s[i + 1] == 0:
            x = x + to_d(x, s[i], denoised) * (s[i + 1] - s[i])
            continue
        t, t_next = -math.log(s[i]), -math.log(s[i + 1])
        h = t_next - t
        s_mid = t + h * r
        fac = 1 / (2 * r)
        sig = lambda tt: math.exp(-tt)  # noqa: E731
        # step 1: ancestral step to the midpoint; the model is evaluated AT the midpoint
        sd, su = get_ancestral_step(sig(t), sig(s_mid), eta)
        s_ = -math.log(sd)
        x2 = (sig(s_) / sig(t)) * x - math.expm1(t - s_) * denoised
        x2 = x2 + ns(sig(t), sig(s_mid)) * s_noise * su
        denoised2 = _model(model, x2, sig(s_mid), extra_args, s_in)
        # step 2
        sd, su = get_ancestral_step(sig(t), sig(t_next), eta)
        t_next_ = -math.log(sd)
        denoised_d = (1 - fac) * denoised + fac * denoised2
        x = (sig(t_next_) / sig(t)) * x - math.expm1(t - t_next_) * denoised_d
        x = x + ns(sig(t), sig(t_next)) * s_noise * su
    return x


@torch.no_grad()
def sample_dpmpp_2m(model, x, sigmas, extra_args=None, callback=None, disable=None):
    extra_args = {} if extra_args is None else extra_args
    r = step_graph.try_sample(model, x, sigmas, extra_args, callback, "dpmpp_2m")
    if r is not None:
        return r
    s = _f(sigmas)
    s_in = _s_in(x)
    old = None
    for i in range(len(s) - 1):
        denoised = _model(model, x, s[i], extra_args, s_in)
        _cb(callback, i, x, s[i], s[i], denoised)
        if s[i + 1] == 0:
            x = denoised
            old = denoised
            continue
        t, t_next = -math.log(s[i]), -math.log(s[i + 1])
        h = t_next - t
        if old is None:
            x = (s[i + 1] / s[i]) * x - math.expm1(-h) * denoised
        else:
            h_last = t - (-math.log(s[i - 1]))
            r = h_last / h
            dd = (1 + 1 / (2 * r)) * denoised - (1 / (2 * r)) * old
            x = (s[i + 1] / s[i]) * x - math.expm1(-h) * dd
        old = denoised
    return x


@torch.no_grad()
def sample_dpmpp_2m_sde(model, x, sigmas, extra_args=None, callback=None, disable=None, eta=1.0, s_noise=1.0,
                        noise_sampler=None, solver_type="midpoint", _cpu_tree=True):
    if solver_type not in ("heun", "midpoint"):
        raise ValueError("solver_type must be 'heun' or 'midpoint'")
    extra_args = {} if extra_args is None else extra_args
    s = _f(sigmas)
    pos = [v for v in s if v > 0]
    ns = noise_sampler or _brownian(x, extra_args, min(pos), max(s), cpu=_cpu_tree)
    s_in = _s_in(x)
    old = None
    h_last = None
    h = None
    for i in range(len(s) - 1):
        denoised = _model(model, x, s[i], extra_args, s_in)
        _cb(callback, i, x, s[i], s[i], denoised)
        if s[i + 1] == 0:
            x = denoised
        else:
            t, tn = -math.log(s[i]), -math.log(s[i + 1])
            h = tn - t
            eta_h = eta * h
            x = (s[i + 1] / s[i]) * math.exp(-eta_h) * x + (-math.expm1(-h - eta_h)) * denoised
            if old is not None:
                r = h_last / h
                if solver_type == "heun":
                    x = x + ((-math.expm1(-h - eta_h)) / (-h - eta_h) + 1) * (1 / r) * (denoised - old)
                else:
                    x = x + 0.5 * (-math.expm1(-h - eta_h)) * (1 / r) * (denoised - old)
            if eta:
                x = x + ns(s[i], s[i + 1]) * s[i + 1] * math.sqrt(-math.expm1(-2 * eta_h)) * s_noise
        old = denoised
        h_last = h
    return x


@torch.no_grad()
def sample_dpmpp_3m_sde(model, x, sigmas, extra_args=None, callback=None, disable=None, eta=1.0, s_noise=1.0,
                        noise_sampler=None, _cpu_tree=True):
    extra_args = {} if extra_args is None else extra_args
    s = _f(sigmas)
    pos = [v for v in s if v > 0]
    ns = noise_sampler or _brownian(x, extra_args, min(pos), max(s), cpu=_cpu_tree)
    s_in = _s_in(x)
    d1 = d2 = None
    h1 = h2 = None
    for i in range(len(s) - 1):
        denoised = _model(model, x, s[i], extra_args, s_in)
        _cb(callback, i, x, s[i], s[i], denoised)
        if s[i + 1] == 0:
            x = denoised
        else:
            t, s_ = -math.log(s[i]), -math.log(s[i + 1])
            h = s_ - t
            h_eta = h * (eta + 1)
            x = math.exp(-h_eta) * x + (-math.expm1(-h_eta)) * denoised
            if h2 is not None:
                r0 = h1 / h
                r1 = h2 / h
                d1_0 = (denoised - d1) / r0
                d1_1 = (d1 - d2) / r1
                d1_ = d1_0 + (d1_0 - d1_1) * r0 / (r0 + r1)
                d2_ = (d1_0 - d1_1) / (r0 + r1)
                phi_2 = math.expm1(-h_eta) / h_eta + 1
                phi_3 = phi_2 / h_eta - 0.5
                x = x + phi_2 * d1_ - phi_3 * d2_
            elif h1 is not None:
                r = h1 / h
                dd = (denoised - d1) / r
                phi_2 = math.expm1(-h_eta) / h_eta + 1
                x = x + phi_2 * dd
            if eta:
                x = x + ns(s[i], s[i + 1]) * s[i + 1] * math.sqrt(-math.expm1(-2 * h * eta)) * s_noise
            h1, h2 = h, h1
        d1, d2 = denoised, d1
    return x


def sample_dpmpp_sde_gpu(model, x, sigmas, extra_args=None, callback=None, disable=None, eta=1.0, s_noise=1.0,
                         noise_sampler=None, r=0.5):
    extra_args = {} if extra_args is None else extra_args
    s = _f(sigmas)
    pos = [v for v in s if v > 0]
    ns = noise_sampler or _brownian(x, extra_args, min(pos), max(s), cpu=False)
    return sample_dpmpp_sde(model, x, sigmas, extra_args, callback, disable, eta, s_noise, ns, r)


def sample_dpmpp_2m_sde_gpu(model, x, sigmas, extra_args=None, callback=None, disable=None, eta=1.0, s_noise=1.0,
                            noise_sampler=None, solver_type="midpoint"):
    return sample_dpmpp_2m_sde(model, x, sigmas, extra_args, callback, disable, eta, s_noise, noise_sampler,
                               solver_type, _cpu_tree=False)


def sample_dpmpp_3m_sde_gpu(model, x, sigmas, extra_args=None, callback=None, disable=None, eta=1.0, s_noise=1.0,
                            noise_sampler=None):
    return sample_dpmpp_3m_sde(model, x, sigmas, extra_args, callback, disable, eta, s_noise, noise_sampler,
                               _cpu_tree=False)


@torch.no_grad()
def sample_heunpp2(model, x, sigmas, extra_args=None, callback=None, disable=None, s_churn=0.0, s_tmin=0.0,
                   s_tmax=float("inf"), s_noise=1.0):
    extra_args = {} if extra_args is None else extra_args
    s = _f(sigmas)
    s_in = _s_in(x)
    s_end = s[-1]
    n = len(s) - 1
    for i in range(n):
        gamma = min(s_churn / n, 2 ** 0.5 - 1) if s_tmin <= s[i] <= s_tmax else 0.0
        sigma_hat = s[i] * (gamma + 1)
        if gamma > 0:
            x = x + torch.randn_like(x) * s_noise * (sigma_hat ** 2 - s[i] ** 2) ** 0.5
        denoised = _model(model, x, sigma_hat, extra_args, s_in)
        d = to_d(x, sigma_hat, denoised)
        _cb(callback, i, x, s[i], sigma_hat, denoised)
        dt = s[i + 1] - sigma_hat
        if s[i + 1] == s_end:
            x = x + d * dt
        elif s[i + 2] == s_end:
            x2 = x + d * dt
            denoised2 = _model(model, x2, s[i + 1], extra_args, s_in)
            d2 = to_d(x2, s[i + 1], denoised2)
            w = 2 * s[0]
            w2 = s[i + 1] / w
            w1 = 1 - w2
            x = x + (d * w1 + d2 * w2) * dt
        else:
            x2 = x + d * dt
            denoised2 = _model(model, x2, s[i + 1], extra_args, s_in)
            d2 = to_d(x2, s[i + 1], denoised2)
            dt2 = s[i + 2] - s[i + 1]
            x3 = x2 + d2 * dt2
            denoised3 = _model(model, x3, s[i + 2], extra_args, s_in)
            d3 = to_d(x3, s[i + 2], denoised3)
            w = 3 * s[0]
            w2 = s[i + 1] / w
            w3 = s[i + 2] / w
            w1 = 1 - w2 - w3
            x = x + (w1 * d + w2 * d2 + w3 * d3) * dt
    return x


def _alphas_cumprod(model):
    ms = model.inner_model.inner_model.model_sampling
    return ms


def generic_step_sampler(model, x, sigmas, extra_args=None, callback=None, disable=None, noise_sampler=None,
                         step_function=None):
    extra_args = {} if extra_args is None else extra_args
    ns = _noise_sampler(x, extra_args, noise_sampler)
    s = _f(sigmas)
    s_in = _s_in(x)
    for i in range(len(s) - 1):
        denoised = _model(model, x, s[i], extra_args, s_in)
        _cb(callback, i, x, s[i], s[i], denoised)
        x = step_function(x / math.sqrt(1.0 + s[i] ** 2.0), s[i], s[i + 1],
                          (x - denoised) / s[i], ns)
        if s[i + 1] != 0:
            x = x * math.sqrt(1.0 + s[i + 1] ** 2.0)
    return x


def DDPMSampler_step(x, sigma, sigma_prev, noise, noise_sampler):
    alpha_cumprod = 1 / ((sigma * sigma) + 1)
    alpha_cumprod_prev = 1 / ((sigma_prev * sigma_prev) + 1)
    alpha = alpha_cumprod / alpha_cumprod_prev
    mu = (1.0 / math.sqrt(alpha)) * (x - (1 - alpha) * noise / math.sqrt(1 - alpha_cumprod))
    if sigma_prev > 0:
        mu = mu + math.sqrt((1 - alpha) * (1. - alpha_cumprod_prev) / (1. - alpha_cumprod)) * noise_sampler(sigma, sigma_prev)
    return mu


def sample_ddpm(model, x, sigmas, extra_args=None, callback=None, disable=None, noise_sampler=None):
    return generic_step_sampler(model, x, sigmas, extra_args, callback, disable, noise_sampler, DDPMSampler_step)


@torch.no_grad()
def sample_lcm(model, x, sigmas, extra_args=None, callback=None, disable=None, noise_sampler=None):
    extra_args = {} if extra_args is None else extra_args
    if noise_sampler is None:
        r = step_graph.try_sample(model, x, sigmas, extra_args, callback, "lcm")
        if r is not None:
            return r
    ns = _noise_sampler(x, extra_args, noise_sampler)
    s = _f(sigmas)
    s_in = _s_in(x)
    for i in range(len(s) - 1):
        denoised = _model(model, x, s[i], extra_args, s_in)
        _cb(callback, i, x, s[i], s[i], denoised)
        x = denoised
        if s[i + 1] > 0:
            x = x + s[i + 1] * ns(s[i], s[i + 1])
    return x


# ------------------------------------------------------------------------------------------------
# DPM-Solver (fast / adaptive) — Lu et al. 2022, in log-sigma time t = -log(sigma)
# ------------------------------------------------------------------------------------------------
class DPMSolver:
    def __init__(self, model, extra_args=None, eps_callback=None, info_callback=None):
        self.model = model
        self.extra_args = {} if extra_args is None else extra_args
        self.eps_callback = eps_callback
        self.info_callback = info_callback

    def t(self, sigma):
        return -math.log(sigma)

    def sigma(self, t):
        return math.exp(-t)

    def eps(self, cache, key, x, t, *args, **kw):
        if key in cache:
            return cache[key], cache
        sigma = self.sigma(t)
        s_in = x.new_ones([x.shape[0]])
        eps = (x - self.model(x, s_in * sigma, *args, **self.extra_args, **kw)) / sigma
        if self.eps_callback is not None:
            self.eps_callback()
        return eps, {key: eps, **cache}

    def dpm_solver_1_step(self, x, t, t_next, eps_cache=None):
        eps_cache = {} if eps_cache is None else eps_cache
        h = t_next - t
        eps, eps_cache = self.eps(eps_cache, "eps", x, t)
        return x - self.sigma(t_next) * math.expm1(h) * eps, eps_cache

    def dpm_solver_2_step(self, x, t, t_next, r1=1 / 2, eps_cache=None):
        eps_cache = {} if eps_cache is None else eps_cache
        h = t_next - t
        eps, eps_cache = self.eps(eps_cache, "eps", x, t)
        s1 = t + r1 * h
        u1 = x - self.sigma(s1) * math.expm1(r1 * h) * eps
        eps_r1, eps_cache = self.eps(eps_cache, "eps_r1", u1, s1)
        return x - self.sigma(t_next) * math.expm1(h) * eps - self.sigma(t_next) / (2 * r1) * math.expm1(h) * (eps_r1 - eps), eps_cache

    def dpm_solver_3_step(self, x, t, t_next, r1=1 / 3, r2=2 / 3, eps_cache=None):
        eps_cache = {} if eps_cache is None else eps_cache
        h = t_next - t
        eps, eps_cache = self.eps(eps_cache, "eps", x, t)
        s1 = t + r1 * h
        s2 = t + r2 * h
        u1 = x - self.sigma(s1) * math.expm1(r1 * h) * eps
        eps_r1, eps_cache = self.eps(eps_cache, "eps_r1", u1, s1)
        u2 = x - self.sigma(s2) * math.expm1(r2 * h) * eps - self.sigma(s2) * (r2 / r1) * (math.expm1(r2 * h) / (r2 * h) - 1) * (eps_r1 - eps)
        eps_r2, eps_cache = self.eps(eps_cache, "eps_r2", u2, s2)
        return x - self.sigma(t_next) * math.expm1(h) * eps - self.sigma(t_next) / r2 * (math.expm1(h) / h - 1) * (eps_r2 - eps), eps_cache

    def dpm_solver_fast(self, x, t_start, t_end, nfe, eta=0.0, s_noise=1.0, noise_sampler=None):
        noise_sampler = _noise_sampler(x, self.extra_args, noise_sampler)
        if not t_end > t_start and eta:
            raise ValueError("eta must be 0 for reverse sampling")
        m = math.floor(nfe / 3) + 1
        ts = [t_start + (t_end - t_start) * k / m for k in range(m + 1)]
        if nfe % 3 == 0:
            orders = [3] * (m - 2) + [2, 1]
        else:
            orders = [3] * (m - 1) + [nfe % 3]
        for i in range(len(orders)):
            eps_cache = {}
            t, t_next = ts[i], ts[i + 1]
            if eta:
                sd, su = get_ancestral_step(self.sigma(t), self.sigma(t_next), eta)
                t_next_ = min(t_next, self.t(sd))
                su = math.sqrt(max(0.0, self.sigma(t_next) ** 2 - self.sigma(t_next_) ** 2))
            else:
                t_next_, su = t_next, 0.0
            eps, eps_cache = self.eps(eps_cache, "eps", x, t)
            denoised = x - self.sigma(t) * eps
            if self.info_callback is not None:
                self.info_callback({"x": x, "i": i, "t": t, "t_up": t, "denoised": denoised})
            if orders[i] == 1:
                x, eps_cache = self.dpm_solver_1_step(x, t, t_next_, eps_cache=eps_cache)
            elif orders[i] == 2:
                x, eps_cache = self.dpm_solver_2_step(x, t, t_next_, eps_cache=eps_cache)
            else:
                x, eps_cache = self.dpm_solver_3_step(x, t, t_next_, eps_cache=eps_cache)
            x = x + su * s_noise * noise_sampler(self.sigma(t), self.sigma(t_next))
        return x

    def dpm_solver_adaptive(self, x, t_start, t_end, order=3, rtol=0.05, atol=0.0078, h_init=0.05, pcoeff=0.0,
                            icoeff=1.0, dcoeff=0.0, accept_safety=0.81, eta=0.0, s_noise=1.0, noise_sampler=None):
        noise_sampler = _noise_sampler(x, self.extra_args, noise_sampler)
        if order not in {2, 3}:
            raise ValueError("order should be 2 or 3")
        forward = t_end > t_start
        if not forward and eta:
            raise ValueError("eta must be 0 for reverse sampling")
        h_init = abs(h_init) * (1 if forward else -1)
        atol_ = atol
        rtol_ = rtol
        s = t_start
        x_prev = x
        accept = True
        pid = PIDStepSizeController(h_init, pcoeff, icoeff, dcoeff, 1.5 if eta else order, accept_safety)
        info = {"steps": 0, "nfe": 0, "n_accept": 0, "n_reject": 0}
        while (s < t_end - 1e-5) if forward else (s > t_end + 1e-5):
            eps_cache = {}
            t = min(t_end, s + pid.h) if forward else max(t_end, s + pid.h)
            if eta:
                sd, su = get_ancestral_step(self.sigma(s), self.sigma(t), eta)
                t_ = min(t, self.t(sd))
                su = math.sqrt(max(0.0, self.sigma(t) ** 2 - self.sigma(t_) ** 2))
            else:
                t_, su = t, 0.0
            eps, eps_cache = self.eps(eps_cache, "eps", x, s)
            denoised = x - self.sigma(s) * eps
            if order == 2:
                x_low, eps_cache = self.dpm_solver_1_step(x, s, t_, eps_cache=eps_cache)
                x_high, eps_cache = self.dpm_solver_2_step(x, s, t_, eps_cache=eps_cache)
            else:
                x_low, eps_cache = self.dpm_solver_2_step(x, s, t_, r1=1 / 3, eps_cache=eps_cache)
                x_high, eps_cache = self.dpm_solver_3_step(x, s, t_, eps_cache=eps_cache)
            delta = torch.maximum(torch.full_like(x_low, atol_), rtol_ * torch.maximum(x_low.abs(), x_prev.abs()))
            error = torch.linalg.norm((x_low - x_high) / delta) / x.numel() ** 0.5
            accept = pid.propose_step(float(error))
            if accept:
                x_prev = x_low
                x = x_high + su * s_noise * noise_sampler(self.sigma(s), self.sigma(t))
                s = t
                info["n_accept"] += 1
            else:
                info["n_reject"] += 1
            info["nfe"] += order
            info["steps"] += 1
            if self.info_callback is not None:
                self.info_callback({"x": x, "i": info["steps"] - 1, "t": s, "t_up": s, "denoised": denoised,
                                    "error": error, "h": pid.h, **info})
        return x, info


class PIDStepSizeController:
    def __init__(self, h, pcoeff, icoeff, dcoeff, order=1, accept_safety=0.81, eps=1e-8):
        self.h = h
        self.b1 = (pcoeff + icoeff + dcoeff) / order
        self.b2 = -(pcoeff + 2 * dcoeff) / order
        self.b3 = dcoeff / order
        self.accept_safety = accept_safety
        self.eps = eps
        self.errs = []

    def limiter(self, x):
        return 1 + math.atan(x - 1)

    def propose_step(self, error):
        inv_error = 1 / (error + self.eps)
        if not self.errs:
            self.errs = [inv_error, inv_error, inv_error]
        self.errs[0] = inv_error
        factor = self.errs[0] ** self.b1 * self.errs[1] ** self.b2 * self.errs[2] ** self.b3
        factor = self.limiter(factor)
        accept = factor >= self.accept_safety
        if accept:
            self.errs[2] = self.errs[1]
            self.errs[1] = self.errs[0]
        self.h *= factor
        return accept


@torch.no_grad()
def sample_dpm_fast(model, x, sigma_min, sigma_max, n, extra_args=None, callback=None, disable=None, eta=0.0,
                    s_noise=1.0, noise_sampler=None):
    if sigma_min <= 0 or sigma_max <= 0:
        raise ValueError("sigma_min and sigma_max must not be 0")
    cb = (lambda info: callback({"sigma": math.exp(-info["t"]), "sigma_hat": math.exp(-info["t_up"]), **info})) \
        if callback is not None else None
    solver = DPMSolver(model, extra_args, info_callback=cb)
    return solver.dpm_solver_fast(x, -math.log(float(sigma_max)), -math.log(float(sigma_min)), n, eta, s_noise, noise_sampler)


@torch.no_grad()
def sample_dpm_adaptive(model, x, sigma_min, sigma_max, extra_args=None, callback=None, disable=None, order=3,
                        rtol=0.05, atol=0.0078, h_init=0.05, pcoeff=0.0, icoeff=1.0, dcoeff=0.0, accept_safety=0.81,
                        eta=0.0, s_noise=1.0, noise_sampler=None, return_info=False):
    if sigma_min <= 0 or sigma_max <= 0:
        raise ValueError("sigma_min and sigma_max must not be 0")
    cb = (lambda info: callback({"sigma": math.exp(-info["t"]), "sigma_hat": math.exp(-info["t_up"]), **info})) \
        if callback is not None else None
    solver = DPMSolver(model, extra_args, info_callback=cb)
    x, info = solver.dpm_solver_adaptive(x, -math.log(float(sigma_max)), -math.log(float(sigma_min)), order, rtol,
                                         atol, h_init, pcoeff, icoeff, dcoeff, accept_safety, eta, s_noise, noise_sampler)
    return (x, info) if return_info else x
