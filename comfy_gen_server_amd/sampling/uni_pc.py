"""UniPC multistep predictor-corrector sampler, bh1 / bh2 variants (Zhao et al., 2023).

Behavioural parity with ``comfy/extra_samplers/uni_pc.py:848-874`` (``sample_unipc`` /
``sample_unipc_bh2``: data prediction, time-uniform given sigmas, order min(3, steps-1),
lower-order final steps, last sigma 0 replaced by 1e-3, VP <-> k-diffusion conversion).
Written directly in the sigma parameterisation: with alpha = 1/sqrt(1+s^2), s_vp = s*alpha and
lambda = -log(s), the data-prediction model is exactly the k-diffusion denoiser D(x, s).
"""
from __future__ import annotations

import math

import torch


def _alpha(s):
    return 1.0 / math.sqrt(1.0 + s * s)


def _lam(s):
    return -math.log(s)


def _unipc_update(x, model_prev, lam_prev, sig_prev, s_t, order, variant, use_corrector, denoise_fn):
    """One UniPC step from the history (lists ordered oldest..newest) to sigma ``s_t``.
    Works on the VP state x_vp; model values are x0 predictions."""
    a_t = _alpha(s_t)
    sv_t = s_t * a_t
    lam_t = _lam(s_t)
    m0 = model_prev[-1]
    lam0 = lam_prev[-1]
    sv0 = sig_prev[-1]
    h = lam_t - lam0
    rks, d1s = [], []
    for i in range(1, order):
        lam_i = lam_prev[-(i + 1)]
        rk = (lam_i - lam0) / h
        rks.append(rk)
        d1s.append((model_prev[-(i + 1)] - m0) / rk)
    rks.append(1.0)
    hh = -h
    h_phi_1 = math.expm1(hh)
    h_phi_k = h_phi_1 / hh - 1.0
    fact = 1
    if variant == "bh1":
        b_h = hh
    elif variant == "bh2":
        b_h = math.expm1(hh)
    else:
        raise NotImplementedError(variant)
    R, b = [], []
    for i in range(1, order + 1):
        R.append([rk ** (i - 1) for rk in rks])
        b.append(h_phi_k * fact / b_h)
        fact *= i + 1
        h_phi_k = h_phi_k / hh - 1.0 / fact
    R = torch.tensor(R, dtype=torch.float64)
    b = torch.tensor(b, dtype=torch.float64)
    rhos_p = None
    if d1s:
        if order == 2:
            rhos_p = [0.5]
        else:
            rhos_p = torch.linalg.solve(R[:-1, :-1], b[:-1]).tolist()
    rhos_c = None
    if use_corrector:
        rhos_c = [0.5] if order == 1 else torch.linalg.solve(R, b).tolist()
    x_t_ = (sv_t / sv0) * x - a_t * h_phi_1 * m0
    pred = sum(r * d for r, d in zip(rhos_p, d1s)) if d1s else 0.0
    x_t = x_t_ - a_t * b_h * pred
    model_t = None
    if use_corrector:
        model_t = denoise_fn(x_t, s_t)
        corr = sum(r * d for r, d in zip(rhos_c[:-1], d1s)) if d1s else 0.0
        d1_t = model_t - m0
        x_t = x_t_ - a_t * b_h * (corr + rhos_c[-1] * d1_t)
    return x_t, model_t


@torch.no_grad()
def sample_unipc(model, noise, sigmas, extra_args=None, callback=None, disable=False, variant="bh1"):
    extra_args = {} if extra_args is None else extra_args
    ts = [float(s) for s in sigmas.detach().cpu()]
    if ts[-1] == 0:
        ts[-1] = 0.001
    s_in = noise.new_ones([noise.shape[0]])
    steps = len(ts) - 1
    order = min(3, len(ts) - 2)
    if order < 1:
        order = 1

    def denoise(x_vp, s):
        xk = x_vp / _alpha(s)              # VP -> k-diffusion scaling
        return model(xk, s_in * s, **extra_args)

    x = noise * _alpha(ts[0])
    step_i = 0
    m = denoise(x, ts[0])
    if callback is not None:
        callback({"x": x, "i": 0, "denoised": m})
    model_prev, lam_prev, sig_prev = [m], [_lam(ts[0])], [ts[0] * _alpha(ts[0])]
    for step in range(1, steps + 1):
        if step < order:
            step_order = step
        else:
            step_order = min(order, steps + 1 - step)
        use_corr = step != steps
        x, mt = _unipc_update(x, model_prev, lam_prev, sig_prev, ts[step], step_order, variant, use_corr, denoise)
        step_i = step
        if step < steps:
            if mt is None:
                mt = denoise(x, ts[step])
            model_prev.append(mt)
            lam_prev.append(_lam(ts[step]))
            sig_prev.append(ts[step] * _alpha(ts[step]))
            if len(model_prev) > order:
                model_prev.pop(0)
                lam_prev.pop(0)
                sig_prev.pop(0)
            if callback is not None:
                callback({"x": x, "i": step_i, "denoised": mt})
    return x / _alpha(ts[-1])


def sample_unipc_bh2(model, noise, sigmas, extra_args=None, callback=None, disable=False):
    return sample_unipc(model, noise, sigmas, extra_args, callback, disable, variant="bh2")
