"""Sampling entry points (parity: ``comfy/sample.py:1-44``).

Initial noise is generated on the HOST with ``torch.manual_seed(seed)`` and per-batch-index replay
(``prepare_noise``) so a seed gives the same image as the reference regardless of the device.
"""
from __future__ import annotations

import numpy as np
import torch

from ..runtime import device as dm
from . import samplers


def prepare_noise(latent_image, seed, noise_inds=None):
    generator = torch.manual_seed(seed)
    if noise_inds is None:
        return torch.randn(latent_image.size(), dtype=torch.float32, layout=latent_image.layout, generator=generator,
                           device="cpu")
    unique, inverse = np.unique(noise_inds, return_inverse=True)
    noises = []
    for i in range(unique[-1] + 1):
        n = torch.randn([1] + list(latent_image.size())[1:], dtype=torch.float32, layout=latent_image.layout,
                        generator=generator, device="cpu")
        if i in unique:
            noises.append(n)
    return torch.cat([noises[i] for i in inverse], dim=0)


def sample(model, noise, steps, cfg, sampler_name, scheduler, positive, negative, latent_image, denoise=1.0,
           disable_noise=False, start_step=None, last_step=None, force_full_denoise=False, noise_mask=None,
           sigmas=None, callback=None, disable_pbar=False, seed=None, noise_inds=None):
    """``noise_inds``: the global batch index of every latent (default 0..B-1) — keys the per-step
    ancestral/SDE noise so it does not depend on how a batch is split (``sampling/rng.py``)."""
    ks = samplers.KSampler(model, steps=steps, device=model.load_device, sampler=sampler_name, scheduler=scheduler,
                           denoise=denoise, model_options=model.model_options)
    out = ks.sample(noise, positive, negative, cfg=cfg, latent_image=latent_image, start_step=start_step,
                    last_step=last_step, force_full_denoise=force_full_denoise, denoise_mask=noise_mask, sigmas=sigmas,
                    callback=callback, disable_pbar=disable_pbar, seed=seed, noise_inds=noise_inds)
    return out.to(dm.intermediate_device())


def sample_custom(model, noise, cfg, sampler, sigmas, positive, negative, latent_image, noise_mask=None,
                  callback=None, disable_pbar=False, seed=None, noise_inds=None):
    out = samplers.sample(model, noise, positive, negative, cfg, model.load_device, sampler, sigmas,
                          model_options=model.model_options, latent_image=latent_image, denoise_mask=noise_mask,
                          callback=callback, disable_pbar=disable_pbar, seed=seed, noise_inds=noise_inds)
    return out.to(dm.intermediate_device())
