"""Noise augmentation modules (parity: ``comfy/ldm/modules/encoders/noise_aug_modules.py`` and
``diffusionmodules/upscaling.py``; C50): unCLIP CLIP-embedding noise augmentation and the x4
upscaler's low-res image concat with noise augmentation."""
from __future__ import annotations

import torch

from .. import ops
from ..sampling.model_sampling import make_beta_schedule


class AbstractLowScaleModel(torch.nn.Module):
    def __init__(self, noise_schedule_config=None):
        super().__init__()
        if noise_schedule_config is not None:
            self.register_schedule(**noise_schedule_config)

    def register_schedule(self, beta_schedule="linear", timesteps=1000, linear_start=1e-4, linear_end=2e-2,
                          cosine_s=8e-3):
        betas = make_beta_schedule(beta_schedule, timesteps, linear_start, linear_end, cosine_s)
        ac = torch.cumprod(1.0 - betas, 0)
        self.num_timesteps = int(timesteps)
        self.register_buffer("sqrt_alphas_cumprod", ac.sqrt().float())
        self.register_buffer("sqrt_one_minus_alphas_cumprod", (1.0 - ac).sqrt().float())

    def q_sample(self, x_start, t, noise=None, seed=None):
        if noise is None:
            if seed is None:
                noise = torch.randn_like(x_start)
            else:
                noise = torch.randn(x_start.size(), dtype=x_start.dtype, layout=x_start.layout,
                                    generator=torch.manual_seed(seed)).to(x_start.device)
        a = self.sqrt_alphas_cumprod.to(x_start.device)[t].view(-1, *([1] * (x_start.ndim - 1)))
        b = self.sqrt_one_minus_alphas_cumprod.to(x_start.device)[t].view(-1, *([1] * (x_start.ndim - 1)))
        return a * x_start + b * noise

    def forward(self, x):
        return x, None


class ImageConcatWithNoiseAugmentation(AbstractLowScaleModel):
    def __init__(self, noise_schedule_config, max_noise_level=1000, to_cuda=False):
        super().__init__(noise_schedule_config=noise_schedule_config)
        self.max_noise_level = max_noise_level

    def forward(self, x, noise_level=None, seed=None):
        if noise_level is None:
            noise_level = torch.randint(0, self.max_noise_level, (x.shape[0],), device=x.device).long()
        return self.q_sample(x, noise_level, seed=seed), noise_level


class Timestep(torch.nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.dim = dim

    def forward(self, t):
        return ops.timestep_embedding(t, self.dim)


class CLIPEmbeddingNoiseAugmentation(AbstractLowScaleModel):
    def __init__(self, *args, clip_stats_path=None, timestep_dim=256, **kwargs):
        super().__init__(*args, **kwargs)
        self.register_buffer("data_mean", torch.zeros(1, timestep_dim), persistent=False)
        self.register_buffer("data_std", torch.ones(1, timestep_dim), persistent=False)
        self.time_embed = Timestep(timestep_dim)
        self.max_noise_level = getattr(self, "num_timesteps", 1000)

    def scale(self, x):
        return (x - self.data_mean.to(x.device)) * 1.0 / self.data_std.to(x.device)

    def unscale(self, x):
        return x * self.data_std.to(x.device) + self.data_mean.to(x.device)

    def forward(self, x, noise_level=None, seed=None):
        if noise_level is None:
            noise_level = torch.randint(0, self.max_noise_level, (x.shape[0],), device=x.device).long()
        x = self.scale(x)
        z = self.q_sample(x, noise_level, seed=seed)
        z = self.unscale(z)
        return z, self.time_embed(noise_level)
