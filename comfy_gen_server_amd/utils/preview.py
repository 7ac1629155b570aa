"""Latent previews (parity: ``latent_preview.py:1-98``; C16): latent2rgb linear map or TAESD decode,
JPEG <= 512 px. Off the critical path: previews are decoded on a side HIP stream so the sampler's
stream never waits for the preview's D2H copy."""
from __future__ import annotations

import threading

import numpy as np
import torch
from PIL import Image

MAX_PREVIEW_RESOLUTION = 512


class LatentPreviewer:
    def decode_latent_to_preview(self, x0):
        raise NotImplementedError

    def decode_latent_to_preview_image(self, preview_format, x0):
        img = self.decode_latent_to_preview(x0)
        return (preview_format, img, MAX_PREVIEW_RESOLUTION)


def _to_pil(t):
    arr = (t.clamp(0, 1) * 255.0).to(torch.uint8).cpu().numpy()
    return Image.fromarray(arr)


class Latent2RGBPreviewer(LatentPreviewer):
    def __init__(self, latent_rgb_factors):
        self.factors = torch.tensor(latent_rgb_factors, dtype=torch.float32)
        self.stream = torch.cuda.Stream() if torch.cuda.is_available() else None

    def decode_latent_to_preview(self, x0):
        src = x0[:1]
        if self.stream is not None and src.is_cuda:
            self.stream.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(self.stream):
                f = self.factors.to(src.device)
                img = torch.einsum("chw,cr->hwr", src[0].float(), f)
                img = ((img + 1.0) / 2.0)
            self.stream.synchronize()
        else:
            f = self.factors.to(src.device)
            img = (torch.einsum("chw,cr->hwr", src[0].float(), f) + 1.0) / 2.0
        return _to_pil(img)


class TAESDPreviewerImpl(LatentPreviewer):
    def __init__(self, taesd):
        self.taesd = taesd

    def decode_latent_to_preview(self, x0):
        s = self.taesd.decode(x0[:1])[0].movedim(0, 2)
        return _to_pil(s)


def get_previewer(device, latent_format, method="none"):
    if method in (None, "none"):
        return None
    if method in ("taesd", "auto") and latent_format.taesd_decoder_name is not None:
        from . import folder_paths
        name = latent_format.taesd_decoder_name
        path = next((f for f in folder_paths.get_filename_list("vae_approx") if f.startswith(name)), None)
        if path is not None:
            from ..models.taesd import TAESD
            from ..runtime.checkpoint import load_state_dict
            t = TAESD(None, folder_paths.get_full_path("vae_approx", path),
                      latent_channels=latent_format.latent_channels).to(device)
            return TAESDPreviewerImpl(t)
    if latent_format.latent_rgb_factors is not None:
        return Latent2RGBPreviewer(latent_format.latent_rgb_factors)
    return None
