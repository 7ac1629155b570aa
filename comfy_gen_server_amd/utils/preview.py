"""Latent previews (parity: ``latent_preview.py:1-98``; C16): latent2rgb linear map or TAESD decode,
JPEG <= 512 px. Off the critical path: latent2rgb previews are computed on a side HIP stream into
pinned memory and handed out only once their event has completed, so neither the sampler's stream
nor the host thread that enqueues the next step ever waits for a preview."""
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
    """latent2rgb (4 -> 3 linear map) preview that never blocks the sampler.

    Each call queues the projection of this step's x0 on a side HIP stream (ordered after the
    sampler's stream up to this point), copies the small RGB image into pinned host memory and
    records an event. It then returns the most recent *earlier* preview whose event has already
    completed (``Event.query()``, no wait) -- a preview lags the sampler by about one step instead of
    stalling it. ``block=True`` (the last step) waits for the newest one."""

    def __init__(self, latent_rgb_factors):
        self.factors = torch.tensor(latent_rgb_factors, dtype=torch.float32)
        self.stream = torch.cuda.Stream() if torch.cuda.is_available() else None
        self._pending = []          # [(event, pinned host image)] in submission order

    def _submit(self, src):
        self.stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.stream):
            src.record_stream(self.stream)
            f = self.factors.to(src.device, non_blocking=True)
            img = (torch.einsum("chw,cr->hwr", src[0].float(), f) + 1.0) / 2.0
            host = torch.empty(img.shape, dtype=img.dtype, pin_memory=True)
            host.copy_(img, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        self._pending.append((ev, host))

    def _ready(self, block=False):
        done = None
        while self._pending and (self._pending[0][0].query() or (block and len(self._pending) == 1)):
            ev, host = self._pending.pop(0)
            ev.synchronize()
            done = host
        if block and self._pending:
            ev, host = self._pending.pop()
            ev.synchronize()
            self._pending.clear()
            done = host
        return done

    def decode_latent_to_preview(self, x0, block=False):
        src = x0[:1]
        if self.stream is None or not src.is_cuda:
            f = self.factors.to(src.device)
            return _to_pil((torch.einsum("chw,cr->hwr", src[0].float(), f) + 1.0) / 2.0)
        self._submit(src)
        host = self._ready(block)
        return None if host is None else _to_pil(host)

    def decode_latent_to_preview_image(self, preview_format, x0, block=False):
        img = self.decode_latent_to_preview(x0, block=block)
        return None if img is None else (preview_format, img, MAX_PREVIEW_RESOLUTION)


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
