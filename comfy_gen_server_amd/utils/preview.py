"""Latent previews (parity: ``latent_preview.py:1-98``; C16): latent2rgb linear map or TAESD decode,
JPEG <= 512 px, every ``--preview-every`` steps. Off the critical path: both previewers compute on a side
HIP stream into pinned memory and hand an image out only once its event has completed, so neither the
sampler's stream nor the host thread that enqueues the next step ever waits for a preview."""
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


class _AsyncPreviewer(LatentPreviewer):
    """A preview that never blocks the sampler.

    Each call queues ``_image(src)`` (-> [H, W, 3] in [0, 1] on the device) for this step's x0 on a side
    HIP stream (ordered after the sampler's stream up to this point), copies the small RGB image into
    pinned host memory and records an event. It then returns the most recent *earlier* preview whose event
    has already completed (``Event.query()``, no wait) -- a preview lags the sampler by about one step
    instead of stalling it. ``block=True`` (the last step) waits for the newest one. At most ``depth``
    previews are in flight: a step that finds the queue full skips its preview rather than waiting."""

    depth = 3

    def __init__(self):
        self.stream = torch.cuda.Stream() if torch.cuda.is_available() else None
        self._pending = []          # [(event, pinned host image)] in submission order
        self.submitted = self.skipped = 0

    def _image(self, src):
        raise NotImplementedError

    def _submit(self, src):
        self.stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.stream):
            src.record_stream(self.stream)
            img = self._image(src).float()
            host = torch.empty(img.shape, dtype=img.dtype, pin_memory=True)
            host.copy_(img, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        self._pending.append((ev, host))
        self.submitted += 1

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
            return _to_pil(self._image(src))
        if len(self._pending) < self.depth or block:
            self._submit(src)
        else:
            self.skipped += 1
        host = self._ready(block)
        return None if host is None else _to_pil(host)

    def decode_latent_to_preview_image(self, preview_format, x0, block=False):
        img = self.decode_latent_to_preview(x0, block=block)
        return None if img is None else (preview_format, img, MAX_PREVIEW_RESOLUTION)


class Latent2RGBPreviewer(_AsyncPreviewer):
    """latent2rgb (4 -> 3 linear map, reference ``latent_preview.py:31-45``) on the side stream."""

    def __init__(self, latent_rgb_factors):
        super().__init__()
        self.factors = torch.tensor(latent_rgb_factors, dtype=torch.float32)

    def _image(self, src):
        f = self.factors.to(src.device, non_blocking=True)
        return (torch.einsum("chw,cr->hwr", src[0].float(), f) + 1.0) / 2.0


class TAESDPreviewerImpl(_AsyncPreviewer):
    """TAESD decode (reference ``latent_preview.py:21-28``) on the side stream: the tiny decoder's convs
    queue there behind the step that produced x0 and overlap the next steps of the sampler."""

    def __init__(self, taesd):
        super().__init__()
        self.taesd = taesd

    def _image(self, src):
        return self.taesd.decode(src)[0].movedim(0, 2)


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
