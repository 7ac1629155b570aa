"""Node helpers: conditioning copy-with-values (``node_helpers.py:2-10``; C18), the sampler progress /
latent-preview callback (``latent_preview.py:81-97``; C16), and server flags visible to nodes."""
from __future__ import annotations

import torch

from ..utils.progress import ProgressBar

_FLAGS = {"disable_metadata": False, "preview_method": "none", "preview_every": 1}


def set_flags(**kw):
    _FLAGS.update(kw)


def args_disable_metadata():
    return _FLAGS["disable_metadata"]


def conditioning_set_values(conditioning, values=None):
    values = values or {}
    c = []
    for t in conditioning:
        n = [t[0], t[1].copy()]
        for k, v in values.items():
            n[1][k] = v
        c.append(n)
    return c


def prepare_callback(model, steps, x0_output_dict=None):
    """Per-step progress (+ optional async latent preview, every ``preview_every`` steps)."""
    from ..utils.preview import get_previewer
    previewer = get_previewer(model.load_device, model.model.latent_format, _FLAGS["preview_method"])
    pbar = ProgressBar(steps)
    every = max(1, int(_FLAGS["preview_every"]))

    def callback(step, x0, x, total_steps):
        if x0_output_dict is not None:
            x0_output_dict["x0"] = x0
        preview = None
        if previewer is not None and (step % every == 0 or step + 1 == total_steps):
            preview = previewer.decode_latent_to_preview_image("JPEG", x0, block=step + 1 == total_steps)
        pbar.update_absolute(step + 1, total_steps, preview)
    return callback
