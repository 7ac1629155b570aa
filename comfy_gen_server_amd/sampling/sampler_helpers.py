"""Sampling preparation (parity: ``comfy/sampler_helpers.py:1-120``, C23): mask preparation,
CONDITIONING list -> cond dicts, gathering ControlNet / GLIGEN models from conds and making
everything resident before the loop."""
from __future__ import annotations

import torch

from ..runtime import device as dm
from . import conds as C


def prepare_mask(noise_mask, shape, device):
    m = torch.nn.functional.interpolate(noise_mask.reshape((-1, 1, noise_mask.shape[-2], noise_mask.shape[-1])),
                                        size=(shape[2], shape[3]), mode="bilinear")
    m = torch.cat([m] * shape[1], dim=1)
    m = C.repeat_to_batch_size(m, shape[0])
    return m.to(device)


def get_models_from_cond(cond, model_type):
    return [c[model_type] for c in cond if model_type in c]


def convert_cond(cond):
    out = []
    for c in cond:
        temp = dict(c[1])
        mc = dict(temp.get("model_conds", {}))
        if c[0] is not None:
            mc["c_crossattn"] = C.CONDCrossAttn(c[0])
            temp["cross_attn"] = c[0]
        temp["model_conds"] = mc
        out.append(temp)
    return out


def get_additional_models(conds, dtype):
    cnets, gligen = [], []
    for k in conds:
        cnets += get_models_from_cond(conds[k], "control")
        gligen += get_models_from_cond(conds[k], "gligen")
    mem = 0
    models = []
    for m in set(cnets):
        models += m.get_models()
        mem += m.inference_memory_requirements(dtype)
    models += [g[1] for g in gligen]
    return models, mem


def cleanup_additional_models(models):
    for m in models:
        if hasattr(m, "cleanup"):
            m.cleanup()


def prepare_sampling(model, noise_shape, conds):
    models, mem = get_additional_models(conds, model.model_dtype())
    dm.load_models_gpu([model] + models, model.memory_required([noise_shape[0] * 2] + list(noise_shape[1:])) + mem)
    return model.model, conds, models


def cleanup_models(conds, models):
    cleanup_additional_models(models)
    ctrl = []
    for k in conds:
        ctrl += get_models_from_cond(conds[k], "control")
    cleanup_additional_models(set(ctrl))
