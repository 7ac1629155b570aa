"""ModelPatcher: copy-on-write view of a shared module with weight patches, object patches and
sampler/transformer hooks (parity: ``comfy/model_patcher.py:1-485``).

* weight patches (diff / lora(+mid) / lokr / loha(+CP) / glora / DoRA) are merged ON THE DEVICE
  in fp32 when the model is made resident (``patch_model``) and the original weights are backed
  up on the device too (288 GB HBM: no host round trip); derived kernel layouts (fused QKV,
  NHWC conv weights, GEGLU interleave) are invalidated after every merge;
* object patches replace attributes (e.g. ``model_sampling``) while resident;
* ``model_options`` carries ``transformer_options.patches`` / ``patches_replace`` and the
  sampler hooks ``sampler_cfg_function``, ``sampler_post_cfg_function``, ``model_function_wrapper``,
  ``denoise_mask_function``.
"""
from __future__ import annotations

import copy
import logging
import os
import uuid

import torch

from . import device as dm


def set_model_options_patch_replace(model_options, patch, name, block_name, number, transformer_index=None):
    to = model_options["transformer_options"] = dict(model_options.get("transformer_options", {}))
    pr = to["patches_replace"] = {k: dict(v) for k, v in to.get("patches_replace", {}).items()}
    pr.setdefault(name, {})
    key = (block_name, number) if transformer_index is None else (block_name, number, transformer_index)
    pr[name][key] = patch
    return model_options


def set_model_options_post_cfg_function(model_options, post_cfg_function, disable_cfg1_optimization=False):
    model_options["sampler_post_cfg_function"] = model_options.get("sampler_post_cfg_function", []) + [post_cfg_function]
    if disable_cfg1_optimization:
        model_options["disable_cfg1_optimization"] = True
    return model_options


def weight_decompose(dora_scale, weight, lora_diff, alpha, strength):
    """DoRA as the reference applies it (``comfy/model_patcher.py:10-19``, ``:353-355``): add the
    strength-scaled low-rank delta, then rescale every input-column slice of the merged weight to the
    learned magnitude ``dora_scale``."""
    wc = weight + (strength * alpha) * lora_diff.to(weight.dtype)
    norm = wc.transpose(0, 1).reshape(wc.shape[1], -1).norm(dim=1, keepdim=True)
    norm = norm.reshape(wc.shape[1], *[1] * (wc.dim() - 1)).transpose(0, 1)
    return wc * (dora_scale.to(weight.device, weight.dtype) / norm)


def _f(t, like):
    return None if t is None else t.to(device=like.device, dtype=torch.float32)


def calculate_weight(patches, weight, key, base_dtype=None):
    """Apply a list of (strength_patch, value, strength_model) to an fp32 ``weight``."""
    for strength, v, strength_model in patches:
        if strength_model != 1.0:
            weight = weight * strength_model
        if isinstance(v, list):
            v = (calculate_weight(v[1:], v[0].clone(), key, base_dtype),)
        if len(v) == 1:
            kind, v = "diff", v
        else:
            kind, v = v
        if kind == "diff":
            w1 = v[0]
            if strength != 0.0:
                if w1.shape != weight.shape:
                    logging.warning("WARNING SHAPE MISMATCH %s WEIGHT NOT MERGED %s != %s", key, w1.shape, weight.shape)
                else:
                    weight = weight + strength * _f(w1, weight)
        elif kind == "lora":
            up, down, alpha, mid, dora = v
            up, down = _f(up, weight), _f(down, weight)
            alpha = (alpha / down.shape[0]) if alpha is not None else 1.0
            if mid is not None:
                mid = _f(mid, weight)
                shp = [down.shape[1], down.shape[0], mid.shape[2], mid.shape[3]]
                down = torch.mm(down.transpose(0, 1).flatten(1), mid.transpose(0, 1).flatten(1)).reshape(shp).transpose(0, 1)
            try:
                diff = _lora_product(up.flatten(1), down.flatten(1),
                                     bf16_ok=base_dtype == torch.bfloat16).reshape(weight.shape)
            except RuntimeError as e:
                logging.error("ERROR %s %s %s", kind, key, e)
                continue
            weight = weight_decompose(dora, weight, diff, alpha, strength) if dora is not None \
                else weight + (strength * alpha) * diff
        elif kind == "lokr":
            w1, w2, alpha, w1a, w1b, w2a, w2b, t2, dora = v
            dim = None
            if w1 is None:
                dim = w1b.shape[0]
                w1 = torch.mm(_f(w1a, weight), _f(w1b, weight))
            else:
                w1 = _f(w1, weight)
            if w2 is None:
                dim = w2b.shape[0]
                if t2 is None:
                    w2 = torch.mm(_f(w2a, weight), _f(w2b, weight))
                else:
                    w2 = torch.einsum("i j k l, j r, i p -> p r k l", _f(t2, weight), _f(w2b, weight), _f(w2a, weight))
            else:
                w2 = _f(w2, weight)
            if w2.dim() == 4:      # conv LoKr: w1 [a, b] -> [a, b, 1, 1] so kron spans the taps of w2
                w1 = w1.unsqueeze(2).unsqueeze(2)
            alpha = (alpha / dim) if (alpha is not None and dim is not None) else 1.0
            diff = torch.kron(w1, w2).reshape(weight.shape)
            weight = weight_decompose(dora, weight, diff, alpha, strength) if dora is not None \
                else weight + (strength * alpha) * diff
        elif kind == "loha":
            w1a, w1b, alpha, w2a, w2b, t1, t2, dora = v
            alpha = (alpha / w1b.shape[0]) if alpha is not None else 1.0
            if t1 is not None:
                m1 = torch.einsum("i j k l, j r, i p -> p r k l", _f(t1, weight), _f(w1b, weight), _f(w1a, weight))
                m2 = torch.einsum("i j k l, j r, i p -> p r k l", _f(t2, weight), _f(w2b, weight), _f(w2a, weight))
            else:
                m1 = torch.mm(_f(w1a, weight), _f(w1b, weight))
                m2 = torch.mm(_f(w2a, weight), _f(w2b, weight))
            diff = (m1 * m2).reshape(weight.shape)
            weight = weight_decompose(dora, weight, diff, alpha, strength) if dora is not None \
                else weight + (strength * alpha) * diff
        elif kind == "glora":
            a1, a2, b1, b2, alpha, dora = v
            alpha = (alpha / a1.shape[0]) if alpha is not None else 1.0
            a1, a2, b1, b2 = (_f(t, weight).flatten(1) for t in (a1, a2, b1, b2))
            diff = (torch.mm(b2, b1) + torch.mm(torch.mm(weight.flatten(1), a2), a1)).reshape(weight.shape)
            weight = weight_decompose(dora, weight, diff, alpha, strength) if dora is not None \
                else weight + (strength * alpha) * diff
        else:
            logging.warning("patch type not recognized %s %s", kind, key)
    return weight


def _lora_product(up: torch.Tensor, down: torch.Tensor, bf16_ok: bool = False) -> torch.Tensor:
    """up [O, r] @ down [r, I] (K20). For a bf16 base weight on the GPU: the HIP MFMA GEMM (bf16
    factors, fp32 accumulate, one bf16 rounding of the rank-r product -- below the bf16 rounding of the
    merged weight itself). fp16 / fp32 base weights, CPU tensors and ranks the GEMM does not tile
    (r % 8): fp32 ``torch.mm`` like the reference (``comfy/model_patcher.py:370``)."""
    if bf16_ok and up.is_cuda and up.shape[1] % 8 == 0 and up.shape[1] == down.shape[0] \
            and os.environ.get("CGS_LORA_HIP", "1") != "0":
        from .. import ops
        return ops.linear(up.to(torch.bfloat16), down.t().contiguous().to(torch.bfloat16)).float()
    return torch.mm(up, down)


def _get_attr(obj, name):
    for a in name.split("."):
        obj = getattr(obj, a)
    return obj


def _set_attr(obj, name, value):
    parts = name.split(".")
    for a in parts[:-1]:
        obj = getattr(obj, a)
    prev = getattr(obj, parts[-1])
    setattr(obj, parts[-1], value)
    return prev


def _in_arena(t) -> bool:
    from . import arena
    return any(a.owns(t) for a in arena._ARENAS.values()) if arena._ARENAS else False


class ModelPatcher:
    def __init__(self, model, load_device, offload_device, size=0, weight_inplace_update=False):
        self.size = size
        self.model = model
        self.patches = {}
        self.backup = {}
        self.object_patches = {}
        self.object_patches_backup = {}
        self.model_options = {"transformer_options": {}}
        self.load_device = load_device
        self.offload_device = offload_device
        self.weight_inplace_update = weight_inplace_update
        self.patches_uuid = uuid.uuid4()
        if not hasattr(self.model, "current_patches_uuid"):
            self.model.current_patches_uuid = None

    @property
    def patches_uuid_applied(self):
        return getattr(self.model, "current_patches_uuid", None)

    def model_size(self):
        if self.size > 0:
            return self.size
        self.size = dm.module_size(self.model)
        return self.size

    def is_resident_on(self, device):
        try:
            p = next(self.model.parameters())
        except StopIteration:
            return True
        return p.device == torch.device(device) or (p.device.type == device.type == "cpu")

    def clone(self):
        n = ModelPatcher(self.model, self.load_device, self.offload_device, self.size, self.weight_inplace_update)
        n.patches = {k: list(v) for k, v in self.patches.items()}
        n.patches_uuid = self.patches_uuid
        n.object_patches = dict(self.object_patches)
        n.model_options = copy.deepcopy(self.model_options)
        n.backup = self.backup
        n.object_patches_backup = self.object_patches_backup
        return n

    def is_clone(self, other):
        return hasattr(other, "model") and self.model is other.model

    def clone_has_same_weights(self, clone):
        return self.is_clone(clone) and self.patches_uuid == clone.patches_uuid

    def memory_required(self, input_shape):
        return self.model.memory_required(input_shape=input_shape)

    # ---------------------------------------------------------------- sampler hooks
    def set_model_sampler_cfg_function(self, fn, disable_cfg1_optimization=False):
        if len(__import__("inspect").signature(fn).parameters) == 3:
            self.model_options["sampler_cfg_function"] = lambda args: fn(args["cond"], args["uncond"], args["cond_scale"])
        else:
            self.model_options["sampler_cfg_function"] = fn
        if disable_cfg1_optimization:
            self.model_options["disable_cfg1_optimization"] = True

    def set_model_sampler_post_cfg_function(self, fn, disable_cfg1_optimization=False):
        self.model_options = set_model_options_post_cfg_function(self.model_options, fn, disable_cfg1_optimization)

    def set_model_unet_function_wrapper(self, fn):
        self.model_options["model_function_wrapper"] = fn

    def set_model_denoise_mask_function(self, fn):
        self.model_options["denoise_mask_function"] = fn

    def set_model_patch(self, patch, name):
        to = self.model_options["transformer_options"]
        to.setdefault("patches", {})
        to["patches"][name] = to["patches"].get(name, []) + [patch]

    def set_model_patch_replace(self, patch, name, block_name, number, transformer_index=None):
        self.model_options = set_model_options_patch_replace(self.model_options, patch, name, block_name, number,
                                                             transformer_index)

    def set_model_attn1_patch(self, p):
        self.set_model_patch(p, "attn1_patch")

    def set_model_attn2_patch(self, p):
        self.set_model_patch(p, "attn2_patch")

    def set_model_attn1_replace(self, p, block_name, number, transformer_index=None):
        self.set_model_patch_replace(p, "attn1", block_name, number, transformer_index)

    def set_model_attn2_replace(self, p, block_name, number, transformer_index=None):
        self.set_model_patch_replace(p, "attn2", block_name, number, transformer_index)

    def set_model_attn1_output_patch(self, p):
        self.set_model_patch(p, "attn1_output_patch")

    def set_model_attn2_output_patch(self, p):
        self.set_model_patch(p, "attn2_output_patch")

    def set_model_input_block_patch(self, p):
        self.set_model_patch(p, "input_block_patch")

    def set_model_input_block_patch_after_skip(self, p):
        self.set_model_patch(p, "input_block_patch_after_skip")

    def set_model_output_block_patch(self, p):
        self.set_model_patch(p, "output_block_patch")

    def add_object_patch(self, name, obj):
        self.object_patches[name] = obj

    def get_model_object(self, name):
        if name in self.object_patches:
            return self.object_patches[name]
        if name in self.object_patches_backup:
            return self.object_patches_backup[name]
        return _get_attr(self.model, name)

    def model_patches_to(self, device):
        to = self.model_options["transformer_options"]
        for group in ("patches", "patches_replace"):
            for name, items in to.get(group, {}).items():
                seq = items.values() if isinstance(items, dict) else items
                for p in seq:
                    if hasattr(p, "to"):
                        p.to(device)
        if "model_function_wrapper" in self.model_options:
            w = self.model_options["model_function_wrapper"]
            if hasattr(w, "to"):
                w.to(device)

    def model_dtype(self):
        if hasattr(self.model, "get_dtype"):
            return self.model.get_dtype()
        return next(self.model.parameters()).dtype

    # ---------------------------------------------------------------- weight patches
    def add_patches(self, patches, strength_patch=1.0, strength_model=1.0):
        p = set()
        sd = self.model_state_dict_keys()
        for k, v in patches.items():
            if k in sd:
                p.add(k)
                self.patches.setdefault(k, []).append((strength_patch, v, strength_model))
        self.patches_uuid = uuid.uuid4()
        return list(p)

    def model_state_dict_keys(self):
        return set(self.model.state_dict().keys())

    def get_key_patches(self, filter_prefix=None):
        sd = self.model_state_dict()
        out = {}
        for k, w in sd.items():
            if filter_prefix is not None and not k.startswith(filter_prefix):
                continue
            out[k] = [w] + self.patches.get(k, []) if k in self.patches else (w,)
        return out

    def model_state_dict(self, filter_prefix=None):
        sd = self.model.state_dict()
        if filter_prefix is not None:
            sd = {k: v for k, v in sd.items() if k.startswith(filter_prefix)}
        return sd

    def patch_weight_to_device(self, key, device_to=None):
        if key not in self.patches:
            return
        w = _get_attr(self.model, key)
        if key not in self.backup:
            self.backup[key] = w.data.clone() if device_to is None else w.data.to(device_to, copy=True)
        base = self.backup[key]
        dev = device_to if device_to is not None else base.device
        out = calculate_weight(self.patches[key], base.to(dev, torch.float32, copy=True), key, base.dtype)
        if _in_arena(w) and out.shape == w.shape:
            w.data.copy_(out.to(base.dtype))         # patched weight stays in its arena block
        else:
            w.data = out.to(base.dtype)

    def patch_model(self, device_to=None, patch_weights=True, force=False):
        for k, obj in self.object_patches.items():
            old = _set_attr(self.model, k, obj)
            if k not in self.object_patches_backup:
                self.object_patches_backup[k] = old
        if device_to is not None and not self.is_resident_on(device_to):
            from . import arena
            wa = arena.get(device_to)
            if wa is not None:
                try:
                    wa.place_module(self.model)      # weights into the HBM slab (C27)
                except arena.ArenaFull as e:         # does not fit: plain caching-allocator residency
                    logging.warning("weight arena: %s; loading %s with the caching allocator",
                                    e, type(self.model).__name__)
                self.model.to(device_to)             # (anything the arena does not hold)
            else:
                self.model.to(device_to)
            from ..models.layers import stamp_epoch
            stamp_epoch(self.model)
        if patch_weights and (force or getattr(self.model, "current_patches_uuid", None) != self.patches_uuid):
            # restore weights that have a backup but are no longer patched
            for k in list(self.backup.keys()):
                if k not in self.patches:
                    _get_attr(self.model, k).data = self.backup.pop(k).to(device_to or self.load_device)
            for k in self.patches:
                self.patch_weight_to_device(k, device_to)
            self.model.current_patches_uuid = self.patches_uuid
            from ..models.layers import invalidate_all
            invalidate_all(self.model)
        return self.model

    def unpatch_model(self, device_to=None, unpatch_weights=True):
        if unpatch_weights:
            for k, w in self.backup.items():
                t = _get_attr(self.model, k)
                if _in_arena(t) and t.shape == w.shape:
                    t.data.copy_(w)
                else:
                    t.data = w
            self.backup.clear()
            self.model.current_patches_uuid = None
            from ..models.layers import invalidate_all
            invalidate_all(self.model)
            if device_to is not None:
                from . import arena
                for a in list(arena._ARENAS.values()):
                    if id(self.model) in a.blocks:
                        a.evict_module(self.model, device_to)
                self.model.to(device_to)
        for k, v in self.object_patches_backup.items():
            _set_attr(self.model, k, v)
        self.object_patches_backup.clear()
