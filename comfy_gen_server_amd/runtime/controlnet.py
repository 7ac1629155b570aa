"""ControlNet / Control-LoRA / T2I-Adapter runtime (parity: ``comfy/controlnet.py:1-554``).

A control object lives inside a conditioning entry (``cond[1]["control"]``); the sampler calls
``pre_run`` once (sigma window from the percent range), ``get_models`` for residency, and
``get_control(x, sigma, cond, batched_number)`` per UNet batch, which returns residual lists
``{"input": [...], "middle": [...], "output": [...]}`` consumed by the UNet's injection points.
Chained nets (``previous_controlnet``) are summed; strength scales the residuals; a sigma outside
the window returns only the previous chain's output.

MI355X notes: the hint image is resized/cast once per shape and kept resident on the device;
control models load next to the UNet (the HBM budget fits UNet + several ControlNets, so no
swapping between steps); Control-LoRA folds ``up @ down`` into the base weights once at
``pre_run`` instead of per forward.
"""
from __future__ import annotations

import logging
import math
import os

import torch

from ..models.cldm import ControlNet as ControlNetModel
from ..models.t2i_adapter import Adapter, Adapter_light
from ..utils import image as U
from . import device as dm
from .checkpoint import load_state_dict
from .convert import state_dict_prefix_replace, unet_to_diffusers
from .patcher import ModelPatcher


def broadcast_image_to(tensor, target_batch_size, batched_number):
    """Repeat a hint batch to the UNet batch (cond/uncond chunks each get the per-chunk hint batch)."""
    cur = tensor.shape[0]
    if cur == 1:
        return tensor
    per = target_batch_size // batched_number
    tensor = tensor[:per]
    if per > tensor.shape[0]:
        tensor = torch.cat([tensor] * (per // tensor.shape[0]) + [tensor[:per % tensor.shape[0]]], dim=0)
    if tensor.shape[0] == target_batch_size:
        return tensor
    return torch.cat([tensor] * batched_number, dim=0)


class ControlBase:
    def __init__(self, device=None):
        self.cond_hint_original = None
        self.cond_hint = None
        self.strength = 1.0
        self.timestep_percent_range = (0.0, 1.0)
        self.global_average_pooling = False
        self.timestep_range = None
        self.compression_ratio = 8
        self.upscale_algorithm = "nearest-exact"
        self.device = device if device is not None else dm.get_torch_device()
        self.previous_controlnet = None

    def set_cond_hint(self, cond_hint, strength=1.0, timestep_percent_range=(0.0, 1.0)):
        self.cond_hint_original = cond_hint
        self.strength = strength
        self.timestep_percent_range = timestep_percent_range
        return self

    def pre_run(self, model, percent_to_timestep_function):
        self.timestep_range = (percent_to_timestep_function(self.timestep_percent_range[0]),
                               percent_to_timestep_function(self.timestep_percent_range[1]))
        if self.previous_controlnet is not None:
            self.previous_controlnet.pre_run(model, percent_to_timestep_function)

    def set_previous_controlnet(self, controlnet):
        self.previous_controlnet = controlnet
        return self

    def cleanup(self):
        if self.previous_controlnet is not None:
            self.previous_controlnet.cleanup()
        self.cond_hint = None
        self.timestep_range = None

    def get_models(self):
        return self.previous_controlnet.get_models() if self.previous_controlnet is not None else []

    def copy_to(self, c):
        c.cond_hint_original = self.cond_hint_original
        c.strength = self.strength
        c.timestep_percent_range = self.timestep_percent_range
        c.global_average_pooling = self.global_average_pooling
        c.compression_ratio = self.compression_ratio
        c.upscale_algorithm = self.upscale_algorithm

    def inference_memory_requirements(self, dtype):
        if self.previous_controlnet is not None:
            return self.previous_controlnet.inference_memory_requirements(dtype)
        return 0

    def _outside_window(self, t):
        if self.timestep_range is None:
            return False
        from ..sampling.samplers import current_sigma
        s = current_sigma.get()           # host copy published by the sampler: no D2H sync per step
        s = float(t[0]) if s is None else s
        return self.outside_window_at(s)

    def outside_window_at(self, sigma: float) -> bool:
        if self.timestep_range is None:
            return False
        return sigma > self.timestep_range[0] or sigma < self.timestep_range[1]

    def prepare_hint(self, x_noisy, batched_number):
        """The per-job hint tensor get_control() would build (resized, cast, batch-broadcast),
        built eagerly so a captured step graph can take it as a static input."""
        dtype = getattr(self, "manual_cast_dtype", None) or self.control_model.dtype
        self._hint_for(x_noisy, dtype)
        if x_noisy.shape[0] != self.cond_hint.shape[0]:
            self.cond_hint = broadcast_image_to(self.cond_hint, x_noisy.shape[0], batched_number)
        return self.cond_hint

    def control_merge(self, control_input, control_output, control_prev, output_dtype):
        out = {"input": [], "middle": [], "output": []}
        for x in control_input or []:
            if x is not None:
                x = (x * self.strength).to(output_dtype)
            out["input"].insert(0, x)
        if control_output is not None:
            n = len(control_output)
            for i, x in enumerate(control_output):
                key = "middle" if i == n - 1 else "output"
                if x is not None:
                    if self.global_average_pooling:
                        x = torch.mean(x, dim=(2, 3), keepdim=True).repeat(1, 1, x.shape[2], x.shape[3])
                    x = (x * self.strength).to(output_dtype)
                out[key].append(x)
        if control_prev is not None:
            for key in ("input", "middle", "output"):
                o = out[key]
                for i, pv in enumerate(control_prev[key]):
                    if i >= len(o):
                        o.append(pv)
                    elif pv is not None:
                        if o[i] is None:
                            o[i] = pv
                        elif o[i].shape[0] < pv.shape[0]:
                            o[i] = pv + o[i]
                        else:
                            o[i] = o[i] + pv
        return out

    def _hint_for(self, x_noisy, dtype, width=None, height=None):
        W = width if width is not None else x_noisy.shape[3] * self.compression_ratio
        H = height if height is not None else x_noisy.shape[2] * self.compression_ratio
        if self.cond_hint is None or self.cond_hint.shape[2] != H or self.cond_hint.shape[3] != W:
            self.cond_hint = U.common_upscale(self.cond_hint_original, W, H, self.upscale_algorithm,
                                              "center").to(dtype).to(self.device)
            return True
        return False


class ControlNet(ControlBase):
    def __init__(self, control_model=None, global_average_pooling=False, device=None, load_device=None,
                 manual_cast_dtype=None):
        super().__init__(device)
        self.control_model = control_model
        self.load_device = load_device
        if control_model is not None:
            self.control_model_wrapped = ModelPatcher(control_model, load_device=load_device,
                                                      offload_device=dm.unet_offload_device())
        self.global_average_pooling = global_average_pooling
        self.model_sampling_current = None
        self.manual_cast_dtype = manual_cast_dtype

    def get_control(self, x_noisy, t, cond, batched_number):
        prev = None
        if self.previous_controlnet is not None:
            prev = self.previous_controlnet.get_control(x_noisy, t, cond, batched_number)
        if self._outside_window(t):
            return prev
        dtype = self.manual_cast_dtype or self.control_model.dtype
        self._hint_for(x_noisy, dtype)
        if x_noisy.shape[0] != self.cond_hint.shape[0]:
            self.cond_hint = broadcast_image_to(self.cond_hint, x_noisy.shape[0], batched_number)
        context = cond.get("crossattn_controlnet", cond["c_crossattn"])
        y = cond.get("y")
        if y is not None:
            y = y.to(dtype)
        ms = self.model_sampling_current
        timestep = ms.timestep(t)
        x_in = ms.calculate_input(t, x_noisy)
        fused = self._fusable(x_noisy, prev)
        if fused is not None:
            # K15: strength and the chained net's residuals are applied inside the zero convs'
            # epilogues; residuals stay in the control model's dtype (the UNet's), no fp32 round trip
            control = self.control_model(x=x_in.to(dtype), hint=self.cond_hint, timesteps=timestep.float(),
                                         context=context.to(dtype), y=y, zero_scale=self.strength,
                                         zero_residuals=fused)
            return {"input": [] if prev is None else list(prev["input"]), "middle": control[-1:],
                    "output": control[:-1]}
        control = self.control_model(x=x_in.to(dtype), hint=self.cond_hint, timesteps=timestep.float(),
                                     context=context.to(dtype), y=y)
        return self.control_merge(None, control, prev, x_noisy.dtype)

    def _fusable(self, x_noisy, prev):
        """Residual list for the fused merge (None entries where there is no previous residual), or
        None when the merge must run unfused: CPU, global-average pooling, CGS_CN_FUSE=0, or a chained
        net whose residual lists / batch sizes do not line up one-to-one with this net's outputs."""
        import os
        from ..models.cldm import ControlNet as _CN
        if not x_noisy.is_cuda or self.global_average_pooling or os.environ.get("CGS_CN_FUSE", "1") == "0" \
                or not isinstance(self.control_model, _CN):
            return None
        n_out = len(self.control_model.zero_convs)
        if prev is None:
            return [None] * (n_out + 1)
        po, pm = list(prev.get("output", [])), list(prev.get("middle", []))
        if len(po) != n_out or len(pm) != 1:
            return None
        res = po + pm
        if any(r is not None and r.shape[0] != x_noisy.shape[0] for r in res):
            return None
        return res

    def copy(self):
        c = ControlNet(None, global_average_pooling=self.global_average_pooling, load_device=self.load_device,
                       manual_cast_dtype=self.manual_cast_dtype)
        c.control_model = self.control_model
        c.control_model_wrapped = self.control_model_wrapped
        self.copy_to(c)
        return c

    def get_models(self):
        return super().get_models() + [self.control_model_wrapped]

    def pre_run(self, model, percent_to_timestep_function):
        super().pre_run(model, percent_to_timestep_function)
        self.model_sampling_current = model.model_sampling

    def cleanup(self):
        self.model_sampling_current = None
        super().cleanup()


class ControlLoraOps:
    """Layer namespace whose Linear / Conv2d hold a low-rank ``up`` / ``down`` pair next to the weight
    and apply ``weight + up @ down`` per call (``comfy/controlnet.py:207``; custom nodes build
    Control-LoRA-style modules with it). ``ControlLora`` below merges the deltas once at load
    instead, so the per-step forward runs the plain fused kernels."""

    class Linear(torch.nn.Module):
        def __init__(self, in_features, out_features, bias=True, device=None, dtype=None):
            super().__init__()
            self.in_features, self.out_features = in_features, out_features
            self.weight = self.bias = self.up = self.down = None

        def forward(self, input):
            w = self.weight.to(input.device, input.dtype)
            if self.up is not None:
                w = w + torch.mm(self.up.flatten(1).float(), self.down.flatten(1).float()).reshape(w.shape).to(w.dtype)
            b = None if self.bias is None else self.bias.to(input.device, input.dtype)
            from .. import ops
            return ops.linear(input, w, b)

    class Conv2d(torch.nn.Module):
        def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                     bias=True, padding_mode="zeros", device=None, dtype=None):
            super().__init__()
            self.in_channels, self.out_channels, self.kernel_size = in_channels, out_channels, kernel_size
            self.stride, self.padding, self.dilation, self.groups = stride, padding, dilation, groups
            self.transposed, self.output_padding, self.padding_mode = False, 0, padding_mode
            self.weight = self.bias = self.up = self.down = None

        def forward(self, input):
            w = self.weight.to(input.device, input.dtype)
            if self.up is not None:
                w = w + torch.mm(self.up.flatten(1).float(), self.down.flatten(1).float()).reshape(w.shape).to(w.dtype)
            b = None if self.bias is None else self.bias.to(input.device, input.dtype)
            return torch.nn.functional.conv2d(input, w, b, self.stride, self.padding, self.dilation, self.groups)


class ControlLora(ControlNet):
    """Control-LoRA: a ControlNet whose encoder weights are the base UNet's plus low-rank deltas
    (``*.up`` / ``*.down``), with full hint block / zero convs / norms in the file."""

    def __init__(self, control_weights, global_average_pooling=False, device=None):
        ControlBase.__init__(self, device)
        self.control_weights = control_weights
        self.global_average_pooling = global_average_pooling
        self.control_model = None
        self.manual_cast_dtype = None

    def pre_run(self, model, percent_to_timestep_function):
        ControlBase.pre_run(self, model, percent_to_timestep_function)
        self.model_sampling_current = model.model_sampling
        cfg = dict(model.model_config.unet_config)
        cfg.pop("out_channels", None)
        cfg["hint_channels"] = self.control_weights["input_hint_block.0.weight"].shape[1]
        dtype = model.get_dtype()
        dev = dm.get_torch_device()
        with torch.device("meta"):
            cm = ControlNetModel(dtype=dtype, device=torch.device("meta"), **cfg)
        cm.to_empty(device=dev)
        own = cm.state_dict()
        base = model.diffusion_model.state_dict()
        new_sd = {k: v for k, v in base.items() if k in own}
        lowrank = {}
        for k, v in self.control_weights.items():
            if k == "lora_controlnet":
                continue
            if k.endswith(".up") or k.endswith(".down"):
                lowrank.setdefault(k.rsplit(".", 1)[0], {})[k.rsplit(".", 1)[1]] = v
            else:
                new_sd[k] = v
        for name, ud in lowrank.items():
            wk = name + ".weight"
            if wk in new_sd and "up" in ud and "down" in ud:
                w = new_sd[wk].to(dev, torch.float32)
                delta = torch.mm(ud["up"].flatten(1).to(dev, torch.float32), ud["down"].flatten(1).to(dev, torch.float32))
                new_sd[wk] = (w + delta.reshape(w.shape)).to(dtype)
        missing, _ = cm.load_state_dict({k: v.to(dev, dtype) for k, v in new_sd.items()}, strict=False)
        if missing:
            logging.debug("control-lora missing keys: %s", missing)
        self.control_model = cm.eval()

    def copy(self):
        c = ControlLora(self.control_weights, global_average_pooling=self.global_average_pooling)
        self.copy_to(c)
        return c

    def cleanup(self):
        self.control_model = None
        super().cleanup()

    def get_models(self):
        return ControlBase.get_models(self)

    def inference_memory_requirements(self, dtype):
        n = sum(v.numel() for v in self.control_weights.values() if hasattr(v, "numel"))
        return n * dm.dtype_size(dtype) + ControlBase.inference_memory_requirements(self, dtype)


def _diffusers_controlnet_to_ldm(data):
    from .detection import unet_config_from_diffusers_unet
    cfg = unet_config_from_diffusers_unet(data)
    keys = unet_to_diffusers(cfg)
    keys["controlnet_mid_block.weight"] = "middle_block_out.0.weight"
    keys["controlnet_mid_block.bias"] = "middle_block_out.0.bias"
    i = 0
    while f"controlnet_down_blocks.{i}.weight" in data:
        for s in ("weight", "bias"):
            keys[f"controlnet_down_blocks.{i}.{s}"] = f"zero_convs.{i}.0.{s}"
        i += 1
    # hint encoder: conv_in, blocks.0..5, conv_out -> input_hint_block.0,2,...,14
    idx = 0
    names = ["controlnet_cond_embedding.conv_in"]
    j = 0
    while f"controlnet_cond_embedding.blocks.{j}.weight" in data:
        names.append(f"controlnet_cond_embedding.blocks.{j}")
        j += 1
    names.append("controlnet_cond_embedding.conv_out")
    for idx, n in enumerate(names):
        for s in ("weight", "bias"):
            keys[f"{n}.{s}"] = f"input_hint_block.{idx * 2}.{s}"
    new_sd = {keys[k]: data.pop(k) for k in list(keys) if k in data}
    if data:
        logging.warning("controlnet leftover keys: %s", list(data)[:20])
    return cfg, new_sd


def load_controlnet(ckpt_path, model=None):
    data = load_state_dict(ckpt_path)
    if "lora_controlnet" in data:
        return ControlLora(data)
    cfg = None
    if "controlnet_cond_embedding.conv_in.weight" in data:       # diffusers format
        cfg, data = _diffusers_controlnet_to_ldm(data)
    pth = "control_model.zero_convs.0.0.weight" in data
    if pth:
        prefix = "control_model."
    elif "zero_convs.0.0.weight" in data:
        prefix = ""
    else:
        net = load_t2i_adapter(data)
        if net is None:
            logging.error("checkpoint holds neither a controlnet nor a t2i adapter: %s", ckpt_path)
        return net
    supported = None
    if cfg is None:
        from .detection import model_config_from_unet
        mc = model_config_from_unet(data, prefix, True)
        supported = mc.supported_inference_dtypes
        cfg = dict(mc.unet_config)
    load_device = dm.get_torch_device()
    dtype = dm.unet_dtype(supported_dtypes=supported) if supported else dm.unet_dtype()
    manual_cast = dm.unet_manual_cast(dtype, load_device)
    cfg = dict(cfg)
    cfg.pop("out_channels", None)
    cfg["hint_channels"] = data[f"{prefix}input_hint_block.0.weight"].shape[1]
    if prefix:
        if "difference" in data:                  # diff controlnet: weights are deltas to the base UNet
            if model is not None:
                dm.load_models_gpu([model])
                msd = model.model_state_dict()
                for k in list(data):
                    if k.startswith(prefix):
                        base_k = "diffusion_model." + k[len(prefix):]
                        if base_k in msd:
                            data[k] = data[k] + msd[base_k].to(data[k].dtype).to(data[k].device)
            else:
                logging.warning("diff controlnet loaded without a model; it will likely not work")
        data = state_dict_prefix_replace(data, {prefix: ""}, filter_keys=True)
    with torch.device("meta"):
        cm = ControlNetModel(dtype=dtype, device=torch.device("meta"), **cfg)
    cm.to_empty(device=dm.unet_offload_device())
    missing, unexpected = cm.load_state_dict(data, strict=False)
    if missing:
        logging.warning("missing controlnet keys: %s", missing)
    if unexpected:
        logging.debug("unexpected controlnet keys: %s", unexpected)
    name = os.path.splitext(ckpt_path)[0]
    gap = name.endswith("_shuffle") or name.endswith("_shuffle_fp16")
    return ControlNet(cm.eval(), global_average_pooling=gap, load_device=load_device, manual_cast_dtype=manual_cast)


# ---------------------------------------------------------------- T2I adapters
class T2IAdapter(ControlBase):
    def __init__(self, t2i_model, channels_in, compression_ratio, upscale_algorithm, device=None):
        super().__init__(device)
        self.t2i_model = t2i_model
        self.channels_in = channels_in
        self.control_input = None
        self.compression_ratio = compression_ratio
        self.upscale_algorithm = upscale_algorithm

    def scale_image_to(self, width, height):
        u = self.t2i_model.unshuffle_amount
        return math.ceil(width / u) * u, math.ceil(height / u) * u

    def get_control(self, x_noisy, t, cond, batched_number):
        prev = None
        if self.previous_controlnet is not None:
            prev = self.previous_controlnet.get_control(x_noisy, t, cond, batched_number)
        if self._outside_window(t):
            return prev
        w, h = self.scale_image_to(x_noisy.shape[3] * self.compression_ratio, x_noisy.shape[2] * self.compression_ratio)
        if self._hint_for(x_noisy, torch.float32, w, h):
            self.control_input = None
            if self.channels_in == 1 and self.cond_hint.shape[1] > 1:
                self.cond_hint = torch.mean(self.cond_hint, 1, keepdim=True)
        if x_noisy.shape[0] != self.cond_hint.shape[0]:
            self.cond_hint = broadcast_image_to(self.cond_hint, x_noisy.shape[0], batched_number)
        if self.control_input is None:            # the adapter runs once per hint (not per step)
            self.t2i_model.to(device=self.device, dtype=x_noisy.dtype)
            with torch.inference_mode():
                self.control_input = self.t2i_model(self.cond_hint.to(x_noisy.dtype))
        ci = [None if a is None else a.clone() for a in self.control_input]
        mid = None
        if self.t2i_model.xl:
            mid, ci = ci[-1:], ci[:-1]
        return self.control_merge(ci, mid, prev, x_noisy.dtype)

    def copy(self):
        c = T2IAdapter(self.t2i_model, self.channels_in, self.compression_ratio, self.upscale_algorithm)
        self.copy_to(c)
        return c


def load_t2i_adapter(data):
    compression_ratio = 8
    upscale = "nearest-exact"
    if "adapter" in data:
        data = data["adapter"]
    if "adapter.body.0.resnets.0.block1.weight" in data:             # diffusers layout
        rep = {}
        for i in range(4):
            for j in range(2):
                rep[f"adapter.body.{i}.resnets.{j}."] = f"body.{i * 2 + j}."
            rep[f"adapter.body.{i}."] = f"body.{i * 2}."
        rep["adapter."] = ""
        data = state_dict_prefix_replace(data, rep)
    keys = data.keys()
    if "body.0.in_conv.weight" in keys:
        model = Adapter_light(cin=data["body.0.in_conv.weight"].shape[1], channels=[320, 640, 1280, 1280], nums_rb=4)
    elif "conv_in.weight" in keys:
        cin = data["conv_in.weight"].shape[1]
        ch = data["conv_in.weight"].shape[0]
        ksize = data["body.0.block2.weight"].shape[2]
        use_conv = any(k.endswith("down_opt.op.weight") for k in keys)
        model = Adapter(cin=cin, channels=[ch, ch * 2, ch * 4, ch * 4], nums_rb=2, ksize=ksize, sk=True,
                        use_conv=use_conv, xl=cin in (256, 768))
    elif "backbone.0.0.weight" in keys or "backbone.10.blocks.0.weight" in keys:
        from ..models.cascade import CascadeControlNet
        large = "backbone.10.blocks.0.weight" in keys
        c_in = data["backbone.0.weight" if large else "backbone.0.0.weight"].shape[1]
        model = CascadeControlNet(c_in=c_in, bottleneck_mode="large" if large else None,
                                  proj_blocks=[0, 4, 8, 12, 51, 55, 59, 63])
        compression_ratio, upscale = (1, "nearest-exact") if large else (32, "bilinear")
    else:
        return None
    missing, unexpected = model.load_state_dict(data, strict=False)
    if missing:
        logging.warning("t2i adapter missing keys: %s", missing)
    if unexpected:
        logging.debug("t2i adapter unexpected keys: %s", unexpected)
    return T2IAdapter(model.eval(), model.input_channels, compression_ratio, upscale)
