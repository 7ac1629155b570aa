"""High-level loaders: CLIP, VAE, checkpoints, standalone UNet/CLIP, LoRA application, saving.

Parity with ``comfy/sd.py:1-622`` (C36): ``CLIP`` (tokenize -> encode_from_tokens with clip-skip
layer options), ``VAE`` (config sniffing: KL / TAESD / Cascade StageA / effnet / previewer;
batched decode/encode with tiled fallback), ``load_checkpoint_guess_config`` (detection ->
family -> dtype policy -> model + VAE + CLIP + ModelPatcher), ``load_unet``, ``load_clip``,
``load_lora_for_models``, ``save_checkpoint``.

Residency: the loaded modules are materialised directly in their inference dtype; nodes make them
resident on the device through ``device.load_models_gpu`` (once; they stay resident).
"""
from __future__ import annotations

import logging
import os
import math

import torch

from .. import ops

from . import device as dm
from . import detection, families
from .checkpoint import load_state_dict, save_state_dict, calculate_parameters, weight_dtype
from .convert import state_dict_prefix_replace
from .lora import load_lora, model_lora_keys_clip, model_lora_keys_unet
from .patcher import ModelPatcher


# ------------------------------------------------------------------------------------------------
class CLIP:
    def __init__(self, target=None, embedding_directory=None, no_init=False, dtype=None, device=None):
        if no_init:
            return
        from ..models.text_encoders import ClipStackTokenizer
        load_device = device or dm.text_encoder_device()
        offload = dm.text_encoder_offload_device()
        dtype = dtype or dm.text_encoder_dtype(load_device)
        self.cond_stage_model = target.stack(dtype=dtype, device=torch.device("meta"))
        self.cond_stage_model.to_empty(device=offload)
        self.tokenizer = ClipStackTokenizer(target.stack, embedding_directory=embedding_directory)
        self.patcher = ModelPatcher(self.cond_stage_model, load_device=load_device, offload_device=offload)
        self.layer_idx = None

    def clone(self):
        n = CLIP(no_init=True)
        n.patcher = self.patcher.clone()
        n.cond_stage_model = self.cond_stage_model
        n.tokenizer = self.tokenizer
        n.layer_idx = self.layer_idx
        return n

    def add_patches(self, patches, strength_patch=1.0, strength_model=1.0):
        return self.patcher.add_patches(patches, strength_patch, strength_model)

    def clip_layer(self, layer_idx):
        self.layer_idx = layer_idx

    def tokenize(self, text, return_word_ids=False):
        return self.tokenizer.tokenize_with_weights(text, return_word_ids)

    def encode_from_tokens(self, tokens, return_pooled=False):
        self.cond_stage_model.reset_clip_options()
        if self.layer_idx is not None:
            self.cond_stage_model.set_clip_options({"layer": self.layer_idx})
        if return_pooled == "unprojected":
            self.cond_stage_model.set_clip_options({"projected_pooled": False})
        dm.load_model_gpu(self.patcher)
        with torch.inference_mode():
            cond, pooled = self.cond_stage_model.encode_token_weights(tokens)
        dev = dm.intermediate_device()
        cond, pooled = cond.to(dev), (pooled.to(dev) if pooled is not None else None)
        if return_pooled:
            return cond, pooled
        return cond

    def encode(self, text):
        return self.encode_from_tokens(self.tokenize(text))

    def load_sd(self, sd, full_model=False):
        if full_model:
            return self.cond_stage_model.load_state_dict(sd, strict=False)
        return self.cond_stage_model.load_sd(sd)

    def get_sd(self):
        return self.cond_stage_model.state_dict()

    def load_model(self):
        dm.load_model_gpu(self.patcher)
        return self.patcher

    def get_key_patches(self):
        return self.patcher.get_key_patches()


# ------------------------------------------------------------------------------------------------
class VAE:
    def __init__(self, sd=None, device=None, config=None, dtype=None):
        from ..models import vae as V
        self.memory_used_encode = lambda shape, dtype: (1767 * shape[2] * shape[3]) * dm.dtype_size(dtype)
        self.memory_used_decode = lambda shape, dtype: (2178 * shape[2] * shape[3] * 64) * dm.dtype_size(dtype)
        self.downscale_ratio = 8
        self.upscale_ratio = 8
        self.latent_channels = 4
        self.output_channels = 3
        self.process_input = lambda image: image * 2.0 - 1.0
        self.process_output = lambda image: torch.clamp((image + 1.0) / 2.0, min=0.0, max=1.0)
        self.kind = "kl"
        if sd is not None and "decoder.up_blocks.0.resnets.0.norm1.weight" in sd:
            from .diffusers import convert_vae_state_dict
            sd = convert_vae_state_dict(sd)
        if config is None:
            if sd is not None and "taesd_decoder.1.weight" in sd:
                from ..models.taesd import TAESD
                self.first_stage_model = TAESD(latent_channels=sd["taesd_decoder.1.weight"].shape[1])
                self.kind = "taesd"
            elif sd is not None and "vquantizer.codebook.weight" in sd:
                from ..models.cascade import StageA
                self.first_stage_model = StageA()
                self.downscale_ratio = 4
                self.upscale_ratio = 4
                self.process_input = lambda image: image
                self.process_output = lambda image: image
                self.kind = "stage_a"
            elif sd is not None and "backbone.1.0.block.0.1.num_batches_tracked" in sd:
                from ..models.cascade import StageC_coder
                self.first_stage_model = StageC_coder()
                self.downscale_ratio = 32
                self.latent_channels = 16
                self.kind = "effnet"
                sd = {"encoder." + k: v for k, v in sd.items()}
            elif sd is not None and "blocks.11.num_batches_tracked" in sd:
                from ..models.cascade import StageC_coder
                self.first_stage_model = StageC_coder()
                self.latent_channels = 16
                self.kind = "previewer"
                sd = {"previewer." + k: v for k, v in sd.items()}
            else:
                ddconfig = dict(double_z=True, z_channels=4, resolution=256, in_channels=3, out_ch=3, ch=128,
                                ch_mult=[1, 2, 4, 4], num_res_blocks=2, attn_resolutions=[], dropout=0.0)
                if sd is not None:
                    # sniff the KL config from key names / shapes (levels, widths, res blocks)
                    if "decoder.conv_out.weight" in sd:
                        ddconfig["ch"] = sd["decoder.conv_out.weight"].shape[1]
                    elif "encoder.conv_in.weight" in sd:
                        ddconfig["ch"] = sd["encoder.conv_in.weight"].shape[0]
                    ch = ddconfig["ch"]
                    nlev = 0
                    while f"decoder.up.{nlev}.block.0.conv1.weight" in sd or f"encoder.down.{nlev}.block.0.conv1.weight" in sd:
                        nlev += 1
                    if nlev:
                        mult = []
                        for i in range(nlev):
                            k = f"decoder.up.{i}.block.0.conv2.weight"
                            k2 = f"encoder.down.{i}.block.0.conv2.weight"
                            w = sd.get(k, sd.get(k2))
                            mult.append(int(w.shape[0] // ch))
                        ddconfig["ch_mult"] = mult
                        self.downscale_ratio = self.upscale_ratio = 2 ** (nlev - 1)
                        nrb = 0
                        while f"decoder.up.0.block.{nrb}.conv1.weight" in sd:
                            nrb += 1
                        if nrb:
                            ddconfig["num_res_blocks"] = nrb - 1
                        else:
                            while f"encoder.down.0.block.{nrb}.conv1.weight" in sd:
                                nrb += 1
                            ddconfig["num_res_blocks"] = max(1, nrb)
                    if "decoder.conv_in.weight" in sd:
                        ddconfig["z_channels"] = sd["decoder.conv_in.weight"].shape[1]
                        self.latent_channels = ddconfig["z_channels"]
                    if "decoder.mid.block_1.mix_factor" in sd:
                        # SVD temporal decoder (sd.py:175-182): time-mixing ResBlocks + AE3DConv out
                        ddconfig.update(video_kernel_size=[3, 1, 1], alpha=0.0)
                        self.kind = "video"
                self.first_stage_model = V.AutoencoderKL(embed_dim=ddconfig["z_channels"], ddconfig=ddconfig,
                                                         device=torch.device("meta"))
                self.first_stage_model.to_empty(device="cpu")
        else:
            self.first_stage_model = V.AutoencoderKL(**config)
        self.first_stage_model = self.first_stage_model.eval()
        if sd is not None:
            m, u = self.first_stage_model.load_state_dict(sd, strict=False)
            if m:
                logging.warning("Missing VAE keys %s", m[:10])
            if u:
                logging.debug("Leftover VAE keys %s", u[:10])
        self.device = device or dm.vae_device()
        self.vae_dtype = dtype or dm.vae_dtype(self.device)
        self.first_stage_model.to(self.vae_dtype)
        self.output_device = dm.intermediate_device()
        self.patcher = ModelPatcher(self.first_stage_model, load_device=self.device,
                                    offload_device=dm.vae_offload_device())
        self.batch = 8

    def _mf(self, x):
        return x.to(device=self.device, dtype=self.vae_dtype).contiguous(
            memory_format=torch.channels_last if self.device.type == "cuda" else torch.contiguous_format)

    def decode(self, samples_in):
        """Batched decode; on HBM exhaustion retry as the 3-pass tiled decode (reference
        ``comfy/sd.py:300-302``). Fault site ``CGS_FAULT=oom:vae_decode`` exercises the fallback."""
        try:
            from ..utils.telemetry import maybe_fault
            maybe_fault("vae", "vae_decode")
            return self._decode_full(samples_in)
        except torch.cuda.OutOfMemoryError:
            logging.warning("Ran out of memory in regular VAE decoding; retrying with tiled VAE decoding.")
            dm.soft_empty_cache(force=True)
            return self.decode_tiled_(samples_in)

    def decode_tiled_(self, samples, tile_x=64, tile_y=64, overlap=16):
        """Three tilings with rotated aspect averaged (reference ``sd.py:261-286``): the seams of one
        tiling fall inside the tiles of the others."""
        return (self.decode_tiled(samples, tile_x // 2, tile_y * 2, overlap) +
                self.decode_tiled(samples, tile_x * 2, tile_y // 2, overlap) +
                self.decode_tiled(samples, tile_x, tile_y, overlap)) / 3.0

    def decode_uint8(self, samples_in):
        """Decode straight to the uint8 [B, H, W, 3] image (server / DP gather format): the conv_out
        output goes through one fused kernel (K23) instead of fp32 upcast + scaling + uint8 passes."""
        if self.kind != "kl" or self.device.type != "cuda" or self.vae_dtype != torch.bfloat16:
            px = self.decode(samples_in)
            return (px.clamp(0, 1) * 255.0 + 0.5).to(torch.uint8)
        try:
            from ..utils.telemetry import maybe_fault
            maybe_fault("vae", "vae_decode")
            dm.load_model_gpu(self.patcher)
            out = []
            with torch.inference_mode():
                for i in range(0, samples_in.shape[0], self.batch):
                    img = self.first_stage_model.decode(self._mf(samples_in[i:i + self.batch]))
                    out.append(ops.vae_out_u8(img.contiguous(memory_format=torch.channels_last)))
            return torch.cat(out, 0)
        except torch.cuda.OutOfMemoryError:
            logging.warning("Ran out of memory in regular VAE decoding; retrying with tiled VAE decoding.")
            dm.soft_empty_cache(force=True)
            px = self.decode_tiled_(samples_in)
            return (px.clamp(0, 1) * 255.0 + 0.5).to(torch.uint8)

    def _decode_full(self, samples_in):
        dm.load_model_gpu(self.patcher)
        out = []
        # the temporal decoder mixes across the frames of a decode call: decode a clip in one call
        step = samples_in.shape[0] if self.kind == "video" else self.batch
        with torch.inference_mode():
            for i in range(0, samples_in.shape[0], max(1, step)):
                s = self._mf(samples_in[i:i + max(1, step)])
                img = self.first_stage_model.decode(s)
                out.append(self.process_output(img.float()).to(self.output_device))
        pixels = torch.cat(out, 0)
        return pixels.movedim(1, -1).contiguous()

    def decode_tiled(self, samples, tile_x=64, tile_y=64, overlap=16):
        from ..utils.image import tiled_scale
        dm.load_model_gpu(self.patcher)
        with torch.inference_mode():
            fn = lambda a: self.process_output(self.first_stage_model.decode(self._mf(a)).float())  # noqa: E731
            out = tiled_scale(samples, fn, tile_x, tile_y, overlap, upscale_amount=self.upscale_ratio,
                              out_channels=self.output_channels, output_device=self.output_device)
        return out.movedim(1, -1)

    def encode(self, pixel_samples):
        """Batched encode with the OOM -> tiled fallback (reference ``comfy/sd.py:326-328``; fault site
        ``CGS_FAULT=oom:vae_encode``)."""
        try:
            from ..utils.telemetry import maybe_fault
            maybe_fault("vae", "vae_encode")
            return self._encode_full(pixel_samples)
        except torch.cuda.OutOfMemoryError:
            logging.warning("Ran out of memory in regular VAE encoding; retrying with tiled VAE encoding.")
            dm.soft_empty_cache(force=True)
            return self.encode_tiled_(pixel_samples)

    def encode_tiled_(self, pixel_samples, tile_x=512, tile_y=512, overlap=64):
        return (self.encode_tiled(pixel_samples, tile_x, tile_y, overlap) +
                self.encode_tiled(pixel_samples, tile_x * 2, tile_y // 2, overlap) +
                self.encode_tiled(pixel_samples, tile_x // 2, tile_y * 2, overlap)) / 3.0

    def _encode_full(self, pixel_samples):
        dm.load_model_gpu(self.patcher)
        px = pixel_samples.movedim(-1, 1)
        out = []
        with torch.inference_mode():
            for i in range(0, px.shape[0], self.batch):
                p = self._mf(self.process_input(px[i:i + self.batch].float()))
                out.append(self.first_stage_model.encode(p).float().to(self.output_device))
        return torch.cat(out, 0)

    def encode_tiled(self, pixel_samples, tile_x=512, tile_y=512, overlap=64):
        from ..utils.image import tiled_scale
        dm.load_model_gpu(self.patcher)
        px = pixel_samples.movedim(-1, 1)
        with torch.inference_mode():
            fn = lambda a: self.first_stage_model.encode(self._mf(self.process_input(a.float()))).float()  # noqa: E731
            return tiled_scale(px, fn, tile_x, tile_y, overlap, upscale_amount=1.0 / self.downscale_ratio,
                               out_channels=self.latent_channels, output_device=self.output_device)

    def get_sd(self):
        return self.first_stage_model.state_dict()


class StyleModel:
    def __init__(self, model, device="cpu"):
        self.model = model

    def get_cond(self, input):
        return self.model(input.last_hidden_state)


def load_style_model(ckpt_path):
    from ..models.t2i_adapter import StyleAdapter
    sd = load_state_dict(ckpt_path)
    keys = sd.keys()
    if "style_embedding" in keys:
        model = StyleAdapter(width=1024, context_dim=768, num_head=8, n_layes=3, num_token=8)
    else:
        raise Exception(f"invalid style model {ckpt_path}")
    model.load_state_dict(sd)
    return StyleModel(model)


# ------------------------------------------------------------------------------------------------
def _materialise(model, sd_dtype, device):
    """Model created on meta -> real storage on ``device`` in its dtype."""
    model.to_empty(device=device)
    return model


def _direct_load_device():
    """Where checkpoint bytes should land: straight into HBM when models stay resident there
    (HIGH_VRAM on a ROCm device — the 288 GB default), else host memory."""
    d = dm.get_torch_device()
    if d.type == "cuda" and dm.vram_state == dm.VRAMState.HIGH_VRAM and os.environ.get("CGS_DIRECT_LOAD", "1") != "0":
        return d
    return torch.device("cpu")


def load_checkpoint_guess_config(ckpt_path, output_vae=True, output_clip=True, output_clipvision=False,
                                 embedding_directory=None, output_model=True, sd=None):
    sd = sd if sd is not None else load_state_dict(ckpt_path, device=_direct_load_device())
    return load_state_dict_guess_config(sd, output_vae, output_clip, output_clipvision, embedding_directory,
                                        output_model)


def load_state_dict_guess_config(sd, output_vae=True, output_clip=True, output_clipvision=False,
                                 embedding_directory=None, output_model=True):
    clip = vae = model_patcher = clipvision = None
    prefix = "model.diffusion_model."
    params = calculate_parameters(sd, prefix)
    load_device = dm.get_torch_device()
    mc = detection.model_config_from_unet(sd, prefix)
    if mc is None:
        raise RuntimeError("ERROR: Could not detect model type of checkpoint")
    uw_dtype = weight_dtype(sd, prefix)
    unet_dtype = dm.unet_dtype(load_device, params, mc.supported_inference_dtypes)
    mc.set_inference_dtype(unet_dtype, dm.unet_manual_cast(unet_dtype, load_device, mc.supported_inference_dtypes))
    if mc.clip_vision_prefix is not None and output_clipvision:
        from .clip_vision import load_clipvision_from_sd
        clipvision = load_clipvision_from_sd(sd, mc.clip_vision_prefix, True)
    if output_model:
        with torch.device("meta"):
            model = mc.get_model(sd, prefix, device=torch.device("meta"))
        model.to_empty(device=dm.unet_offload_device())
        model.model_sampling = model.model_sampling.__class__(mc)   # buffers were on meta
        model.load_model_weights(sd, prefix)
        model.diffusion_model.to(unet_dtype)
        model_patcher = ModelPatcher(model, load_device=load_device, offload_device=dm.unet_offload_device())
    if output_vae:
        vsd = state_dict_prefix_replace(sd, {k: "" for k in mc.vae_key_prefix}, filter_keys=True)
        vsd = mc.process_vae_state_dict(vsd)
        vae = VAE(sd=vsd)
    if output_clip:
        ct = mc.clip_target()
        if ct is not None:
            csd = mc.process_clip_state_dict(sd)
            if csd:
                clip = CLIP(ct, embedding_directory=embedding_directory)
                m, u = clip.load_sd(csd, full_model=True)
                m = [k for k in m if not k.endswith(".position_ids") and "logit_scale" not in k]
                if m:
                    logging.warning("clip missing: %s", m[:10])
            else:
                logging.warning("no CLIP/text encoder weights in checkpoint, the text encoder model will not be loaded.")
    leftover = [k for k in sd if not k.startswith(prefix)]
    if leftover:
        logging.debug("left over keys: %s", leftover[:10])
    return model_patcher, clip, vae, clipvision


def load_unet_state_dict(sd, dtype=None):
    params = calculate_parameters(sd)
    load_device = dm.get_torch_device()
    if "input_blocks.0.0.weight" in sd or "clf.1.weight" in sd:
        mc = detection.model_config_from_unet(sd, "")
        if mc is None:
            return None
        new_sd = sd
    else:
        from .diffusers import model_config_from_diffusers_unet, convert_unet_from_diffusers
        mc = model_config_from_diffusers_unet(sd)
        if mc is None:
            return None
        new_sd = convert_unet_from_diffusers(sd, mc.unet_config)
    unet_dtype = dtype or dm.unet_dtype(load_device, params, mc.supported_inference_dtypes)
    mc.set_inference_dtype(unet_dtype, dm.unet_manual_cast(unet_dtype, load_device))
    with torch.device("meta"):
        model = mc.get_model(new_sd, "", device=torch.device("meta"))
    model.to_empty(device=dm.unet_offload_device())
    model.model_sampling = model.model_sampling.__class__(mc)
    model.load_model_weights(new_sd, "")
    model.diffusion_model.to(unet_dtype)
    return ModelPatcher(model, load_device=load_device, offload_device=dm.unet_offload_device())


def load_unet(path, dtype=None):
    sd = load_state_dict(path, device=_direct_load_device())
    m = load_unet_state_dict(sd, dtype)
    if m is None:
        raise RuntimeError(f"ERROR UNSUPPORTED UNET {path}")
    return m


class CLIPType:
    STABLE_DIFFUSION = 1
    STABLE_CASCADE = 2


def load_clip(ckpt_paths, embedding_directory=None, clip_type=CLIPType.STABLE_DIFFUSION):
    from ..models import text_encoders as te
    sds = [load_state_dict(p) for p in ckpt_paths]
    conv = []
    for sd in sds:
        if "text_model.encoder.layers.1.mlp.fc1.weight" in sd:
            conv.append(state_dict_prefix_replace(sd, {"": "transformer."}))
        elif "transformer.resblocks.1.mlp.c_fc.weight" in sd:
            from .convert import openclip_to_hf
            conv.append(openclip_to_hf(dict(sd), "", "transformer."))
        else:
            conv.append(sd)
    sds = conv

    def width(sd):
        w = sd.get("transformer.text_model.encoder.layers.0.self_attn.q_proj.weight")
        return None if w is None else w.shape[0]

    class T:
        pass

    if len(sds) == 1:
        w = width(sds[0])
        if clip_type == CLIPType.STABLE_CASCADE:
            stack, names = te.StableCascadeClipModel, ["g"]
        elif w == 1280:
            stack, names = te.SDXLRefinerClipModel, ["g"]
        elif w == 1024:
            stack, names = te.SD2ClipModel, ["h"]
        else:
            stack, names = te.SD1ClipModel, ["l"]
    else:
        stack, names = te.SDXLClipModel, ["l", "g"]
        sds = sorted(sds, key=lambda s: width(s) or 0)
    ct = families.ClipTarget(stack)
    clip = CLIP(ct, embedding_directory=embedding_directory)
    merged = {}
    for n, sd in zip(names, sds):
        for k, v in sd.items():
            merged[f"clip_{n}.{k}"] = v
    clip.load_sd(merged, full_model=True)
    return clip


def load_lora_for_models(model, clip, lora, strength_model, strength_clip):
    key_map = {}
    if model is not None:
        key_map = model_lora_keys_unet(model.model, key_map)
    if clip is not None:
        key_map = model_lora_keys_clip(clip.cond_stage_model, key_map)
    loaded = load_lora(lora, key_map)
    new_model = new_clip = None
    if model is not None:
        new_model = model.clone()
        k = set(new_model.add_patches(loaded, strength_model))
    else:
        k = set()
    if clip is not None:
        new_clip = clip.clone()
        k1 = set(new_clip.add_patches(loaded, strength_clip))
    else:
        k1 = set()
    for x in loaded:
        if x not in k and x not in k1:
            logging.warning("NOT LOADED %s", x)
    return new_model, new_clip


def save_checkpoint(output_path, model, clip=None, vae=None, clip_vision=None, metadata=None, extra_keys=None):
    clip_sd = vae_sd = cv_sd = None
    load_models = [model]
    if clip is not None:
        load_models.append(clip.load_model())
        clip_sd = clip.get_sd()
    if vae is not None:
        vae_sd = vae.get_sd()
    if clip_vision is not None:
        cv_sd = clip_vision.get_sd()
    dm.load_models_gpu(load_models)
    sd = model.model.state_dict_for_saving(clip_sd, vae_sd, cv_sd)
    for k, v in (extra_keys or {}).items():
        sd[k] = v
    save_state_dict(sd, output_path, metadata=metadata)
