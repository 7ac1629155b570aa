"""Model-patch nodes (parity: ``comfy_extras/nodes_model_advanced.py``, ``nodes_freelunch.py``, ``nodes_sag.py``,
``nodes_pag.py``, ``nodes_perpneg.py``, ``nodes_hypertile.py``, ``nodes_tomesd.py``, ``nodes_model_downscale.py``,
``nodes_differential_diffusion.py``, ``nodes_video_model.py`` CFG guidances).

Every node clones the ModelPatcher and installs a hook (object patch, sampler cfg / post-cfg
function, attention patch or replace, block patch, denoise-mask function); the UNet and the CFG
plumbing (sampling.samplers) call them at the same points as the reference. A patched model takes
the hook-aware transformer path; the hook-free fast path (fused epilogues) stays for plain models.
"""
from __future__ import annotations

import logging
import math

import torch
import torch.nn.functional as F

from .. import ops
from ..runtime import latent_formats
from ..runtime.patcher import set_model_options_patch_replace
from ..sampling import model_sampling as MS
from ..sampling import sampler_helpers
from ..sampling.samplers import _host_sigma
from ..sampling import samplers as SM
from ..utils import image as U
from .. import ops

# ================================================================ model sampling overrides


def rescale_zero_terminal_snr_sigmas(sigmas):
    """Zero-terminal-SNR rescale of a discrete schedule (Lin et al. 2023), in sigma space."""
    ab_sqrt = (1.0 / (sigmas * sigmas + 1.0)).sqrt()
    a0, aT = ab_sqrt[0].clone(), ab_sqrt[-1].clone()
    ab_sqrt = (ab_sqrt - aT) * (a0 / (a0 - aT))
    ab = ab_sqrt ** 2
    ab[-1] = 4.8973451890853435e-08
    return ((1.0 - ab) / ab) ** 0.5


class ModelSamplingDiscrete:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model": ("MODEL",), "sampling": (["eps", "v_prediction", "lcm", "x0"],),
                             "zsnr": ("BOOLEAN", {"default": False})}}
    RETURN_TYPES = ("MODEL",)
    FUNCTION = "patch"
    CATEGORY = "advanced/model"

    def patch(self, model, sampling, zsnr):
        m = model.clone()
        base = MS.ModelSamplingDiscrete
        ptype = {"eps": MS.EPS, "v_prediction": MS.V_PREDICTION, "lcm": MS.LCM, "x0": MS.X0}[sampling]
        if sampling == "lcm":
            base = MS.ModelSamplingDiscreteDistilled

        class ModelSamplingAdvanced(base, ptype):
            pass
        ms = ModelSamplingAdvanced(model.model.model_config)
        if zsnr:
            ms.set_sigmas(rescale_zero_terminal_snr_sigmas(ms.sigmas))
        m.add_object_patch("model_sampling", ms)
        return (m,)


class ModelSamplingStableCascade:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model": ("MODEL",),
                             "shift": ("FLOAT", {"default": 2.0, "min": 0.0, "max": 100.0, "step": 0.01})}}
    RETURN_TYPES = ("MODEL",)
    FUNCTION = "patch"
    CATEGORY = "advanced/model"

    def patch(self, model, shift):
        m = model.clone()

        class ModelSamplingAdvanced(MS.StableCascadeSampling, MS.EPS):
            pass
        ms = ModelSamplingAdvanced(model.model.model_config)
        ms.set_parameters(shift)
        m.add_object_patch("model_sampling", ms)
        return (m,)


class ModelSamplingContinuousEDM:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model": ("MODEL",), "sampling": (["v_prediction", "edm_playground_v2.5", "eps"],),
                             "sigma_max": ("FLOAT", {"default": 120.0, "min": 0.0, "max": 1000.0, "step": 0.001,
                                                     "round": False}),
                             "sigma_min": ("FLOAT", {"default": 0.002, "min": 0.0, "max": 1000.0, "step": 0.001,
                                                     "round": False})}}
    RETURN_TYPES = ("MODEL",)
    FUNCTION = "patch"
    CATEGORY = "advanced/model"

    def patch(self, model, sampling, sigma_max, sigma_min):
        m = model.clone()
        sigma_data = 1.0
        lf = None
        ptype = {"eps": MS.EPS, "v_prediction": MS.V_PREDICTION, "edm_playground_v2.5": MS.EDM}[sampling]
        if sampling == "edm_playground_v2.5":
            sigma_data = 0.5
            lf = latent_formats.SDXL_Playground_2_5()

        class ModelSamplingAdvanced(MS.ModelSamplingContinuousEDM, ptype):
            pass
        ms = ModelSamplingAdvanced(model.model.model_config)
        ms.set_parameters(sigma_min, sigma_max, sigma_data)
        m.add_object_patch("model_sampling", ms)
        if lf is not None:
            m.add_object_patch("latent_format", lf)
        return (m,)


# ================================================================ CFG-function patches
def _bcast(sigma, ref):
    return sigma.view(sigma.shape[:1] + (1,) * (ref.ndim - 1))


class RescaleCFG:
    """CFG rescale (Lin et al. 2023 §3.4) done on the v-prediction of the model output."""

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model": ("MODEL",),
                             "multiplier": ("FLOAT", {"default": 0.7, "min": 0.0, "max": 1.0, "step": 0.01})}}
    RETURN_TYPES = ("MODEL",)
    FUNCTION = "patch"
    CATEGORY = "advanced/model"

    def patch(self, model, multiplier):
        def rescale_cfg(args):
            cond, uncond, scale = args["cond"], args["uncond"], args["cond_scale"]
            x_orig = args["input"]
            sigma = _bcast(args["sigma"], cond)
            x = x_orig / (sigma * sigma + 1.0)
            to_v = lambda e: ((x - (x_orig - e)) * (sigma ** 2 + 1.0) ** 0.5) / sigma  # noqa: E731
            vc, vu = to_v(cond), to_v(uncond)
            v_cfg = vu + scale * (vc - vu)
            v_resc = v_cfg * (torch.std(vc, dim=(1, 2, 3), keepdim=True) / torch.std(v_cfg, dim=(1, 2, 3), keepdim=True))
            v_final = multiplier * v_resc + (1.0 - multiplier) * v_cfg
            return x_orig - (x - v_final * sigma / (sigma * sigma + 1.0) ** 0.5)
        m = model.clone()
        m.set_model_sampler_cfg_function(rescale_cfg)
        return (m,)


class VideoLinearCFGGuidance:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model": ("MODEL",),
                             "min_cfg": ("FLOAT", {"default": 1.0, "min": 0.0, "max": 100.0, "step": 0.5, "round": 0.01})}}
    RETURN_TYPES = ("MODEL",)
    FUNCTION = "patch"
    CATEGORY = "sampling/video_models"

    def patch(self, model, min_cfg):
        def linear_cfg(args):
            c, u = args["cond"], args["uncond"]
            s = torch.linspace(min_cfg, args["cond_scale"], c.shape[0], device=c.device).reshape(-1, 1, 1, 1)
            return u + s * (c - u)
        m = model.clone()
        m.set_model_sampler_cfg_function(linear_cfg)
        return (m,)


class VideoTriangleCFGGuidance:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model": ("MODEL",),
                             "min_cfg": ("FLOAT", {"default": 1.0, "min": 0.0, "max": 100.0, "step": 0.5, "round": 0.01})}}
    RETURN_TYPES = ("MODEL",)
    FUNCTION = "patch"
    CATEGORY = "sampling/video_models"

    def patch(self, model, min_cfg):
        def tri_cfg(args):
            c, u = args["cond"], args["uncond"]
            t = torch.linspace(0, 1, c.shape[0], device=c.device)
            tri = 2 * (t - torch.floor(t + 0.5)).abs()          # triangle wave, period 1
            s = (tri * (args["cond_scale"] - min_cfg) + min_cfg).reshape(-1, 1, 1, 1)
            return u + s * (c - u)
        m = model.clone()
        m.set_model_sampler_cfg_function(tri_cfg)
        return (m,)


def perp_neg(x, pos_pred, neg_pred, nocond_pred, neg_scale, cond_scale):
    """Perp-Neg combine (nodes_perpneg.py:9-16): projection over the WHOLE tensor (not per sample)."""
    pos = pos_pred - nocond_pred
    neg = neg_pred - nocond_pred
    perp = neg - (torch.mul(neg, pos).sum() / (torch.norm(pos) ** 2)) * pos
    return nocond_pred + cond_scale * (pos - perp * neg_scale)


class PerpNeg:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model": ("MODEL",), "empty_conditioning": ("CONDITIONING",),
                             "neg_scale": ("FLOAT", {"default": 1.0, "min": 0.0, "max": 100.0, "step": 0.01})}}
    RETURN_TYPES = ("MODEL",)
    FUNCTION = "patch"
    CATEGORY = "_for_testing"

    def patch(self, model, empty_conditioning, neg_scale):
        m = model.clone()
        nocond = sampler_helpers.convert_cond(empty_conditioning)

        def cfg_function(args):
            mdl = args["model"]
            x = args["input"]
            processed = SM.encode_model_conds(mdl.extra_conds, nocond, x, x.device, "negative")
            (nocond_pred,) = SM.calc_cond_batch(mdl, [processed], x, args["sigma"], args["model_options"])
            return x - perp_neg(x, args["cond_denoised"], args["uncond_denoised"], nocond_pred, neg_scale,
                                args["cond_scale"])
        m.set_model_sampler_cfg_function(cfg_function)
        return (m,)


# ================================================================ attention-based guidance
def attention_with_probs(q, k, v, heads):
    """Attention that also returns the softmax probabilities [(b*h), Sq, Sk] (fp32); K05 op."""
    return ops.attention_with_probs(q, k, v, heads)


def gaussian_blur_2d(img, kernel_size, sigma):
    half = (kernel_size - 1) * 0.5
    # built on the device: no host->device copy, so SAG's post-CFG hook is hipGraph-capturable
    t = torch.linspace(-half, half, steps=kernel_size, device=img.device, dtype=torch.float32)
    pdf = torch.exp(-0.5 * (t / sigma).pow(2))
    k1 = (pdf / pdf.sum()).to(dtype=img.dtype)
    k2 = torch.outer(k1, k1).expand(img.shape[-3], 1, kernel_size, kernel_size)
    p = kernel_size // 2
    return F.conv2d(F.pad(img, (p, p, p, p), mode="reflect"), k2, groups=img.shape[-3])


def create_blur_map(x0, attn, sigma=3.0, threshold=1.0):
    """Blur x0 where the uncond middle-block self-attention is 'spread' (SAG degraded input)."""
    _, hw1, _ = attn.shape
    b, _, lh, lw = x0.shape
    attn = attn.reshape(b, -1, hw1, attn.shape[-1])
    mask = attn.mean(1).sum(1) > threshold
    ratio = 2 ** (math.ceil(math.sqrt(lh * lw / hw1)) - 1).bit_length()
    mask = mask.reshape(b, math.ceil(lh / ratio), math.ceil(lw / ratio))[:, None].to(x0.dtype)
    mask = F.interpolate(mask, (lh, lw))
    blurred = gaussian_blur_2d(x0, kernel_size=9, sigma=sigma)
    return blurred * mask + x0 * (1 - mask)


class SelfAttentionGuidance:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model": ("MODEL",),
                             "scale": ("FLOAT", {"default": 0.5, "min": -2.0, "max": 5.0, "step": 0.1}),
                             "blur_sigma": ("FLOAT", {"default": 2.0, "min": 0.0, "max": 10.0, "step": 0.1})}}
    RETURN_TYPES = ("MODEL",)
    FUNCTION = "patch"
    CATEGORY = "_for_testing"

    def patch(self, model, scale, blur_sigma):
        m = model.clone()
        state = {"attn": None}

        def attn_and_record(q, k, v, extra):
            heads = extra["n_heads"]
            cou = extra["cond_or_uncond"]
            b = q.shape[0] // len(cou)
            if 1 in cou:
                out, probs = attention_with_probs(q, k, v, heads)
                i = cou.index(1)
                state["attn"] = probs[heads * b * i:heads * b * (i + 1)]
                return out
            return ops.attention(q, k, v, heads)

        def post_cfg(args):
            res = args["denoised"]
            if min(res.shape[2:]) <= 4 or state["attn"] is None:
                return res
            uncond_pred = args["uncond_denoised"]
            x = args["input"]
            degraded = create_blur_map(uncond_pred, state["attn"], blur_sigma, 1.0)
            (sag,) = SM.calc_cond_batch(args["model"], [args["uncond"]], degraded + x - uncond_pred, args["sigma"],
                                        args["model_options"])
            return res + (degraded - sag) * scale

        m.set_model_sampler_post_cfg_function(post_cfg, disable_cfg1_optimization=True)
        m.set_model_attn1_replace(attn_and_record, "middle", 0, 0)
        return (m,)


class PerturbedAttentionGuidance:
    """PAG: a second conditional pass with the middle block's self-attention replaced by identity
    (output = V), guidance = cfg + scale * (cond - perturbed)."""

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model": ("MODEL",),
                             "scale": ("FLOAT", {"default": 3.0, "min": 0.0, "max": 100.0, "step": 0.1, "round": 0.01})}}
    RETURN_TYPES = ("MODEL",)
    FUNCTION = "patch"
    CATEGORY = "_for_testing"

    def patch(self, model, scale):
        m = model.clone()

        def perturbed_attention(q, k, v, extra, mask=None):
            return v

        def post_cfg(args):
            res = args["denoised"]
            if scale == 0:
                return res
            mo = set_model_options_patch_replace(args["model_options"].copy(), perturbed_attention, "attn1",
                                                 "middle", 0)
            (pag,) = SM.calc_cond_batch(args["model"], [args["cond"]], args["input"], args["sigma"], mo)
            return res + (args["cond_denoised"] - pag) * scale

        m.set_model_sampler_post_cfg_function(post_cfg)
        return (m,)


# ================================================================ block patches
def fourier_filter(x, threshold, scale):
    """Scale the low-frequency square (|f| < threshold around DC) of each channel by ``scale``
    (ops.fourier_filter: HIP DFT-coefficient kernels on the device, torch.fft on the CPU)."""
    return ops.fourier_filter(x, threshold, scale)


def _fourier_safe(hsp, s, cpu_devs):
    if hsp.device not in cpu_devs:
        try:
            return fourier_filter(hsp, 1, s)
        except Exception:
            logging.warning("FreeU Fourier filter failed on %s, using the CPU", hsp.device)
            cpu_devs.add(hsp.device)
    return fourier_filter(hsp.cpu(), 1, s).to(hsp.device)


class FreeU:
    @classmethod
    def INPUT_TYPES(s):
        f = lambda d: ("FLOAT", {"default": d, "min": 0.0, "max": 10.0, "step": 0.01})  # noqa: E731
        return {"required": {"model": ("MODEL",), "b1": f(1.1), "b2": f(1.2), "s1": f(0.9), "s2": f(0.2)}}
    RETURN_TYPES = ("MODEL",)
    FUNCTION = "patch"
    CATEGORY = "model_patches"
    V2 = False

    def patch(self, model, b1, b2, s1, s2):
        mc = model.model.model_config.unet_config["model_channels"]
        scales = {mc * 4: (b1, s1), mc * 2: (b2, s2)}
        cpu_devs = set()
        v2 = self.V2

        def output_block_patch(h, hsp, transformer_options):
            sc = scales.get(h.shape[1])
            if sc is None:
                return h, hsp
            half = h.shape[1] // 2
            h = h.clone()
            if v2:
                hm = h.mean(1, keepdim=True)
                B = hm.shape[0]
                hmax = hm.view(B, -1).max(dim=-1, keepdim=True)[0][:, :, None, None]
                hmin = hm.view(B, -1).min(dim=-1, keepdim=True)[0][:, :, None, None]
                hm = (hm - hmin) / (hmax - hmin)
                h[:, :half] = h[:, :half] * ((sc[0] - 1) * hm + 1)
            else:
                h[:, :half] = h[:, :half] * sc[0]
            return h, _fourier_safe(hsp, sc[1], cpu_devs)

        m = model.clone()
        m.set_model_output_block_patch(output_block_patch)
        return (m,)


class FreeU_V2(FreeU):
    V2 = True

    @classmethod
    def INPUT_TYPES(s):
        f = lambda d: ("FLOAT", {"default": d, "min": 0.0, "max": 10.0, "step": 0.01})  # noqa: E731
        return {"required": {"model": ("MODEL",), "b1": f(1.3), "b2": f(1.4), "s1": f(0.9), "s2": f(0.2)}}


class PatchModelAddDownscale:
    """Kohya deep-shrink: downscale the hidden state after input block N for the early (high
    sigma) part of sampling; output blocks upsample back to the skip's size."""
    upscale_methods = ["bicubic", "nearest-exact", "bilinear", "area", "bislerp"]

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model": ("MODEL",),
                             "block_number": ("INT", {"default": 3, "min": 1, "max": 32, "step": 1}),
                             "downscale_factor": ("FLOAT", {"default": 2.0, "min": 0.1, "max": 9.0, "step": 0.001}),
                             "start_percent": ("FLOAT", {"default": 0.0, "min": 0.0, "max": 1.0, "step": 0.001}),
                             "end_percent": ("FLOAT", {"default": 0.35, "min": 0.0, "max": 1.0, "step": 0.001}),
                             "downscale_after_skip": ("BOOLEAN", {"default": True}),
                             "downscale_method": (s.upscale_methods,), "upscale_method": (s.upscale_methods,)}}
    RETURN_TYPES = ("MODEL",)
    FUNCTION = "patch"
    CATEGORY = "_for_testing"

    def patch(self, model, block_number, downscale_factor, start_percent, end_percent, downscale_after_skip,
              downscale_method, upscale_method):
        ms = model.get_model_object("model_sampling")
        s_start = ms.percent_to_sigma(start_percent)
        s_end = ms.percent_to_sigma(end_percent)

        def input_block_patch(h, transformer_options):
            if transformer_options["block"][1] == block_number:
                sigma = _host_sigma(transformer_options["sigmas"])   # host copy: no sync, capturable
                if s_end <= sigma <= s_start:
                    h = U.common_upscale(h, round(h.shape[-1] / downscale_factor),
                                         round(h.shape[-2] / downscale_factor), downscale_method, "disabled")
            return h

        def output_block_patch(h, hsp, transformer_options):
            if h.shape[2] != hsp.shape[2]:
                h = U.common_upscale(h, hsp.shape[-1], hsp.shape[-2], upscale_method, "disabled")
            return h, hsp

        m = model.clone()
        if downscale_after_skip:
            m.set_model_input_block_patch_after_skip(input_block_patch)
        else:
            m.set_model_input_block_patch(input_block_patch)
        m.set_model_output_block_patch(output_block_patch)
        return (m,)


class DifferentialDiffusion:
    """Per-pixel denoise strength: a mask pixel joins the denoising once the schedule's progress
    passes its value (threshold on the normalised timestep)."""

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model": ("MODEL",)}}
    RETURN_TYPES = ("MODEL",)
    FUNCTION = "apply"
    CATEGORY = "_for_testing"

    def apply(self, model):
        m = model.clone()
        m.set_model_denoise_mask_function(self.forward)
        return (m,)

    def forward(self, sigma, denoise_mask, extra_options):
        mdl = extra_options["model"]
        ms = mdl.inner_model.model_sampling
        step_sigmas = extra_options["sigmas"]
        sigma_to = ms.sigma_min
        if step_sigmas[-1] > sigma_to:
            sigma_to = step_sigmas[-1]
        ts_from = ms.timestep(step_sigmas[0])
        ts_to = ms.timestep(torch.as_tensor(sigma_to))
        cur = ms.timestep(sigma[0])
        threshold = (cur - ts_to) / (ts_from - ts_to)
        return (denoise_mask >= threshold).to(denoise_mask.dtype)


# ================================================================ attention token patches
def _random_divisor(value, min_value, max_options=1):
    min_value = min(min_value, value)
    divisors = [i for i in range(min_value, value + 1) if value % i == 0]
    ns = [value // i for i in divisors[:max_options]]
    idx = int(torch.randint(0, len(ns), (1,)).item()) if len(ns) > 1 else 0
    return ns[idx]


class HyperTile:
    """Tile the self-attention of the largest (up to max_depth) resolutions into ~tile_size windows."""

    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model": ("MODEL",), "tile_size": ("INT", {"default": 256, "min": 1, "max": 2048}),
                             "swap_size": ("INT", {"default": 2, "min": 1, "max": 128}),
                             "max_depth": ("INT", {"default": 0, "min": 0, "max": 10}),
                             "scale_depth": ("BOOLEAN", {"default": False})}}
    RETURN_TYPES = ("MODEL",)
    FUNCTION = "patch"
    CATEGORY = "model_patches"

    def patch(self, model, tile_size, swap_size, max_depth, scale_depth):
        latent_tile = max(32, tile_size) // 8
        state = {"t": None}

        def hypertile_in(q, k, v, extra):
            tokens = q.shape[-2]
            shape = extra["original_shape"]
            levels = [(shape[-2] / 2 ** i) * (shape[-1] / 2 ** i) for i in range(max_depth + 1)]
            if tokens in levels:
                aspect = shape[-1] / shape[-2]
                hw = q.size(1)
                h, w = round(math.sqrt(hw * aspect)), round(math.sqrt(hw / aspect))
                factor = 2 ** levels.index(tokens) if scale_depth else 1
                nh = _random_divisor(h, latent_tile * factor, swap_size)
                nw = _random_divisor(w, latent_tile * factor, swap_size)
                if nh * nw > 1:
                    b, _, c = q.shape
                    q = (q.reshape(b, nh, h // nh, nw, w // nw, c).permute(0, 1, 3, 2, 4, 5)
                         .reshape(b * nh * nw, (h // nh) * (w // nw), c))
                    state["t"] = (nh, nw, h, w)
            return q, k, v

        def hypertile_out(out, extra):
            if state["t"] is not None:
                nh, nw, h, w = state["t"]
                state["t"] = None
                bt, _, c = out.shape
                b = bt // (nh * nw)
                out = (out.reshape(b, nh, nw, h // nh, w // nw, c).permute(0, 1, 3, 2, 4, 5).reshape(b, h * w, c))
            return out

        m = model.clone()
        m.set_model_attn1_patch(hypertile_in)
        m.set_model_attn1_output_patch(hypertile_out)
        return (m,)


def bipartite_soft_matching_random2d(metric, w, h, sx, sy, r, no_rand=False):
    """ToMe for SD token merging: one random dst token per (sy x sx) cell, the r most similar src
    tokens merged (mean) into their best dst; returns (merge, unmerge)."""
    B, N, _ = metric.shape
    if r <= 0 or w == 1 or h == 1:
        return (lambda x, mode=None: x), (lambda x: x)
    dev = metric.device
    with torch.no_grad():
        hsy, wsx = h // sy, w // sx
        if no_rand:
            pick = torch.zeros(hsy, wsx, 1, device=dev, dtype=torch.int64)
        else:
            pick = torch.randint(sy * sx, size=(hsy, wsx, 1), device=dev)
        cell = torch.zeros(hsy, wsx, sy * sx, device=dev, dtype=torch.int64)
        cell.scatter_(2, pick, -torch.ones_like(pick))
        cell = cell.view(hsy, wsx, sy, sx).transpose(1, 2).reshape(hsy * sy, wsx * sx)
        if hsy * sy < h or wsx * sx < w:
            full = torch.zeros(h, w, device=dev, dtype=torch.int64)
            full[:hsy * sy, :wsx * sx] = cell
            cell = full
        order = cell.reshape(1, -1, 1).argsort(dim=1)       # dst tokens (-1) first
        num_dst = hsy * wsx
        a_idx, b_idx = order[:, num_dst:, :], order[:, :num_dst, :]

        def split(x):
            C = x.shape[-1]
            return (torch.gather(x, 1, a_idx.expand(B, N - num_dst, C)),
                    torch.gather(x, 1, b_idx.expand(B, num_dst, C)))
        a, b = split(metric)
        r = min(a.shape[1], r)
        node_max, node_idx = ops.tome_match(a, b)     # fused cosine-similarity argmax (K30)
        edge = node_max.argsort(dim=-1, descending=True)[..., None]
        unm_idx, src_idx = edge[..., r:, :], edge[..., :r, :]
        dst_idx = torch.gather(node_idx[..., None], -2, src_idx)

    def merge(x, mode="mean"):
        src, dst = split(x)
        n, t1, c = src.shape
        unm = torch.gather(src, -2, unm_idx.expand(n, t1 - r, c))
        src = torch.gather(src, -2, src_idx.expand(n, r, c))
        dst = dst.scatter_reduce(-2, dst_idx.expand(n, r, c), src, reduce=mode)
        return torch.cat([unm, dst], dim=1)

    def unmerge(x):
        ul = unm_idx.shape[1]
        unm, dst = x[..., :ul, :], x[..., ul:, :]
        c = unm.shape[-1]
        src = torch.gather(dst, -2, dst_idx.expand(B, r, c))
        out = torch.zeros(B, N, c, device=x.device, dtype=x.dtype)
        out.scatter_(-2, b_idx.expand(B, num_dst, c), dst)
        a_exp = a_idx.expand(B, a_idx.shape[1], 1)
        out.scatter_(-2, torch.gather(a_exp, 1, unm_idx).expand(B, ul, c), unm)
        out.scatter_(-2, torch.gather(a_exp, 1, src_idx).expand(B, r, c), src)
        return out
    return merge, unmerge


def _tome_functions(x, ratio, original_shape):
    _, _, oh, ow = original_shape
    down = int(math.ceil(math.sqrt((oh * ow) // x.shape[1])))
    if down <= 1:
        w, h = int(math.ceil(ow / down)), int(math.ceil(oh / down))
        return bipartite_soft_matching_random2d(x, w, h, 2, 2, int(x.shape[1] * ratio))
    return (lambda y: y), (lambda y: y)


class TomePatchModel:
    @classmethod
    def INPUT_TYPES(s):
        return {"required": {"model": ("MODEL",),
                             "ratio": ("FLOAT", {"default": 0.3, "min": 0.0, "max": 1.0, "step": 0.01})}}
    RETURN_TYPES = ("MODEL",)
    FUNCTION = "patch"
    CATEGORY = "_for_testing"

    def patch(self, model, ratio):
        state = {"u": None}

        def tome_m(q, k, v, extra):
            mfn, state["u"] = _tome_functions(q, ratio, extra["original_shape"])
            return mfn(q), k, v

        def tome_u(n, extra):
            return state["u"](n)

        m = model.clone()
        m.set_model_attn1_patch(tome_m)
        m.set_model_attn1_output_patch(tome_u)
        return (m,)


NODE_CLASS_MAPPINGS = {
    "ModelSamplingDiscrete": ModelSamplingDiscrete, "ModelSamplingContinuousEDM": ModelSamplingContinuousEDM,
    "ModelSamplingStableCascade": ModelSamplingStableCascade, "RescaleCFG": RescaleCFG,
    "VideoLinearCFGGuidance": VideoLinearCFGGuidance, "VideoTriangleCFGGuidance": VideoTriangleCFGGuidance,
    "PerpNeg": PerpNeg, "SelfAttentionGuidance": SelfAttentionGuidance,
    "PerturbedAttentionGuidance": PerturbedAttentionGuidance, "FreeU": FreeU, "FreeU_V2": FreeU_V2,
    "PatchModelAddDownscale": PatchModelAddDownscale, "DifferentialDiffusion": DifferentialDiffusion,
    "HyperTile": HyperTile, "TomePatchModel": TomePatchModel,
}
NODE_DISPLAY_NAME_MAPPINGS = {"PatchModelAddDownscale": "PatchModelAddDownscale (Kohya Deep Shrink)",
                              "SelfAttentionGuidance": "Self-Attention Guidance",
                              "DifferentialDiffusion": "Differential Diffusion", "PerpNeg": "Perp-Neg (DEPRECATED by PerpNegGuider)"}
