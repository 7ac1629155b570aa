"""Upscale-model loading + tiled upscaling (parity target: comfy_extras/nodes_upscale_model.py and the
chaiNNer RRDB / SRVGG architectures): random ESRGAN checkpoints in old- and new-arch key layouts and a
Real-ESRGAN compact net load, report the right scale, and match an independent NCHW forward."""
import os

import pytest
import torch
import torch.nn.functional as F

from comfy_gen_server_amd.models import upscalers


def _esrgan_new_arch(nf=16, nb=2, gc=8, scale=4, in_nc=3, out_nc=3, seed=0):
    g = torch.Generator().manual_seed(seed)
    r = lambda *s: torch.randn(*s, generator=g) * 0.05  # noqa: E731
    sd = {"conv_first.weight": r(nf, in_nc, 3, 3), "conv_first.bias": r(nf)}
    for b in range(nb):
        for j in range(1, 4):
            for c in range(1, 6):
                cin = nf + (c - 1) * gc
                cout = nf if c == 5 else gc
                sd[f"body.{b}.rdb{j}.conv{c}.weight"] = r(cout, cin, 3, 3)
                sd[f"body.{b}.rdb{j}.conv{c}.bias"] = r(cout)
    sd["conv_body.weight"], sd["conv_body.bias"] = r(nf, nf, 3, 3), r(nf)
    for u in range(1, {4: 3, 2: 2, 1: 1}[scale]):
        sd[f"conv_up{u}.weight"], sd[f"conv_up{u}.bias"] = r(nf, nf, 3, 3), r(nf)
    sd["conv_hr.weight"], sd["conv_hr.bias"] = r(nf, nf, 3, 3), r(nf)
    sd["conv_last.weight"], sd["conv_last.bias"] = r(out_nc, nf, 3, 3), r(out_nc)
    return sd


def _esrgan_ref(sd, x, nb):
    lr = lambda t: F.leaky_relu(t, 0.2)  # noqa: E731
    c = lambda t, n: F.conv2d(t, sd[f"{n}.weight"], sd[f"{n}.bias"], padding=1)  # noqa: E731
    fea = c(x, "conv_first")
    h = fea
    for b in range(nb):
        inp = h
        for j in range(1, 4):
            xs = [h]
            for k in range(1, 5):
                xs.append(lr(c(torch.cat(xs, 1), f"body.{b}.rdb{j}.conv{k}")))
            h = c(torch.cat(xs, 1), f"body.{b}.rdb{j}.conv5") * 0.2 + h
        h = h * 0.2 + inp
    h = c(h, "conv_body") + fea
    u = 1
    while f"conv_up{u}.weight" in sd:
        h = lr(c(F.interpolate(h, scale_factor=2, mode="nearest"), f"conv_up{u}"))
        u += 1
    return c(lr(c(h, "conv_hr")), "conv_last")


def _to_old_arch(sd):
    out = {}
    for k, v in sd.items():
        if k.startswith("body."):
            p = k.split(".")
            out[f"model.1.sub.{p[1]}.RDB{p[2][3:]}.{p[3]}.0.{p[4]}"] = v
    m = {"conv_first": "model.0", "conv_body": "model.1.sub.2", "conv_up1": "model.3", "conv_up2": "model.6",
         "conv_hr": "model.8", "conv_last": "model.10"}
    for a, b in m.items():
        for kind in ("weight", "bias"):
            out[f"{b}.{kind}"] = sd[f"{a}.{kind}"]
    return out


def test_esrgan_new_and_old_arch_match_reference():
    sd = _esrgan_new_arch()
    x = torch.rand(1, 3, 12, 10)
    ref = _esrgan_ref(sd, x, 2)
    for state in (sd, _to_old_arch(sd)):
        m = upscalers.load_state_dict(dict(state)).eval()
        assert isinstance(m, upscalers.RRDBNet) and m.scale == 4 and m.num_blocks == 2
        with torch.no_grad():
            y = m(x)
        assert y.shape == (1, 3, 48, 40)
        assert torch.allclose(y, ref, atol=1e-5)


def test_esrgan_pixel_unshuffle_variant_and_srvgg():
    sd = _esrgan_new_arch(in_nc=12, scale=4)       # Real-ESRGAN x2plus layout
    m = upscalers.load_state_dict({"params_ema": sd})
    assert m.shuffle_factor == 2 and m.scale == 2
    with torch.no_grad():
        assert m(torch.rand(1, 3, 9, 7)).shape == (1, 3, 18, 14)
    g = torch.Generator().manual_seed(1)
    nf, ncv, s = 16, 3, 4
    vsd = {"body.0.weight": torch.randn(nf, 3, 3, 3, generator=g) * 0.1, "body.0.bias": torch.zeros(nf),
           "body.1.weight": torch.full((nf,), 0.25)}
    i = 2
    for _ in range(ncv):
        vsd[f"body.{i}.weight"] = torch.randn(nf, nf, 3, 3, generator=g) * 0.1
        vsd[f"body.{i}.bias"] = torch.zeros(nf)
        vsd[f"body.{i + 1}.weight"] = torch.full((nf,), 0.25)
        i += 2
    vsd[f"body.{i}.weight"] = torch.randn(3 * s * s, nf, 3, 3, generator=g) * 0.1
    vsd[f"body.{i}.bias"] = torch.zeros(3 * s * s)
    v = upscalers.load_state_dict(vsd)
    assert isinstance(v, upscalers.SRVGGNetCompact) and v.scale == 4 and v.num_conv == ncv
    x = torch.rand(1, 3, 8, 8)
    h = x
    for k in range(0, i, 2):
        h = F.prelu(F.conv2d(h, vsd[f"body.{k}.weight"], vsd[f"body.{k}.bias"], padding=1), vsd[f"body.{k + 1}.weight"])
    h = F.conv2d(h, vsd[f"body.{i}.weight"], vsd[f"body.{i}.bias"], padding=1)
    ref = F.pixel_shuffle(h, s) + F.interpolate(x, scale_factor=s, mode="nearest")
    with torch.no_grad():
        assert torch.allclose(v(x), ref, atol=1e-5)
    with pytest.raises(upscalers.UnsupportedModel):     # recognised family, malformed file
        upscalers.load_state_dict({"layers.0.residual_group.blocks.0.norm1.weight": torch.zeros(1)})
    with pytest.raises(upscalers.UnsupportedModel, match="DAT"):
        upscalers.load_state_dict({"layers.0.blocks.2.attn.attn_mask_0": torch.zeros(1)})


def test_upscale_nodes_tiled(tmp_path):
    from safetensors.torch import save_file
    from comfy_gen_server_amd.graph import registry
    from comfy_gen_server_amd.utils import folder_paths
    registry.init_nodes(custom_nodes=False)
    N = registry.NODE_CLASS_MAPPINGS
    sd = _esrgan_new_arch(scale=2, seed=3)
    os.makedirs(tmp_path / "upscale_models")
    save_file(sd, str(tmp_path / "upscale_models" / "tiny_x2.safetensors"))
    folder_paths.add_model_folder_path("upscale_models", str(tmp_path / "upscale_models"))
    model = N["UpscaleModelLoader"]().load_model("tiny_x2.safetensors")[0]
    img = torch.rand(1, 40, 36, 3)
    out = N["ImageUpscaleWithModel"]().upscale(model, img)[0]
    assert out.shape == (1, 80, 72, 3)
    with torch.no_grad():
        ref = _esrgan_ref(sd, img.movedim(-1, 1), 2).clamp(0, 1).movedim(1, -1)
    assert (out - ref).abs().max() < 1e-4      # single tile (< 512 px): exact


@pytest.mark.gpu
def test_upscale_esrgan_gpu(cuda):
    """Full-width ESRGAN (nf 64, gc 32) on the device through the bf16 NHWC conv kernels."""
    from comfy_gen_server_amd import ops
    sd = _esrgan_new_arch(nf=64, nb=1, gc=32, scale=4, seed=5)
    m = upscalers.load_state_dict(dict(sd)).eval().to(device=cuda, dtype=torch.bfloat16)
    x = torch.rand(1, 3, 64, 48)
    ops.reset_stats()
    with torch.no_grad():
        y = m(x.to(cuda, torch.bfloat16)).float().cpu()
        ref = _esrgan_ref(sd, x, 1)
    assert ops.stats().get(("conv", "hip"), 0) > 10
    assert ((y - ref).norm() / ref.norm()).item() < 3e-2


def _swin_seed(kind, dim=48, ws=8, nf=32):
    """Shape-defining keys for the Swin family; the rest is random-initialised by the test."""
    Z = torch.zeros
    b0 = "layers.0.residual_group.blocks.0."
    sd = {"conv_first.weight": Z(dim, 3, 3, 3), b0 + "mlp.fc1.bias": Z(dim * 2),
          "conv_before_upsample.0.weight": Z(nf, dim, 3, 3), "upsample.0.weight": Z(4 * nf, nf, 3, 3),
          "conv_last.weight": Z(3, nf, 3, 3), b0 + "attn.relative_position_index": Z(ws * ws, ws * ws)}
    for i in range(2):
        for j in range(2):
            sd[f"layers.{i}.residual_group.blocks.{j}.norm1.weight"] = Z(dim)
            if kind == "hat":
                sd[f"layers.{i}.residual_group.blocks.{j}.conv_block.cab.0.weight"] = Z(dim // 3, dim, 3, 3)
                sd[f"layers.{i}.residual_group.blocks.{j}.conv_block.cab.3.attention.1.weight"] = Z(dim // 16, dim, 1, 1)
    if kind == "swin2sr":
        sd["patch_embed.proj.weight"] = Z(dim, dim, 1, 1)
        sd[b0 + "attn.logit_scale"] = Z(3, 1, 1)
    else:
        sd[b0 + "attn.relative_position_bias_table"] = Z((2 * ws - 1) ** 2, 3)
    if kind == "hat":
        sd["relative_position_index_SA"] = Z(ws * ws, ws * ws)
        sd["layers.0.residual_group.overlap_attn.relative_position_bias_table"] = Z((ws + 12 - 1) ** 2, 3)
        sd["layers.0.conv.weight"] = Z(dim, dim, 3, 3)
    return sd


def _random_swin(kind):
    from comfy_gen_server_amd.models import swin_sr
    from comfy_gen_server_amd.models.layers import init_random_
    if kind == "dat":
        from comfy_gen_server_amd.models.dat import DAT
        Z = torch.zeros
        seed = {"conv_first.weight": Z(64, 3, 3, 3), "conv_before_upsample.0.weight": Z(64, 64, 3, 3),
                "upsample.0.weight": Z(256, 64, 3, 3), "conv_last.weight": Z(3, 64, 3, 3),
                "layers.0.blocks.1.attn.temperature": Z(4, 1, 1), "layers.0.blocks.0.ffn.fc1.weight": Z(128, 64),
                "layers.0.blocks.2.attn.attn_mask_0": Z(1)}
        seed.update({f"layers.{i}.blocks.{j}.norm1.weight": Z(64) for i in range(2) for j in range(4)})
        m = DAT(seed, strict=False)
        init_random_(m, seed=4)
        sd = {k: v.clone() for k, v in m.state_dict().items()}
        sd["layers.0.blocks.2.attn.attn_mask_0"] = Z(1)        # file-only buffer the loader sniffs
        return sd
    if kind in ("scunet", "omnisr"):
        if kind == "scunet":
            m = swin_sr.SCUNet({}, strict=False)
        else:
            from comfy_gen_server_amd.models.omnisr import OmniSR
            m = OmniSR({"input.weight": torch.zeros(64, 3, 3, 3), "up.0.weight": torch.zeros(12, 64, 3, 3),
                        "residual_layer.1.residual_layer.0.layer.0.fn.0.weight": torch.zeros(64, 64, 1, 1)},
                       strict=False)
        init_random_(m, seed=4)
        return {k: v.clone() for k, v in m.state_dict().items()}
    seed = _swin_seed(kind)
    m = swin_sr.HAT(seed, strict=False) if kind == "hat" else swin_sr.SwinIR(seed, v2=kind == "swin2sr", strict=False)
    init_random_(m, seed=4)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    sd.update({k: v for k, v in seed.items() if "position_index" in k})   # file-only index buffers
    return sd


@pytest.mark.parametrize("kind", ["swinir", "swin2sr", "hat", "scunet", "omnisr", "dat"])
def test_swin_family_dispatch_and_forward(kind):
    sd = _random_swin(kind)
    m = upscalers.load_state_dict(sd)
    s = 1 if kind == "scunet" else 2
    assert m.model_arch == {"swinir": "SwinIR", "swin2sr": "Swin2SR", "hat": "HAT", "scunet": "SCUNet",
                            "omnisr": "OmniSR", "dat": "DAT"}[kind]
    assert m.scale == s
    with torch.no_grad():
        y = m(torch.rand(1, 3, 17, 16))
    assert y.shape == (1, 3, 17 * s, 16 * s) and torch.isfinite(y).all()


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["swinir", "swin2sr", "hat", "scunet", "omnisr", "dat"])
def test_swin_family_gpu(cuda, kind):
    """Swin-family upscalers in bf16 on the device (HIP GEMMs for qkv/proj/MLP, MFMA convs) vs fp32 CPU."""
    from comfy_gen_server_amd import ops
    sd = _random_swin(kind)
    m = upscalers.load_state_dict(sd)
    x = torch.rand(1, 3, 40, 32)
    with torch.no_grad():
        ref = m(x)
        g = m.to(device=cuda, dtype=torch.bfloat16)
        ops.reset_stats()
        y = g(x.to(cuda, torch.bfloat16)).float().cpu()
    assert ops.stats().get(("gemm", "hip"), 0) + ops.stats().get(("gemm", "lib"), 0) > 0
    assert ops.stats().get(("attention", "hip"), 0) > 0          # window attention on the flash kernel
    assert ((y - ref).norm() / ref.norm()).item() < 3e-2


def _random_lama():
    from comfy_gen_server_amd.models.lama import LaMa
    from comfy_gen_server_amd.models.layers import init_random_
    m = LaMa({}, strict=False)
    init_random_(m, seed=2)
    with torch.no_grad():
        for k, v in m.state_dict().items():
            if "running_var" in k:
                v.abs_().add_(0.5)
    return {k.replace("model.model", "generator.model"): v.clone() for k, v in m.state_dict().items()}


def test_lama_dispatch_keeps_unmasked_pixels():
    m = upscalers.load_state_dict(_random_lama())
    assert m.model_arch == "LaMa" and m.scale == 1
    img = torch.rand(1, 3, 32, 40)
    mask = torch.zeros(1, 1, 32, 40)
    mask[..., 8:20, 10:30] = 1
    with torch.no_grad():
        y = m(img, mask)
    assert y.shape == img.shape
    assert torch.equal(y[..., :8, :], img[..., :8, :])          # outside the hole: untouched


@pytest.mark.gpu
def test_lama_gpu(cuda):
    """FFC generator in bf16 on the device (spectral path in fp32 via rocFFT) vs fp32 CPU."""
    m = upscalers.load_state_dict(_random_lama())
    img = torch.rand(1, 3, 64, 64)
    mask = (torch.rand(1, 1, 64, 64) > 0.5).float()
    with torch.no_grad():
        ref = m(img, mask)
        g = m.to(device=cuda, dtype=torch.bfloat16)
        y = g(img.to(cuda, torch.bfloat16), mask.to(cuda, torch.bfloat16)).float().cpu()
    assert ((y - ref).norm() / ref.norm()).item() < 3e-2


def _random_gfpgan():
    from comfy_gen_server_amd.models.face import GFPGANv1Clean
    from comfy_gen_server_amd.models.layers import init_random_
    m = GFPGANv1Clean({}, strict=False)
    init_random_(m, seed=3, std_scale=0.5)
    return {k: v.clone() for k, v in m.state_dict().items()}


def test_gfpgan_dispatch_and_activation_modulation():
    """Activation-side modulation == the per-sample modulated-weight grouped conv (batch of 2)."""
    from comfy_gen_server_amd.models.face import ModulatedConv2d
    m = upscalers.load_state_dict(_random_gfpgan())
    assert m.model_arch == "GFPGAN" and m.scale == 8
    mc = ModulatedConv2d(16, 8, 3, 12, demodulate=True, sample_mode="upsample")
    torch.nn.init.normal_(mc.modulation.weight)
    torch.nn.init.normal_(mc.modulation.bias)
    x, st = torch.randn(2, 16, 5, 6), torch.randn(2, 12)
    s = F.linear(st, mc.modulation.weight, mc.modulation.bias).view(2, 1, 16, 1, 1)
    w = mc.weight * s
    w = w * torch.rsqrt(w.pow(2).sum([2, 3, 4]) + 1e-8).view(2, 8, 1, 1, 1)
    xu = F.interpolate(x, scale_factor=2, mode="bilinear", align_corners=False)
    ref = F.conv2d(xu.reshape(1, 32, 10, 12), w.view(16, 16, 3, 3), padding=1, groups=2).view(2, 8, 10, 12)
    with torch.no_grad():
        assert torch.allclose(mc(x, st), ref, atol=1e-4)


@pytest.mark.gpu
def test_gfpgan_gpu(cuda):
    m = upscalers.load_state_dict(_random_gfpgan())
    x = torch.rand(1, 3, 512, 512) * 2 - 1
    with torch.no_grad():
        ref, _ = m(x, randomize_noise=False)
        g = m.to(device=cuda, dtype=torch.bfloat16)
        y, _ = g(x.to(cuda, torch.bfloat16), randomize_noise=False)
    y = y.float().cpu()
    assert ((y - ref).norm() / ref.norm()).item() < 3e-2


def _random_face(kind):
    from comfy_gen_server_amd.models import face
    from comfy_gen_server_amd.models.layers import init_random_
    m = face.RestoreFormer({}, strict=False) if kind == "restoreformer" else face.CodeFormer({}, strict=False)
    init_random_(m, seed=5, std_scale=0.5)
    return {k: v.clone() for k, v in m.state_dict().items()}


@pytest.mark.parametrize("kind", ["restoreformer", "codeformer"])
def test_face_vq_dispatch(kind):
    m = upscalers.load_state_dict(_random_face(kind))
    assert m.model_arch == {"restoreformer": "RestoreFormer", "codeformer": "CodeFormer"}[kind] and m.scale == 8


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["restoreformer", "codeformer"])
def test_face_vq_gpu(cuda, kind):
    """VQ face restorers in bf16 on the device (multi-head / wide-head HIP attention at 16x16)."""
    from comfy_gen_server_amd import ops
    m = upscalers.load_state_dict(_random_face(kind))
    x = torch.rand(1, 3, 512, 512) * 2 - 1
    with torch.no_grad():
        g = m.to(device=cuda, dtype=torch.bfloat16)
        ops.reset_stats()
        y, _ = g(x.to(cuda, torch.bfloat16))
    assert ops.stats().get(("attention", "hip"), 0) > 0
    y = y.float().cpu()
    assert y.shape == (1, 3, 512, 512) and torch.isfinite(y).all()
