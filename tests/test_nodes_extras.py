"""CPU unit tests for the extra node modules (reference: comfy_extras/*)."""
import math
import os

import pytest
import torch

from comfy_gen_server_amd.runtime import device as dm


@pytest.fixture(scope="module", autouse=True)
def _cpu():
    dm.set_cpu_mode(True)
    from comfy_gen_server_amd.graph import registry
    registry.init_nodes(custom_nodes=False)


def N(name):
    from comfy_gen_server_amd.graph import registry
    return registry.NODE_CLASS_MAPPINGS[name]()


def test_registry_has_extras():
    from comfy_gen_server_amd.graph import registry
    for n in ("SamplerCustomAdvanced", "KarrasScheduler", "LatentInterpolate", "RebatchLatents", "GrowMask",
              "PorterDuffImageComposite", "Canny", "Morphology", "ImageBlend", "AlignYourStepsScheduler"):
        assert n in registry.NODE_CLASS_MAPPINGS, n


def test_schedulers_and_sigma_ops():
    s = N("KarrasScheduler").get_sigmas(10, 14.6, 0.03, 7.0)[0]
    assert s.shape[0] == 11 and s[-1] == 0 and torch.all(s[:-1] > s[1:-1].min() - 1)
    a, b = N("SplitSigmas").get_sigmas(s, 4)
    assert torch.equal(torch.cat([a, b[1:]]), s)
    f = N("FlipSigmas").get_sigmas(s)[0]
    assert f[0] > 0 and f[-1] == s[0]
    ays = N("AlignYourStepsScheduler").get_sigmas("SDXL", 10, 1.0)[0]
    assert ays.shape[0] == 11 and ays[-1] == 0


def test_latent_ops():
    a = {"samples": torch.randn(2, 4, 8, 8)}
    b = {"samples": torch.randn(1, 4, 4, 4)}
    s = N("LatentAdd").op(a, b)[0]["samples"]
    assert s.shape == (2, 4, 8, 8)
    i = N("LatentInterpolate").op(a, a, 0.3)[0]["samples"]
    assert torch.allclose(i, a["samples"], atol=1e-5)
    bt = N("LatentBatch").batch(a, a)[0]
    assert bt["samples"].shape[0] == 4 and bt["batch_index"] == [0, 1, 0, 1]
    rb = N("RebatchLatents").rebatch([a, a, {"samples": torch.zeros(3, 4, 16, 16)}], [3])[0]
    assert [r["samples"].shape[0] for r in rb] == [3, 1, 3]


def test_mask_ops():
    m = torch.zeros(1, 9, 9)
    m[0, 4, 4] = 1.0
    g = N("GrowMask").expand_mask(m, 1, True)[0]
    assert g.sum() == 5            # cross footprint
    g2 = N("GrowMask").expand_mask(m, 1, False)[0]
    assert g2.sum() == 9
    assert N("GrowMask").expand_mask(g2, -1, False)[0].sum() == 1
    f = N("FeatherMask").feather(torch.ones(1, 4, 8), 0, 0, 4, 0)[0]
    assert f[0, 0, -1] == pytest.approx(0.25) and f[0, 0, 0] == 1.0
    c = N("MaskComposite").combine(torch.ones(1, 4, 4), torch.zeros(1, 2, 2), 1, 1, "multiply")[0]
    assert c.sum() == 12
    img = torch.rand(1, 8, 8, 3)
    d = {"samples": torch.zeros(1, 4, 8, 8)}
    out = N("LatentCompositeMasked").composite(d, {"samples": torch.ones(1, 4, 2, 2)}, 16, 8, False)[0]
    assert out["samples"].sum() == 16 and out["samples"][0, 0, 1, 2] == 1
    assert N("ImageCompositeMasked").composite(img, img, 0, 0, False)[0].shape == img.shape


def test_image_postprocessing():
    img = torch.rand(2, 16, 16, 3)
    assert N("ImageBlur").blur(img, 2, 1.0)[0].shape == img.shape
    const = torch.full((1, 8, 8, 3), 0.5)
    assert torch.allclose(N("ImageSharpen").sharpen(const, 1, 1.0, 1.0)[0], const, atol=1e-5)
    assert torch.allclose(N("ImageBlend").blend_images(img, img, 0.5, "normal")[0], img, atol=1e-6)
    q = N("ImageQuantize").quantize(img, 4, "bayer-4")[0]
    assert all(len(torch.unique(q[b].reshape(-1, 3), dim=0)) <= 4 for b in range(2))
    mp = N("ImageScaleToTotalPixels").upscale(img, "bilinear", 0.0625)[0]
    assert mp.shape[1] * mp.shape[2] == pytest.approx(0.0625 * 1024 * 1024, rel=0.05)
    rgb, a = N("SplitImageWithAlpha").split_image_with_alpha(torch.rand(1, 4, 4, 4))
    j = N("JoinImageWithAlpha").join_image_with_alpha(rgb, a)[0]
    assert j.shape[-1] == 4
    pd = N("PorterDuffImageComposite").composite(img, torch.ones(2, 16, 16), img * 0, torch.ones(2, 16, 16),
                                                 "SRC_OVER")
    assert torch.allclose(pd[0], img)


def test_morphology_and_canny():
    img = torch.zeros(1, 32, 32, 3)
    img[:, 8:24, 8:24, :] = 1.0
    d = N("Morphology").process(img, "dilate", 3)[0]
    assert d[0, 7, 7, 0] == 1 and d[0, 6, 6, 0] == 0
    e = N("Morphology").process(img, "erode", 3)[0]
    assert e[0, 8, 8, 0] == 0 and e[0, 9, 9, 0] == 1
    grad = N("Morphology").process(img, "gradient", 3)[0]
    assert grad[0, 16, 16, 0] == 0 and grad[0, 8, 16, 0] == 1
    edges = N("Canny").detect_edge(img, 0.2, 0.5)[0]
    assert edges[0, 16, 16, 0] == 0 and edges[0, 2, 2, 0] == 0
    assert edges[0, :, 7:9, 0].sum() > 8            # left border of the square is an edge


@pytest.fixture(scope="module")
def tiny():
    from comfy_gen_server_amd.tools.synth import build_pipeline
    patcher, clip, vae = build_pipeline("tiny", device=torch.device("cpu"), dtype=torch.float32, seed=0)
    pos = N("CLIPTextEncode").encode(clip, "a cat")[0]
    neg = N("CLIPTextEncode").encode(clip, "")[0]
    return patcher, clip, vae, pos, neg


def _sample(model, pos, neg, steps=2, sampler="euler", latent=None):
    latent = latent or {"samples": torch.zeros(2, 4, 16, 16)}
    return N("KSampler").sample(model, 1, steps, 5.0, sampler, "normal", pos, neg, latent, 1.0)[0]["samples"]


@pytest.mark.parametrize("patch", ["freeu", "freeu2", "rescale", "sag", "pag", "perpneg", "hypertile", "tome",
                                   "downscale", "msd_v", "msd_lcm_zsnr", "edm", "video_lin", "video_tri"])
def test_model_patches_run(tiny, patch):
    patcher, clip, vae, pos, neg = tiny
    base = _sample(patcher, pos, neg)
    if patch == "freeu":
        m = N("FreeU").patch(patcher, 1.1, 1.2, 0.9, 0.2)[0]
    elif patch == "freeu2":
        m = N("FreeU_V2").patch(patcher, 1.3, 1.4, 0.9, 0.2)[0]
    elif patch == "rescale":
        m = N("RescaleCFG").patch(patcher, 0.7)[0]
    elif patch == "sag":
        m = N("SelfAttentionGuidance").patch(patcher, 0.5, 2.0)[0]
    elif patch == "pag":
        m = N("PerturbedAttentionGuidance").patch(patcher, 3.0)[0]
    elif patch == "perpneg":
        m = N("PerpNeg").patch(patcher, neg, 1.0)[0]
    elif patch == "hypertile":
        m = N("HyperTile").patch(patcher, 64, 2, 0, False)[0]
    elif patch == "tome":
        m = N("TomePatchModel").patch(patcher, 0.3)[0]
    elif patch == "downscale":
        m = N("PatchModelAddDownscale").patch(patcher, 1, 2.0, 0.0, 1.0, True, "bicubic", "bicubic")[0]
    elif patch == "msd_v":
        m = N("ModelSamplingDiscrete").patch(patcher, "v_prediction", False)[0]
    elif patch == "msd_lcm_zsnr":
        m = N("ModelSamplingDiscrete").patch(patcher, "lcm", True)[0]
    elif patch == "edm":
        m = N("ModelSamplingContinuousEDM").patch(patcher, "v_prediction", 120.0, 0.002)[0]
    elif patch == "video_lin":
        m = N("VideoLinearCFGGuidance").patch(patcher, 1.0)[0]
    else:
        m = N("VideoTriangleCFGGuidance").patch(patcher, 1.0)[0]
    out = _sample(m, pos, neg)
    assert out.shape == base.shape and torch.isfinite(out).all()
    # the base patcher is untouched (clone semantics)
    assert torch.allclose(_sample(patcher, pos, neg), base)


def test_differential_diffusion_and_custom_sampler(tiny):
    patcher, clip, vae, pos, neg = tiny
    m = N("DifferentialDiffusion").apply(patcher)[0]
    lat = {"samples": torch.zeros(1, 4, 16, 16), "noise_mask": torch.linspace(0, 1, 256).reshape(1, 16, 16)}
    out = N("KSampler").sample(m, 1, 3, 5.0, "euler", "normal", pos, neg, lat, 1.0)[0]["samples"]
    assert torch.isfinite(out).all()
    sig = N("BasicScheduler").get_sigmas(patcher, "karras", 3, 1.0)[0]
    for guider in (N("CFGGuider").get_guider(patcher, pos, neg, 5.0)[0],
                   N("DualCFGGuider").get_guider(patcher, pos, pos, neg, 5.0, 3.0)[0],
                   N("BasicGuider").get_guider(patcher, pos)[0],
                   N("PerpNegGuider").get_guider(patcher, pos, neg, neg, 5.0, 1.0)[0]):
        out, den = N("SamplerCustomAdvanced").sample(N("RandomNoise").get_noise(3)[0], guider,
                                                     N("KSamplerSelect").get_sampler("dpmpp_2m")[0], sig,
                                                     {"samples": torch.zeros(1, 4, 16, 16)})
        assert out["samples"].shape == (1, 4, 16, 16) and torch.isfinite(den["samples"]).all()
    o1, _ = N("SamplerCustom").sample(patcher, True, 5, 5.0, pos, neg,
                                      N("SamplerEulerAncestral").get_sampler(1.0, 1.0)[0], sig,
                                      {"samples": torch.zeros(1, 4, 16, 16)})
    noisy = N("AddNoise").add_noise(patcher, N("RandomNoise").get_noise(3)[0], sig, o1)[0]
    assert noisy["samples"].shape == o1["samples"].shape


def test_clip_vision_and_image_conditioning(tiny, tmp_path):
    from comfy_gen_server_amd.models.layers import init_random_
    from comfy_gen_server_amd.runtime import clip_vision as CV
    patcher, clip, vae, pos, neg = tiny
    cfg = dict(hidden_size=64, intermediate_size=128, num_attention_heads=2, num_hidden_layers=3,
               hidden_act="gelu", projection_dim=32, patch_size=14, image_size=224)
    cv = CV.ClipVisionModel(cfg)
    init_random_(cv.model, seed=1)
    img = torch.rand(1, 300, 200, 3)
    out = cv.encode_image(img)
    assert out.image_embeds.shape == (1, 32) and out.last_hidden_state.shape == (1, 257, 64)
    assert out.penultimate_hidden_states.shape == (1, 257, 64)
    px = CV.clip_preprocess(img)
    assert px.shape == (1, 3, 224, 224)
    # OpenCLIP-layout round trip through the converter (H/G/L detection needs full depth; check keys)
    sd = {f"visual.transformer.resblocks.0.attn.in_proj_weight": torch.zeros(192, 64),
          "visual.conv1.weight": torch.zeros(64, 3, 14, 14), "visual.proj": torch.zeros(64, 32)}
    conv = CV.convert_to_transformers(dict(sd), "visual.")
    assert "vision_model.encoder.layers.0.self_attn.q_proj.weight" in conv
    assert conv["visual_projection.weight"].shape == (32, 64)
    p2, n2, lat = N("StableZero123_Conditioning").encode(cv, img, vae, 64, 64, 2, 10.0, 30.0)
    assert p2[0][0].shape == (1, 1, 36) and lat["samples"].shape == (2, 4, 8, 8)
    p3, _, lat3 = N("SV3D_Conditioning").encode(cv, img, vae, 64, 64, 5, 10.0)
    assert len(p3[0][1]["azimuth"]) == 5 and lat3["samples"].shape[0] == 5
    p4, _, lat4 = N("SVD_img2vid_Conditioning").encode(cv, img, vae, 64, 64, 3, 127, 6, 0.0)
    assert p4[0][1]["motion_bucket_id"] == 127 and lat4["samples"].shape == (3, 4, 8, 8)
    ip, _, il = N("InstructPixToPixConditioning").encode(pos, neg, torch.rand(1, 67, 65, 3), vae)
    assert ip[0][1]["concat_latent_image"].shape[-2:] == (8, 8)
    sx = N("CLIPTextEncodeSDXLRefiner").encode(clip, 6.0, 1024, 1024, "x")[0]
    assert sx[0][1]["aesthetic_score"] == 6.0


def test_merge_and_save_roundtrip(tiny, tmp_path):
    import os
    from comfy_gen_server_amd.tools.synth import build_pipeline
    from comfy_gen_server_amd.utils import folder_paths
    patcher, clip, vae, pos, neg = tiny
    other, _, _ = build_pipeline("tiny", device=torch.device("cpu"), dtype=torch.float32, seed=7, with_clip=False,
                                 with_vae=False)
    ref1 = _sample(patcher, pos, neg)
    ref2 = _sample(other, pos, neg)
    m1 = N("ModelMergeSimple").merge(patcher, other, 1.0)[0]       # ratio 1.0 keeps model1
    assert torch.allclose(_sample(m1, pos, neg), ref1, atol=1e-5)
    m0 = N("ModelMergeSimple").merge(patcher, other, 0.0)[0]       # ratio 0.0 -> model2 weights
    assert torch.allclose(_sample(m0, pos, neg), ref2, atol=1e-4)
    mb = N("ModelMergeBlocks").merge(patcher, other, input=1.0, middle=1.0, out=1.0)[0]
    assert torch.allclose(_sample(mb, pos, neg), ref1, atol=1e-5)
    folder_paths.set_output_directory(str(tmp_path))
    N("CheckpointSave").save(patcher, clip, vae, "checkpoints/rt")
    files = os.listdir(tmp_path / "checkpoints")
    assert len(files) == 1 and files[0].endswith(".safetensors")
    from comfy_gen_server_amd.runtime import sd as sdl
    mp, cl, va, _ = sdl.load_checkpoint_guess_config(str(tmp_path / "checkpoints" / files[0]))
    assert torch.allclose(_sample(mp, pos, neg), ref1, atol=1e-4)
    N("VAESave").save(vae, "vae/v")
    N("CLIPSave").save(clip, "clip/c")
    assert os.listdir(tmp_path / "vae") and os.listdir(tmp_path / "clip")


def test_controlnet_roundtrip(tiny, tmp_path):
    """Random tiny ControlNet: save -> ControlNetLoader -> ControlNetApply(Advanced) -> KSampler;
    zero convs at zero reproduce the plain model, non-zero changes the result; strength 0 == off."""
    import copy
    from safetensors.torch import save_file
    from comfy_gen_server_amd.models.cldm import ControlNet as CN
    from comfy_gen_server_amd.models.layers import init_random_
    from comfy_gen_server_amd.tools.synth import TINY_UNET
    from comfy_gen_server_amd.utils import folder_paths
    patcher, clip, vae, pos, neg = tiny
    cfg = copy.deepcopy(TINY_UNET)
    cfg.update(num_heads=2, num_head_channels=-1)
    cn = CN(hint_channels=3, **cfg)
    init_random_(cn, seed=3)
    sd = {k: v.contiguous() for k, v in cn.state_dict().items()}
    os.makedirs(tmp_path / "controlnet", exist_ok=True)
    save_file(sd, str(tmp_path / "controlnet" / "cn.safetensors"))
    zero = {k: (torch.zeros_like(v) if ("zero_convs" in k or "middle_block_out" in k) else v) for k, v in sd.items()}
    save_file(zero, str(tmp_path / "controlnet" / "cn_zero.safetensors"))
    folder_paths.add_model_folder_path("controlnet", str(tmp_path / "controlnet"))
    hint = torch.rand(1, 128, 128, 3)
    base = _sample(patcher, pos, neg)
    net0 = N("ControlNetLoader").load_controlnet("cn_zero.safetensors")[0]
    p0 = N("ControlNetApply").apply_controlnet(pos, net0, hint, 1.0)[0]
    assert torch.allclose(_sample(patcher, p0, neg), base, atol=1e-5)
    net = N("ControlNetLoader").load_controlnet("cn.safetensors")[0]
    p1, n1 = N("ControlNetApplyAdvanced").apply_controlnet(pos, neg, net, hint, 1.0, 0.0, 1.0)
    out = _sample(patcher, p1, n1)
    assert torch.isfinite(out).all() and not torch.allclose(out, base, atol=1e-4)
    ps, ns = N("ControlNetApplyAdvanced").apply_controlnet(pos, neg, net, hint, 0.0, 0.0, 1.0)
    assert torch.allclose(_sample(patcher, ps, ns), base, atol=1e-5)
    # chained nets + percent window that excludes every step
    p2, n2 = N("ControlNetApplyAdvanced").apply_controlnet(p1, n1, net, hint, 0.5, 0.0, 1.0)
    assert torch.isfinite(_sample(patcher, p2, n2)).all()
    pw, nw = N("ControlNetApplyAdvanced").apply_controlnet(pos, neg, net, hint, 1.0, 0.99, 1.0)
    d = (_sample(patcher, pw, nw, steps=2) - base).abs().max()   # only batching-order fp32 noise
    assert d < 1e-4 * base.abs().max()


def test_t2i_adapter_shapes():
    from comfy_gen_server_amd.models.t2i_adapter import Adapter, Adapter_light, StyleAdapter
    a = Adapter(channels=[32, 64, 128, 128], nums_rb=2, cin=192, ksize=1, sk=True, use_conv=False, xl=False)
    f = a(torch.rand(1, 3, 128, 128))
    assert len(f) == 12 and f[2].shape == (1, 32, 16, 16) and f[11].shape == (1, 128, 2, 2)
    ax = Adapter(channels=[32, 64, 128, 128], nums_rb=2, cin=768, ksize=1, sk=True, use_conv=False, xl=True)
    fx = ax(torch.rand(1, 3, 128, 128))
    assert [i for i, t in enumerate(fx) if t is not None] == [3, 5, 8, 10]
    al = Adapter_light(channels=[32, 64, 128, 128], nums_rb=1, cin=192)
    assert al(torch.rand(1, 3, 64, 64))[-1].shape == (1, 128, 1, 1)
    st = StyleAdapter(width=64, context_dim=32, num_head=4, n_layes=2, num_token=3)
    assert st(torch.rand(2, 5, 64)).shape == (2, 3, 32)


def test_taesd_and_gligen(tiny):
    from comfy_gen_server_amd.models.taesd import TAESD
    from comfy_gen_server_amd.models.gligen import FourierEmbedder, gligen_from_state_dict, PositionNet, \
        GatedSelfAttentionDense
    from comfy_gen_server_amd.models.layers import init_random_
    t = TAESD()
    init_random_(t, seed=0)
    z = t.encode(torch.rand(1, 3, 64, 64) * 2 - 1)
    assert z.shape == (1, 4, 8, 8)
    assert t.decode(z).shape == (1, 3, 64, 64)
    fe = FourierEmbedder(num_freqs=3)
    x = torch.rand(2, 5, 4)
    ref = torch.cat([torch.cat([torch.sin(f * x), torch.cos(f * x)], -1) for f in fe.freq_bands], -1)
    assert torch.allclose(fe(x), ref, atol=1e-6)
    # GLIGEN on the tiny UNet: one gated block per transformer block (tiny has 4+1 with context 64)
    patcher, clip, vae, pos, neg = tiny
    sd = {}
    blocks = [("input_blocks", 1, 32), ("input_blocks", 3, 64), ("middle_block", 1, 64), ("output_blocks", 0, 64),
              ("output_blocks", 1, 64), ("output_blocks", 2, 32), ("output_blocks", 3, 32)]
    for part, b, dim in blocks:
        g = GatedSelfAttentionDense(dim, 64, 2, dim // 2)
        init_random_(g, seed=b)
        for k, v in g.state_dict().items():
            sd[f"model.diffusion_model.{part}.{b}.1.transformer_blocks.0.fuser.{k}"] = v
    pn = PositionNet(64, 64)
    init_random_(pn, seed=9)
    for k, v in pn.state_dict().items():
        sd[f"position_net.{k}"] = v
    gl = gligen_from_state_dict(sd)
    from comfy_gen_server_amd.runtime.patcher import ModelPatcher
    gp = ModelPatcher(gl, load_device=torch.device("cpu"), offload_device=torch.device("cpu"))
    cond = N("GLIGENTextBoxApply").append(pos, clip, gp, "a dog", 32, 32, 0, 0)[0]
    assert cond[0][1]["gligen"][0] == "position"
    out = _sample(patcher, cond, neg)
    assert torch.isfinite(out).all()
