"""SVD / SV3D / Stable-Zero123 families: state-dict detection from key names and shapes (meta
tensors, full-size configs) and a tiny video UNet sampling step through the model wrapper."""
import pytest
import torch

from comfy_gen_server_amd.models.unet import UNetModel
from comfy_gen_server_amd.runtime import detection, families, model_base

SVD_CFG = dict(in_channels=8, out_channels=4, model_channels=320, num_res_blocks=[2, 2, 2, 2],
               channel_mult=[1, 2, 4, 4], transformer_depth=[1, 1, 1, 1, 1, 1, 0, 0],
               transformer_depth_output=[1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0], transformer_depth_middle=1,
               num_heads=-1, num_head_channels=64, use_linear_in_transformer=True, context_dim=1024,
               num_classes="sequential", use_temporal_resblock=True, use_temporal_attention=True,
               extra_ff_mix_layer=True, use_spatial_context=True, merge_strategy="learned_with_images",
               merge_factor=0.0, video_kernel_size=[3, 1, 1])


def _meta_sd(cfg, prefix="model.diffusion_model."):
    with torch.device("meta"):
        m = UNetModel(**cfg)
    return {prefix + k: v for k, v in m.state_dict().items()}


@pytest.mark.parametrize("adm,cls", [(768, families.SVD_img2vid), (256, families.SV3D_u), (1280, families.SV3D_p)])
def test_detect_video_families(adm, cls):
    sd = _meta_sd(dict(SVD_CFG, adm_in_channels=adm))
    mc = detection.model_config_from_unet(sd, "model.diffusion_model.")
    assert type(mc) is cls
    cfg = mc.unet_config
    assert cfg["use_temporal_resblock"] and cfg["use_temporal_attention"] and cfg["video_kernel_size"] == [3, 1, 1]
    assert mc.model_type(sd) == model_base.ModelType.V_PREDICTION_EDM


def test_detect_zero123():
    cfg = dict(in_channels=8, out_channels=4, model_channels=320, num_res_blocks=[2, 2, 2, 2],
               channel_mult=[1, 2, 4, 4], transformer_depth=[1, 1, 1, 1, 1, 1, 0, 0],
               transformer_depth_output=[1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0], transformer_depth_middle=1,
               num_heads=8, use_linear_in_transformer=False, context_dim=768)
    sd = _meta_sd(cfg)
    sd["cc_projection.weight"] = torch.empty(768, 772, device="meta")
    sd["cc_projection.bias"] = torch.empty(768, device="meta")
    mc = detection.model_config_from_unet(sd, "model.diffusion_model.")
    assert type(mc) is families.Stable_Zero123
    with torch.device("meta"):
        model = mc.get_model(sd, "model.diffusion_model.", device=torch.device("meta"))
    assert isinstance(model, model_base.Stable_Zero123)
    assert tuple(model.cc_projection.weight.shape) == (768, 772)


def test_svd_model_extra_conds_and_step():
    """Tiny SVD-shaped model: extra_conds produce y / c_concat / c_crossattn / num_video_frames and
    apply_model runs the video UNet over 2 videos x 3 frames."""
    small = dict(SVD_CFG, model_channels=64, num_res_blocks=[1, 1], channel_mult=[1, 2], transformer_depth=[1, 1],
                 transformer_depth_output=[1, 1, 1, 1], num_head_channels=16, context_dim=64, adm_in_channels=768)
    mc = families.SVD_img2vid(small)
    mc.set_inference_dtype(torch.float32)
    model = mc.get_model({})
    from comfy_gen_server_amd.models.layers import init_random_
    init_random_(model.diffusion_model, seed=0)
    noise = torch.randn(3, 4, 8, 8)
    conds = model.extra_conds(noise=noise, device="cpu", cross_attn=torch.randn(1, 1, 64),
                              concat_latent_image=torch.randn(1, 4, 8, 8), fps=7, motion_bucket_id=100)
    assert conds["num_video_frames"].cond == 3 and conds["y"].cond.shape == (1, 768)
    b = 2 * 3                                   # cond + uncond batched, 3 frames each
    x = torch.randn(b, 4, 8, 8)
    sigma = torch.full((b,), 5.0)
    y = conds["y"].process_cond(b, "cpu").cond
    cc = conds["c_concat"].process_cond(b, "cpu").cond
    ca = conds["c_crossattn"].process_cond(b, "cpu").cond
    with torch.no_grad():
        out = model.apply_model(x, sigma, c_concat=cc, c_crossattn=ca, y=y, num_video_frames=3)
    assert out.shape == x.shape and torch.isfinite(out).all()
