"""Video UNet / temporal VAE on the device (temporal Conv3d through the MFMA conv kernel, clip-wide
GroupNorm through the NHWC GN kernel) vs the fp32 CPU path with the same weights."""
import pytest
import torch

from comfy_gen_server_amd import ops
from comfy_gen_server_amd.models.layers import init_random_
from comfy_gen_server_amd.models.unet import UNetModel
from comfy_gen_server_amd.models.vae import Decoder

pytestmark = pytest.mark.gpu

CFG = dict(in_channels=8, model_channels=64, out_channels=4, num_res_blocks=[1, 1], channel_mult=[1, 2],
           transformer_depth=[1, 1], transformer_depth_output=[1, 1, 1, 1], transformer_depth_middle=1,
           num_heads=-1, num_head_channels=32, use_linear_in_transformer=True, context_dim=64,
           num_classes="sequential", adm_in_channels=32, use_temporal_resblock=True, use_temporal_attention=True,
           extra_ff_mix_layer=True, use_spatial_context=True, merge_strategy="learned_with_images",
           merge_factor=0.0, video_kernel_size=[3, 1, 1])


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def test_video_unet_device_matches_cpu(cuda):
    torch.manual_seed(0)
    m = UNetModel(**CFG, dtype=torch.float32)
    init_random_(m, seed=4)
    x = torch.randn(2 * 4, 8, 16, 16)
    t = torch.rand(8) * 900
    c = torch.randn(8, 1, 64)
    y = torch.randn(8, 32)
    with torch.no_grad():
        ref = m(x, t, context=c, y=y, num_video_frames=4)
        md = UNetModel(**CFG, dtype=torch.bfloat16, device=cuda)
        md.load_state_dict(m.state_dict())
        ops.reset_stats()
        out = md(x.to(cuda), t.to(cuda), context=c.to(cuda), y=y.to(cuda), num_video_frames=4)
    st = ops.stats()
    assert st.get(("conv", "hip"), 0) > 0 and st.get(("attention", "hip"), 0) > 0, st
    assert _rel(out.cpu(), ref) < 3e-2


def test_temporal_vae_device_matches_cpu(cuda):
    kw = dict(ch=64, out_ch=3, ch_mult=[1, 2], num_res_blocks=1, z_channels=4, video_kernel_size=[3, 1, 1])
    m = Decoder(**kw)
    init_random_(m, seed=7)
    for k, v in m.state_dict().items():
        if k.endswith("mix_factor"):
            v.fill_(0.2)
    z = torch.randn(5, 4, 16, 16)
    with torch.no_grad():
        ref = m(z)
        md = Decoder(**kw, dtype=torch.bfloat16, device=cuda)
        md.load_state_dict(m.state_dict())
        out = md(z.to(cuda, torch.bfloat16).contiguous(memory_format=torch.channels_last))
    assert _rel(out.cpu(), ref) < 3e-2
