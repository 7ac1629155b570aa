"""fp16 / fp32 UNets on the device (--fp16-unet / --force-fp32): the decoder's skip concat must not take
the bf16-only dual-source conv path (K14), and every conv that cannot run the HIP kernel must see the
materialised concat. The output is compared with the same weights in fp32 on the CPU."""
import pytest
import torch

pytestmark = pytest.mark.gpu

CFG = dict(in_channels=4, model_channels=64, out_channels=4, num_res_blocks=1, channel_mult=(1, 2),
           transformer_depth=[1, 1], transformer_depth_output=[1, 1, 1, 1], transformer_depth_middle=1,
           context_dim=64, num_heads=2, use_linear_in_transformer=True)


@pytest.mark.parametrize("dtype", [torch.float16, torch.float32, torch.bfloat16])
def test_unet_forward_dtypes(dtype):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from comfy_gen_server_amd.models.layers import init_random_
    from comfy_gen_server_amd.models.unet import UNetModel
    torch.manual_seed(0)
    ref = UNetModel(dtype=torch.float32, device="cpu", **CFG)
    init_random_(ref, seed=3)
    dev = UNetModel(dtype=dtype, device="cuda", **CFG)
    dev.load_state_dict({k: v.to(dtype) for k, v in ref.state_dict().items()})
    x = torch.randn(2, 4, 32, 32)
    t = torch.tensor([500.0, 20.0])
    ctx = torch.randn(2, 77, 64)
    with torch.inference_mode():
        want = ref(x, t, ctx).float()
        got = dev(x.cuda().to(dtype), t.cuda(), ctx.cuda().to(dtype)).float().cpu()
    assert torch.isfinite(got).all()
    rel = (got - want).norm() / want.norm()
    assert rel < (3e-2 if dtype == torch.bfloat16 else 1e-2), float(rel)
