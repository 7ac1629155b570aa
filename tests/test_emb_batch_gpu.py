"""The UNet's ResBlock time-embedding projections as ONE GEMM per forward (``UNetModel._emb_proj``) and the
GroupNorm kernels reading their ``pre_add`` column slice in place through a row stride
(``cgs_groupnorm_nhwc_{ws,dual,part}_pld``): GroupNorm against an fp32 reference of
``F.group_norm(x + pre_add[:, :, None, None])``, and the UNet with the batched projection against the same
weights with per-block projections (``CGS_EMB_BATCH=0``) and against fp32 on the CPU."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ref(x, pre, w, b, groups, eps, silu):
    y = F.group_norm(x.float() + pre.float()[:, :, None, None], groups, w.float(), b.float(), eps)
    return F.silu(y) if silu else y


@pytest.mark.parametrize("form", ["ws", "dual", "part"])
def test_groupnorm_strided_pre_add(cuda, form):
    from comfy_gen_server_amd import _native, ops
    assert _native.has_kernel("cgs_groupnorm_nhwc_ws_pld")
    torch.manual_seed(0)
    N, C, H, W = 2, 320, 16, 16
    big = torch.randn(N, 1000, device=cuda).to(torch.bfloat16)       # the batched projection
    pre = big[:, 200:200 + C]                                        # a column slice: row stride 1000
    assert pre.stride() == (1000, 1)
    w = (1 + 0.1 * torch.randn(C, device=cuda)).to(torch.bfloat16)
    b = (0.1 * torch.randn(C, device=cuda)).to(torch.bfloat16)
    ops.reset_stats()
    if form == "part":       # statistics as a conv epilogue leaves them (conv2d(gn_stats=True)), then finalize + apply
        x = (2 * torch.randn(N, C, H, W, device=cuda) - 1).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        v = x.permute(0, 2, 3, 1).reshape(N, H * W // 64, 64, C).float()      # 64-pixel blocks
        mean = v.mean(2)
        part = torch.stack([mean, ((v - mean[:, :, None]) ** 2).sum(2)], -1).contiguous()   # [N, blocks, C, 2]
        x._cgs_gnpart = (part.reshape(-1), x.data_ptr())
        y = ops.group_norm(x, 32, w, b, 1e-5, silu=True, pre_add=pre)
        ref = _ref(x, pre, w, b, 32, 1e-5, True)
    elif form == "dual":     # over cat([x, x2]) without the concat
        x = torch.randn(N, 192, H, W, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        x2 = torch.randn(N, C - 192, H, W, device=cuda).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        y = ops.group_norm(x, 32, w, b, 1e-5, silu=True, pre_add=pre, x2=x2)
        ref = _ref(torch.cat([x, x2], 1), pre, w, b, 32, 1e-5, True)
    else:
        x = (3 * torch.randn(N, C, H, W, device=cuda) + 1).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        y = ops.group_norm(x, 32, w, b, 1e-5, silu=False, pre_add=pre)
        ref = _ref(x, pre, w, b, 32, 1e-5, False)
    assert ops.stats().get(("groupnorm", "hip"), 0) == 1
    err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
    assert err < 2e-2, err
    # the slice was read in place: a contiguous copy of it gives the same result
    y2 = ops.group_norm(x, 32, w, b, 1e-5, silu=form != "ws", pre_add=pre.contiguous(),
                        x2=x2 if form == "dual" else None)
    assert torch.equal(y, y2)


def test_unet_batched_time_embedding(cuda, monkeypatch):
    from comfy_gen_server_amd import ops
    from comfy_gen_server_amd.models.layers import init_random_
    from comfy_gen_server_amd.models.unet import ResBlock, UNetModel
    cfg = dict(in_channels=4, model_channels=64, out_channels=4, num_res_blocks=1, channel_mult=(1, 2),
               transformer_depth=[1, 1], transformer_depth_output=[1, 1, 1, 1], transformer_depth_middle=1,
               context_dim=64, num_heads=2, use_linear_in_transformer=True)
    torch.manual_seed(0)
    ref = UNetModel(dtype=torch.float32, device="cpu", **cfg)
    init_random_(ref, seed=3)
    dev = UNetModel(dtype=torch.bfloat16, device="cuda", **cfg)
    dev.load_state_dict({k: v.to(torch.bfloat16) for k, v in ref.state_dict().items()})
    x = torch.randn(2, 4, 32, 32)
    t = torch.tensor([500.0, 20.0])
    ctx = torch.randn(2, 77, 64)
    n_blocks = sum(1 for m in dev.modules() if isinstance(m, ResBlock) and not m.skip_t_emb)
    assert n_blocks >= 5
    outs = {}
    with torch.inference_mode():
        for mode in ("1", "0"):
            monkeypatch.setenv("CGS_EMB_BATCH", mode)
            ops.reset_stats()
            outs[mode] = dev(x.cuda().to(torch.bfloat16), t.cuda(), ctx.cuda().to(torch.bfloat16)).float().cpu()
            outs["gemms" + mode] = ops.stats().get(("gemm", "hip"), 0)
        want = ref(x, t, ctx).float()
    # one projection GEMM instead of one per block
    assert outs["gemms0"] - outs["gemms1"] == n_blocks - 1, (outs["gemms0"], outs["gemms1"], n_blocks)
    assert dev.__dict__["_derived"]["emb_proj"][1].shape[0] == sum(
        m.out_channels for m in dev.modules() if isinstance(m, ResBlock) and not m.skip_t_emb)
    for mode in ("1", "0"):
        rel = ((outs[mode] - want).norm() / want.norm()).item()
        assert rel < 3e-2, (mode, rel)
    rel = ((outs["1"] - outs["0"]).norm() / outs["0"].norm()).item()
    assert rel < 1e-2, rel
