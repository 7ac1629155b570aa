"""Stable Cascade stages: the NHWC re-formulations (patchify GEMMs, pixel (un)shuffle order, GRN,
depthwise conv, blocks) against direct NCHW torch math of comfy/ldm/cascade/common.py, plus tiny
Stage C / B / A models end to end (sampling through the Stage C wrapper) and checkpoint key names."""
import math

import pytest
import torch
import torch.nn.functional as F

from comfy_gen_server_amd.models import cascade as SC
from comfy_gen_server_amd.models.layers import init_random_


def _ln2d(x, eps=1e-6):
    return F.layer_norm(x.permute(0, 2, 3, 1), (x.shape[1],), eps=eps).permute(0, 3, 1, 2)


def _grn_ref(x_nhwc, gamma, beta):
    gx = torch.norm(x_nhwc, p=2, dim=(1, 2), keepdim=True)
    nx = gx / (gx.mean(dim=-1, keepdim=True) + 1e-6)
    return gamma * (x_nhwc * nx) + beta + x_nhwc


def _mlp_ref(m, x):
    h = F.gelu(F.linear(x, m[0].weight, m[0].bias))
    h = _grn_ref(h, m[2].gamma, m[2].beta)
    return F.linear(h, m[4].weight, m[4].bias)


def test_resblock_matches_nchw_reference():
    torch.manual_seed(0)
    blk = SC.ResBlock(16, c_skip=8)
    init_random_(blk, seed=1)
    x = torch.randn(2, 16, 6, 5)
    skip = torch.randn(2, 8, 6, 5)
    dw = F.conv2d(x, blk.depthwise.weight, blk.depthwise.bias, padding=1, groups=16)
    h = torch.cat([_ln2d(dw), skip], dim=1)
    ref = _mlp_ref(blk.channelwise, h.permute(0, 2, 3, 1)).permute(0, 3, 1, 2) + x
    out = blk(x.permute(0, 2, 3, 1).contiguous(), skip.permute(0, 2, 3, 1).contiguous()).permute(0, 3, 1, 2)
    assert torch.allclose(out, ref, atol=1e-4, rtol=1e-4)


def test_attn_and_timestep_blocks_match_reference():
    torch.manual_seed(0)
    c, cc, heads = 16, 12, 2
    blk = SC.AttnBlock(c, cc, heads, self_attn=True)
    init_random_(blk, seed=2)
    x = torch.randn(2, c, 4, 3)
    cond = torch.randn(2, 5, cc)
    kv = F.linear(F.silu(cond), blk.kv_mapper[1].weight, blk.kv_mapper[1].bias)
    xn = _ln2d(x).flatten(2).transpose(1, 2)
    kvin = torch.cat([xn, kv], dim=1)
    a = blk.attention.attn
    q, k, v = (F.linear(t, m.weight, m.bias) for t, m in ((xn, a.to_q), (kvin, a.to_k), (kvin, a.to_v)))
    sp = lambda t: t.view(2, -1, heads, c // heads).transpose(1, 2)  # noqa: E731
    o = F.scaled_dot_product_attention(sp(q), sp(k), sp(v)).transpose(1, 2).reshape(2, -1, c)
    o = F.linear(o, a.out_proj.weight, a.out_proj.bias)
    ref = x + o.transpose(1, 2).reshape(x.shape)
    out = blk(x.permute(0, 2, 3, 1).contiguous(), cond).permute(0, 3, 1, 2)
    assert torch.allclose(out, ref, atol=1e-4, rtol=1e-4)

    tb = SC.TimestepBlock(c, 8, conds=["sca", "crp"])
    init_random_(tb, seed=3)
    t = torch.randn(2, 24)
    ts = t.chunk(3, dim=1)
    ab = F.linear(ts[0], tb.mapper.weight, tb.mapper.bias)
    ab = ab + F.linear(ts[1], tb.mapper_sca.weight, tb.mapper_sca.bias)
    ab = ab + F.linear(ts[2], tb.mapper_crp.weight, tb.mapper_crp.bias)
    aa, bb = ab[:, :, None, None].chunk(2, dim=1)
    ref = x * (1 + aa) + bb
    out = tb(x.permute(0, 2, 3, 1).contiguous(), t).permute(0, 3, 1, 2)
    assert torch.allclose(out, ref, atol=1e-5)


def test_patch_convs_and_depthwise_match_torch():
    torch.manual_seed(0)
    pc = SC._PatchConv(8, 12, 2, stride=2)
    init_random_(pc, seed=4)
    x = torch.randn(2, 8, 6, 4)
    ref = F.conv2d(x, pc.weight, pc.bias, stride=2)
    out = pc.forward_nhwc(x.permute(0, 2, 3, 1).contiguous()).permute(0, 3, 1, 2)
    assert torch.allclose(out, ref, atol=1e-5)
    pt = SC._PatchConvTranspose(12, 8, 2)
    init_random_(pt, seed=5)
    y = torch.randn(2, 12, 3, 2)
    ref = F.conv_transpose2d(y, pt.weight, pt.bias, stride=2)
    out = pt.forward_nhwc(y.permute(0, 2, 3, 1).contiguous()).permute(0, 3, 1, 2)
    assert torch.allclose(out, ref, atol=1e-5)
    dw = SC.DepthwiseConv2d(8, 3, replicate=True)
    init_random_(dw, seed=6)
    ref = F.conv2d(F.pad(x, (1, 1, 1, 1), mode="replicate"), dw.weight, dw.bias, groups=8)
    out = dw.forward_nhwc(x.permute(0, 2, 3, 1).contiguous()).permute(0, 3, 1, 2)
    assert torch.allclose(out, ref, atol=1e-5)


def _tiny_c():
    return dict(c_in=16, c_out=16, c_r=16, c_cond=32, c_hidden=[32, 32], nhead=[2, 2], blocks=[[1, 1], [1, 1]],
                block_repeat=[[1, 1], [2, 1]], level_config=["CTA", "CTA"], c_clip_text=24, c_clip_text_pooled=24,
                c_clip_img=768, c_clip_seq=2, switch_level=[False])


def test_stage_c_b_forward_and_keys():
    torch.manual_seed(0)
    m = SC.StageC(**_tiny_c())
    init_random_(m, seed=7)
    sd = m.state_dict()
    for k in ("down_downscalers.1.1.blocks.0.weight", "up_upscalers.0.1.blocks.1.weight", "clf.1.weight",
              "embedding.1.weight", "down_blocks.0.0.channelwise.2.gamma", "down_blocks.0.2.kv_mapper.1.weight",
              "down_blocks.0.2.attention.attn.out_proj.weight", "down_blocks.0.1.mapper_crp.weight",
              "up_repeat_mappers.0.0.weight", "up_blocks.1.0.channelwise.0.weight"):
        assert k in sd, k
    assert sd["up_blocks.1.0.channelwise.0.weight"].shape[1] == 64     # c + c_skip at level 0
    x = torch.randn(2, 16, 6, 6)
    out = m(x, torch.tensor([0.3, 0.7]), torch.randn(2, 7, 24), torch.randn(2, 1, 24), torch.randn(2, 1, 768))
    assert out.shape == x.shape and torch.isfinite(out).all()
    # ControlNet residuals ("input" list, popped per ResBlock) change the output
    cn = [torch.randn(2, 32, 3, 3) * 0.1 for _ in range(8)]
    out2 = m(x, torch.tensor([0.3, 0.7]), torch.randn(2, 7, 24), torch.randn(2, 1, 24), torch.randn(2, 1, 768),
             control={"input": cn})
    assert out2.shape == x.shape

    b = SC.StageB(c_in=4, c_out=4, c_r=16, patch_size=2, c_cond=32, c_hidden=[16, 24, 32], nhead=[-1, 2, 2],
                  blocks=[[1, 1, 1], [1, 1, 1]], block_repeat=[[1, 1, 1], [2, 1, 1]], level_config=["CT", "CTA", "CTA"],
                  c_clip=24, c_clip_seq=2, c_effnet=16)
    init_random_(b, seed=8)
    bsd = b.state_dict()
    for k in ("effnet_mapper.2.weight", "pixels_mapper.0.weight", "clip_mapper.weight", "down_downscalers.1.1.weight",
              "up_upscalers.0.1.weight", "up_upscalers.1.1.bias"):
        assert k in bsd, k
    assert bsd["up_upscalers.0.1.weight"].shape == (32, 24, 2, 2)          # ConvTranspose2d [Cin, Cout, k, k]
    xb = torch.randn(2, 4, 16, 16)
    ob = b(xb, torch.tensor([0.5, 0.5]), torch.randn(2, 16, 3, 3), torch.randn(2, 1, 24))
    assert ob.shape == xb.shape and torch.isfinite(ob).all()


def test_stage_a_and_coders():
    torch.manual_seed(0)
    a = SC.StageA(levels=2, bottleneck_blocks=2, c_hidden=32, c_latent=4, codebook_size=16)
    init_random_(a, seed=9)
    for bn in (a.down_blocks[-1][1],):
        bn.running_mean.zero_()
        bn.running_var.fill_(1.0)
    img = torch.rand(1, 3, 32, 32)
    z = a.encode(img)
    assert z.shape == (1, 4, 8, 8)
    q, zz, idx = a.encode(img, quantize=True)
    assert q.shape == z.shape and idx.shape == (1, 8, 8)
    assert torch.allclose(q.permute(0, 2, 3, 1).reshape(-1, 4), a.vquantizer.codebook.weight[idx.flatten()])
    assert a.decode(z).shape == (1, 3, 32, 32)
    assert "vquantizer.codebook.weight" in a.state_dict() and "down_blocks.0.depthwise.1.weight" in a.state_dict()

    feats = SC.efficientnet_v2_s_features()
    n = sum(p.numel() for p in feats.parameters())
    assert abs(n - 20_177_488) < 1000, n                        # torchvision efficientnet_v2_s().features
    assert "1.0.block.0.1.num_batches_tracked" in feats.state_dict()
    coder = SC.StageC_coder().eval()
    assert coder.encode(torch.rand(1, 3, 64, 64) * 2 - 1).shape == (1, 16, 2, 2)
    assert coder.decode(torch.randn(1, 16, 4, 4)).shape == (1, 3, 32, 32)
    assert "blocks.11.num_batches_tracked" in coder.previewer.state_dict()


def test_stage_c_wrapper_samples_and_cascade_nodes():
    from comfy_gen_server_amd.graph import registry
    from comfy_gen_server_amd.runtime import families
    from comfy_gen_server_amd.runtime.patcher import ModelPatcher
    registry.init_nodes(custom_nodes=False)
    NM = registry.NODE_CLASS_MAPPINGS
    cfg = dict(_tiny_c(), stable_cascade_stage="c")
    fam = families.Stable_Cascade_C(cfg)
    model = fam.get_model({})
    init_random_(model.diffusion_model, seed=10)
    model.diffusion_model.float()
    patcher = ModelPatcher(model, load_device=torch.device("cpu"), offload_device=torch.device("cpu"))
    pos = [[torch.randn(1, 7, 24), {"pooled_output": torch.randn(1, 24)}]]
    neg = [[torch.zeros(1, 7, 24), {"pooled_output": torch.zeros(1, 24)}]]
    lat_c, lat_b = NM["StableCascade_EmptyLatentImage"]().generate(256, 256, 42, 2)
    assert lat_c["samples"].shape == (2, 16, 6, 6) and lat_b["samples"].shape == (2, 4, 64, 64)
    out = NM["KSampler"]().sample(patcher, 1, 3, 4.0, "euler_ancestral", "simple", pos, neg, lat_c, 1.0)[0]
    assert out["samples"].shape == (2, 16, 6, 6) and torch.isfinite(out["samples"]).all()
    cond_b = NM["StableCascade_StageB_Conditioning"]().set_prior(pos, out)[0]
    assert cond_b[0][1]["stable_cascade_prior"] is out["samples"]
