"""K17 / K24 region accumulate: the cond area/mask accumulation of calc_cond_batch (reference
comfy/samplers.py:205-228) and the feathered tile blend of tiled_scale (comfy/utils.py)."""
import pytest
import torch

from comfy_gen_server_amd import ops


def _feather_ref(ps, feather):
    mask = torch.ones_like(ps)
    for t in range(feather):                       # the reference's loop form
        a = (1.0 / feather) * (t + 1)
        mask[:, :, t:1 + t, :] *= a
        mask[:, :, mask.shape[2] - 1 - t:mask.shape[2] - t, :] *= a
        mask[:, :, :, t:1 + t] *= a
        mask[:, :, :, mask.shape[3] - 1 - t:mask.shape[3] - t] *= a
    return mask


def _check(dev, dtype):
    g = torch.Generator().manual_seed(0)
    out = torch.zeros(2, 3, 20, 24)
    div = torch.ones(2, 3, 20, 24) * 1e-37
    ref_o, ref_d = out.clone(), div.clone()
    piece = torch.randn(2, 3, 9, 11, generator=g)
    mult = torch.rand(2, 1, 9, 11, generator=g)
    # area + mask (mult broadcast over channels), a strided piece
    o_dev, d_dev = out.to(dev), div.to(dev)
    pd = torch.randn(2, 11, 9, 3, generator=g)
    piece_strided = pd.permute(0, 3, 2, 1)
    ops.region_accumulate(o_dev, d_dev, piece_strided.to(dev, dtype), 5, 7, mult=mult.to(dev, dtype))
    ref_o[:, :, 5:14, 7:18] += piece_strided.to(dtype).float() * mult.to(dtype).float()
    ref_d[:, :, 5:14, 7:18] += mult.to(dtype).float()
    # feathered tile, clipped at the border
    ps = torch.randn(2, 3, 8, 8, generator=g)
    ops.region_accumulate(o_dev, d_dev, ps.to(dev, dtype), 14, 18, feather=3)
    m = _feather_ref(ps, 3)[:, :, :6, :6]
    ref_o[:, :, 14:20, 18:24] += ps.to(dtype).float()[:, :, :6, :6] * m
    ref_d[:, :, 14:20, 18:24] += m
    y = ops.region_normalize(o_dev, d_dev)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert torch.allclose(o_dev.cpu(), ref_o, atol=tol, rtol=tol)
    assert torch.allclose(d_dev.cpu(), ref_d, atol=tol, rtol=tol)
    assert torch.allclose(y.cpu(), ref_o / ref_d, atol=tol * 10, rtol=tol * 10)


def test_region_accumulate_cpu():
    _check(torch.device("cpu"), torch.float32)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_region_accumulate_hip(cuda, dtype):
    ops.reset_stats()
    _check(cuda, dtype)
    assert ops.stats().get(("region_acc", "hip"), 0) == 3


def _clip_check(dev, dtype):
    g = torch.Generator().manual_seed(0)
    tok = torch.randn(100, 16, generator=g).to(dev, dtype)
    pos = torch.randn(77, 16, generator=g).to(dev, dtype)
    ids = torch.randint(0, 100, (3, 9), generator=g)
    ids[1, 4] = 99
    ids[1, 6] = 99                                      # ties: the first maximum wins (torch.argmax)
    y = ops.clip_embed(ids.to(dev), tok, pos)
    ref = tok.float().cpu()[ids] + pos.float().cpu()[:9]
    assert torch.allclose(y.float().cpu(), ref, atol=1e-2 if dtype != torch.float32 else 1e-6)
    x = torch.randn(3, 9, 16, generator=g).to(dev, dtype)
    p = ops.pooled_gather(x, ids.to(dev))
    refp = x.cpu()[torch.arange(3), ids.argmax(dim=-1)]
    assert torch.equal(p.cpu(), refp)


def test_clip_embed_cpu():
    _clip_check(torch.device("cpu"), torch.float32)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_clip_embed_hip(cuda, dtype):
    ops.reset_stats()
    _clip_check(cuda, dtype)
    assert ops.stats().get(("clip_embed", "hip"), 0) == 2


@pytest.mark.gpu
def test_lora_merge_product_on_hip(cuda):
    """K20: the LoRA up @ down product of calculate_weight runs on the HIP GEMM on the device."""
    from comfy_gen_server_amd.runtime.patcher import calculate_weight
    g = torch.Generator().manual_seed(0)
    w = torch.randn(640, 1280, generator=g)
    up, down = torch.randn(640, 32, generator=g) * 0.1, torch.randn(32, 1280, generator=g) * 0.1
    ref = calculate_weight([(0.8, ("lora", (up, down, 16.0, None, None)), 1.0)], w.clone(), "k")
    # bf16 base weight: the rank-r product runs on the HIP GEMM (its one bf16 rounding is below the
    # merged bf16 weight's own)
    ops.reset_stats()
    out = calculate_weight([(0.8, ("lora", (up.to(cuda), down.to(cuda), 16.0, None, None)), 1.0)], w.to(cuda), "k",
                           base_dtype=torch.bfloat16)
    assert ops.stats().get(("gemm", "hip"), 0) == 1
    assert torch.allclose(out.cpu(), ref, atol=2e-3, rtol=1e-3)
    # fp32 base weight: fp32 torch.mm like the reference, no bf16 GEMM
    ops.reset_stats()
    out32 = calculate_weight([(0.8, ("lora", (up.to(cuda), down.to(cuda), 16.0, None, None)), 1.0)], w.to(cuda), "k")
    assert ops.stats().get(("gemm", "hip"), 0) == 0
    assert torch.allclose(out32.cpu(), ref, atol=2e-5, rtol=1e-5)
