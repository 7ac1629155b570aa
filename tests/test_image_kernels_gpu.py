"""HIP image / utility kernels (csrc/kernels/image.hip) against plain PyTorch fp32 references:
resize (nearest / nearest-exact / bilinear / bicubic / area), StyleGAN fused bias-act and
upfirdn2d, VQ nearest-codebook, ConvNeXt-V2 GRN. CPU tests pin the torch fallbacks to the same
references so both paths implement one definition."""
import pytest
import torch
import torch.nn.functional as F

from comfy_gen_server_amd import ops

MODES = ["nearest", "nearest-exact", "bilinear", "bicubic", "area"]


def _ref_resize(x, size, mode, align=None):
    kw = {"align_corners": align} if mode in ("bilinear", "bicubic") else {}
    return F.interpolate(x.float(), size=size, mode=mode, **kw)


def _ref_fba(x, b, slope=0.2, scale=2 ** 0.5):
    return F.leaky_relu(x.float() + b.float().view(1, -1, *([1] * (x.dim() - 2))), slope) * scale


def _ref_grn(x, g, b):
    gx = torch.norm(x.float(), p=2, dim=(1, 2), keepdim=True)
    nx = gx / (gx.mean(dim=-1, keepdim=True) + 1e-6)
    return g.float() * (x.float() * nx) + b.float() + x.float()


def test_cpu_fallbacks_match_references():
    x = torch.randn(2, 3, 9, 7)
    for m in MODES:
        assert torch.allclose(ops.interpolate(x, (13, 5), m), _ref_resize(x, (13, 5), m), atol=1e-6)
    b = torch.randn(3)
    assert torch.allclose(ops.fused_bias_act(x, b), _ref_fba(x, b), atol=1e-6)
    k = torch.tensor([1., 3., 3., 1.])
    k = (k[None] * k[:, None]) / 64
    y = ops.upfirdn2d(x, k, up=2, pad=(2, 1))
    assert y.shape == (2, 3, 18, 14)
    z, cb = torch.randn(50, 8), torch.randn(40, 8)
    q, idx = ops.vq_nearest(z, cb)
    assert torch.equal(idx, torch.cdist(z, cb).argmin(1)) and torch.equal(q, cb[idx])
    xn, g, bb = torch.randn(2, 5, 6, 16), torch.randn(16), torch.randn(16)
    assert torch.allclose(ops.grn_nhwc(xn, g, bb), _ref_grn(xn, g, bb), atol=1e-5)


def test_upfirdn2d_reference_is_true_convolution():
    """down=1/up=1 upfirdn2d with an asymmetric kernel == conv2d with the flipped kernel."""
    x = torch.randn(1, 2, 8, 8)
    k = torch.arange(1., 10.).view(3, 3)
    y = ops.upfirdn2d_reference(x, k, (1, 1), (1, 1), (1, 1, 1, 1))
    ref = F.conv2d(x.view(2, 1, 8, 8), torch.flip(k, [0, 1])[None, None], padding=1).view(1, 2, 8, 8)
    assert torch.allclose(y, ref, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_resize_gpu(cuda, mode, dtype):
    x = torch.randn(2, 4, 37, 53)
    for size in [(64, 96), (20, 31), (37, 53)]:
        aligns = [False, True] if mode in ("bilinear", "bicubic") else [None]
        for al in aligns:
            ops.reset_stats()
            y = ops.interpolate(x.to(cuda, dtype), size, mode, align_corners=al).float().cpu()
            assert ops.stats().get(("resize", "hip"), 0) == 1
            ref = _ref_resize(x.to(dtype), size, mode, al)
            tol = 1e-4 if dtype == torch.float32 else 2e-2 * max(1.0, ref.abs().max().item())
            assert (y - ref).abs().max().item() < tol, (mode, size, al)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_fused_bias_act_gpu(cuda, dtype):
    x, b = torch.randn(3, 24, 11, 7), torch.randn(24)
    ops.reset_stats()
    y = ops.fused_bias_act(x.to(cuda, dtype), b.to(cuda, dtype), 0.2, 2 ** 0.5).float().cpu()
    assert ops.stats().get(("fused_bias_act", "hip"), 0) == 1
    ref = _ref_fba(x.to(dtype), b.to(dtype))
    assert (y - ref).abs().max().item() < (1e-5 if dtype == torch.float32 else 5e-2)
    x2 = torch.randn(64, 512)                      # [rows, C] (EqualLinear activation)
    y2 = ops.fused_bias_act(x2.to(cuda), b.new_ones(512).to(cuda)).cpu()
    assert torch.allclose(y2, _ref_fba(x2, torch.ones(512)), atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [dict(up=2, down=1, pad=(2, 1)), dict(up=1, down=2, pad=(1, 1)),
                                 dict(up=1, down=1, pad=(1, 2)), dict(up=2, down=2, pad=(-1, 0))])
def test_upfirdn2d_gpu(cuda, cfg):
    k = torch.tensor([1., 3., 3., 1.])
    k = (k[None] * k[:, None])
    k = k / k.sum() * (cfg["up"] ** 2)
    x = torch.randn(2, 6, 17, 12)
    ops.reset_stats()
    y = ops.upfirdn2d(x.to(cuda), k, **cfg).cpu()
    assert ops.stats().get(("upfirdn2d", "hip"), 0) == 1
    p = cfg["pad"]
    ref = ops.upfirdn2d_reference(x, k, (cfg["up"],) * 2, (cfg["down"],) * 2, (p[0], p[1], p[0], p[1]))
    assert y.shape == ref.shape and torch.allclose(y, ref, atol=1e-5)
    yb = ops.upfirdn2d(x.to(cuda, torch.bfloat16), k, **cfg).float().cpu()
    assert (yb - ref).abs().max().item() < 5e-2


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(4096, 8192, 4), (256, 1024, 256), (33, 100, 64)])
def test_vq_nearest_gpu(cuda, shape):
    M, n, D = shape
    g = torch.Generator().manual_seed(0)
    cb = torch.randn(n, D, generator=g)
    z = cb[torch.randint(0, n, (M,), generator=g)] + 0.01 * torch.randn(M, D, generator=g)
    ops.reset_stats()
    q, idx = ops.vq_nearest(z.to(cuda), cb.to(cuda))
    assert ops.stats().get(("vq", "hip"), 0) == 1
    ref_idx = torch.cdist(z.double(), cb.double()).argmin(1)
    assert torch.equal(idx.cpu(), ref_idx) and torch.equal(q.cpu(), cb[ref_idx])


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(2, 24, 24, 8192), (4, 64, 64, 1536), (1, 5, 7, 64)])
@pytest.mark.parametrize("pre_gelu", [False, True])
def test_grn_v2_gpu(cuda, shape, pre_gelu):
    """K28 v2: vectorised GRN (per-slice partials, no atomics) with the optional fused pre-GELU of
    Cascade's Linear -> GELU -> GRN, vs fp32 torch."""
    N, H, W, C = shape
    x, g, b = torch.randn(*shape), torch.randn(C) * 0.5, torch.randn(C) * 0.1
    ops.reset_stats()
    y = ops.grn_nhwc(x.to(cuda, torch.bfloat16), g.to(cuda, torch.bfloat16), b.to(cuda, torch.bfloat16),
                     pre_gelu=pre_gelu).float().cpu()
    assert ops.stats().get(("grn", "hip"), 0) == 1
    xr = x.to(torch.bfloat16).float()
    ref = _ref_grn(F.gelu(xr) if pre_gelu else xr, g.to(torch.bfloat16), b.to(torch.bfloat16))
    assert ((y - ref).norm() / ref.norm()).item() < 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(2, 24, 24, 8192), (3, 7, 5, 2056), (1, 33, 1, 4096)])
@pytest.mark.parametrize("pre_gelu", [False, True])
def test_grn_apply_row_tiled_matches_grid_stride(cuda, shape, pre_gelu):
    """The row-tiled GRN apply (per-thread channel coefficients, cgs_grn_set_rows(1), the default) vs the
    grid-stride apply it replaced (0): same values to fp32 rounding of the coefficient product."""
    from comfy_gen_server_amd import _native
    lib = _native.load_kernels()
    N, H, W, C = shape
    torch.manual_seed(2)
    x = torch.randn(*shape, device=cuda).to(torch.bfloat16)
    g = (torch.randn(C, device=cuda) * 0.5).to(torch.bfloat16)
    b = (torch.randn(C, device=cuda) * 0.1).to(torch.bfloat16)
    try:
        lib.cgs_grn_set_rows(0)
        old = ops.grn_nhwc(x, g, b, pre_gelu=pre_gelu).float()
        lib.cgs_grn_set_rows(1)
        new = ops.grn_nhwc(x, g, b, pre_gelu=pre_gelu).float()
    finally:
        lib.cgs_grn_set_rows(1)
    assert ((new - old).norm() / old.norm()).item() < 1e-3


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_grn_gpu(cuda, dtype):
    x, g, b = torch.randn(2, 24, 24, 2048), torch.randn(2048) * 0.5, torch.randn(2048) * 0.1
    ops.reset_stats()
    y = ops.grn_nhwc(x.to(cuda, dtype), g.to(cuda, dtype), b.to(cuda, dtype)).float().cpu()
    assert ops.stats().get(("grn", "hip"), 0) == 1
    ref = _ref_grn(x.to(dtype), g.to(dtype), b.to(dtype))
    rel = ((y - ref).norm() / ref.norm()).item()
    assert rel < (1e-5 if dtype == torch.float32 else 1e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_softmax_rows_and_attention_probs_gpu(cuda, dtype):
    """K05: the materialised attention map (SAG / PAG) from the HIP row softmax == fp32 reference."""
    x = torch.randn(37, 1024) * 4
    ops.reset_stats()
    y = ops.softmax_rows(x.to(cuda, dtype), 0.125).cpu()
    assert ops.stats().get(("softmax", "hip"), 0) == 1
    assert torch.allclose(y, torch.softmax(x.to(dtype).float() * 0.125, -1), atol=1e-5)
    q, k, v = (torch.randn(2, 256, 4 * 64) for _ in range(3))
    o, p = ops.attention_with_probs(q.to(cuda), k.to(cuda), v.to(cuda), 4)
    qh, kh = (t.view(2, 256, 4, 64).transpose(1, 2).reshape(8, 256, 64) for t in (q, k))
    pref = torch.softmax(qh @ kh.transpose(1, 2) / 8.0, -1)
    assert torch.allclose(p.cpu(), pref, atol=1e-5)
    from comfy_gen_server_amd.ops.core import attention_reference
    assert torch.allclose(o.cpu(), attention_reference(q, k, v, 4), atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("b,heads,sq,sk,d", [(2, 5, 300, 77, 64), (1, 10, 1024, 1024, 64), (3, 2, 65, 130, 40)])
def test_attention_probs_bf16_mfma_gpu(cuda, b, heads, sq, sk, d):
    """K05 device path: fp32-MFMA batched GEMMs over the strided per-head views (q from a fused QKV)
    + in-place HIP softmax, vs the fp32 reference of the same bf16 inputs."""
    torch.manual_seed(6)
    qkv = torch.randn(b, sq, 3 * heads * d).to(torch.bfloat16)
    hd = heads * d
    q = qkv[..., :hd]
    k = torch.randn(b, sk, hd).to(torch.bfloat16)
    v = torch.randn(b, sk, hd).to(torch.bfloat16)
    ops.reset_stats()
    o, p = ops.attention_with_probs(q.to(cuda), k.to(cuda), v.to(cuda), heads)
    st = ops.stats()
    assert st.get(("attention", "hip"), 0) == 1 and st.get(("softmax", "hip"), 0) == 1, st
    qh = q.float().reshape(b, sq, heads, d).transpose(1, 2).reshape(b * heads, sq, d)
    kh = k.float().reshape(b, sk, heads, d).transpose(1, 2).reshape(b * heads, sk, d)
    pref = torch.softmax(qh @ kh.transpose(1, 2) * d ** -0.5, -1)
    assert (p.cpu() - pref).abs().max().item() < 1e-4
    from comfy_gen_server_amd.ops.core import attention_reference
    oref = attention_reference(q.float(), k.float(), v.float(), heads)
    assert ((o.float().cpu() - oref).norm() / oref.norm()).item() < 1e-2


def test_attention_probs_cpu():
    q, k, v = (torch.randn(1, 16, 2 * 8) for _ in range(3))
    o, p = ops.attention_with_probs(q, k, v, 2)
    assert p.shape == (2, 16, 16) and torch.allclose(p.sum(-1), torch.ones(2, 16))


@pytest.mark.gpu
def test_vae_out_u8_matches_reference(cuda):
    """K23: the fused bf16 NHWC -> uint8 HWC kernel equals clamp((x+1)/2)*255+0.5 -> uint8."""
    from comfy_gen_server_amd import ops
    torch.manual_seed(0)
    x = (torch.randn(2, 3, 37, 53, device=cuda) * 1.5).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    ops.reset_stats()
    y = ops.vae_out_u8(x)
    ref = (torch.clamp((x.float() + 1.0) / 2.0, 0.0, 1.0).movedim(1, -1) * 255.0 + 0.5).to(torch.uint8)
    assert ops.stats().get(("vae_u8", "hip"), 0) == 1
    assert y.shape == (2, 37, 53, 3) and torch.equal(y, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("shape,t,cl", [((2, 1280, 32, 32), 1, True), ((2, 640, 64, 64), 1, False),
                                        ((1, 96, 17, 24), 2, True), ((3, 64, 8, 8), 4, False)])
def test_fourier_filter_vs_fft(cuda, shape, t, cl):
    """K29: FreeU's low-frequency scaling from (2t)^2 DFT coefficients == the reference's
    fftn -> fftshift -> mask -> ifftshift -> ifftn -> real (comfy_extras/nodes_freelunch.py:6-23)."""
    from comfy_gen_server_amd import ops
    from comfy_gen_server_amd.ops import dispatch
    dispatch.reset_stats()
    torch.manual_seed(3)
    x = (torch.randn(*shape, device=cuda) + 0.3).to(torch.bfloat16)
    if cl:
        x = x.contiguous(memory_format=torch.channels_last)
    y = ops.fourier_filter(x, t, 0.2)
    assert dispatch.stats().get(("fourier", "hip"), 0) == 1
    B, C, H, W = shape
    xf = torch.fft.fftshift(torch.fft.fftn(x.float(), dim=(-2, -1)), dim=(-2, -1))
    mask = torch.ones_like(xf.real)
    mask[..., H // 2 - t:H // 2 + t, W // 2 - t:W // 2 + t] = 0.2
    ref = torch.fft.ifftn(torch.fft.ifftshift(xf * mask, dim=(-2, -1)), dim=(-2, -1)).real
    assert (y.float() - ref).abs().max().item() < 2e-2 * ref.abs().max().item()


def test_fourier_filter_cpu_is_reference():
    from comfy_gen_server_amd import ops
    x = torch.randn(2, 8, 12, 10)
    y = ops.fourier_filter(x, 1, 0.5)
    xf = torch.fft.fftshift(torch.fft.fftn(x, dim=(-2, -1)), dim=(-2, -1))
    xf[..., 5:7, 4:6] *= 0.5
    ref = torch.fft.ifftn(torch.fft.ifftshift(xf, dim=(-2, -1)), dim=(-2, -1)).real
    assert torch.allclose(y, ref, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("B,Na,Nb,C", [(2, 3072, 1024, 320), (3, 100, 37, 64), (1, 65, 200, 1280)])
def test_tome_match_vs_reference(cuda, B, Na, Nb, C):
    """K30: fused cosine-similarity argmax == normalise + matmul + max (comfy_extras/nodes_tomesd.py)."""
    from comfy_gen_server_amd import ops
    from comfy_gen_server_amd.ops import dispatch
    dispatch.reset_stats()
    torch.manual_seed(4)
    a = torch.randn(B, Na, C, device=cuda).to(torch.bfloat16)
    b = torch.randn(B, Nb, C, device=cuda).to(torch.bfloat16)
    vmax, imax = ops.tome_match(a, b)
    assert dispatch.stats().get(("tome", "hip"), 0) == 1
    af, bf = a.float(), b.float()
    s = (af / af.norm(dim=-1, keepdim=True)) @ (bf / bf.norm(dim=-1, keepdim=True)).transpose(-1, -2)
    rv, ri = s.max(dim=-1)
    assert (vmax - rv).abs().max().item() < 1e-4
    picked = torch.gather(s, -1, imax[..., None])[..., 0]      # the chosen dst is (one of) the best
    assert (picked - rv).abs().max().item() < 1e-4
