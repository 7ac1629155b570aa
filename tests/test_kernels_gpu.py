"""HIP kernel numerics vs plain PyTorch fp32 references (SURVEY §7.4 'Kernel unit tests').

Every test asserts the native path actually ran (ops.stats) so a silent fallback fails."""
import math

import pytest
import torch
import torch.nn.functional as F

from comfy_gen_server_amd import ops, _native
from comfy_gen_server_amd.ops import core

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _native_loaded(cuda, monkeypatch):
    assert _native.load_kernels() is not None, _native.kernels_error()
    monkeypatch.setenv("CGS_AUTOTUNE", "0")    # variant fixtures pick the kernel explicitly
    ops.reset_stats()
    yield


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("N,C,H,W,G", [(2, 320, 32, 32, 32), (2, 640, 16, 16, 32), (1, 1280, 8, 8, 32),
                                       (2, 960, 16, 16, 32), (1, 128, 64, 64, 32), (3, 64, 5, 7, 32),
                                       (2, 2560, 16, 16, 32), (2, 1920, 8, 8, 32), (1, 3840, 4, 5, 32),
                                       (1, 4096, 6, 6, 32)])
@pytest.mark.parametrize("silu", [False, True])
def test_groupnorm(cuda, N, C, H, W, G, silu):
    torch.manual_seed(0)
    x = (torch.randn(N, C, H, W, device=cuda) * 3 + 1).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = torch.randn(C, device=cuda).to(torch.bfloat16)
    b = torch.randn(C, device=cuda).to(torch.bfloat16)
    pre = torch.randn(N, C, device=cuda).to(torch.bfloat16)
    y = ops.group_norm(x, G, w, b, 1e-5, silu=silu, pre_add=pre)
    ref = F.group_norm(x.float() + pre.float()[:, :, None, None], G, w.float(), b.float(), 1e-5)
    if silu:
        ref = F.silu(ref)
    assert ops.stats().get(("groupnorm", "hip"), 0) == 1
    assert _rel(y, ref) < 1e-2


@pytest.mark.parametrize("N,C,H,W,pre,shift", [(4, 320, 128, 128, False, 1.0), (3, 640, 96, 80, True, 1.0),
                                                 (2, 128, 256, 256, False, 40.0), (5, 512, 33, 17, False, 8.0)])
def test_groupnorm_large_and_no_preadd(cuda, N, C, H, W, pre, shift):
    # grid-stride rows cross image boundaries (per-thread coefficient reload), no pre-add, large means
    torch.manual_seed(1)
    x = (torch.randn(N, C, H, W, device=cuda) + shift).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = torch.randn(C, device=cuda).to(torch.bfloat16)
    b = torch.randn(C, device=cuda).to(torch.bfloat16)
    p = torch.randn(N, C, device=cuda).to(torch.bfloat16) if pre else None
    y = ops.group_norm(x, 32, w, b, 1e-6, silu=True, pre_add=p)
    xf = x.float() + (p.float()[:, :, None, None] if pre else 0.0)
    ref = F.silu(F.group_norm(xf, 32, w.float(), b.float(), 1e-6))
    assert ops.stats().get(("groupnorm", "hip"), 0) == 1
    assert _rel(y, ref) < 1e-2


@pytest.mark.parametrize("rows,C", [(100, 640), (4096, 1280), (77, 768), (33, 2048), (5, 5120), (1001, 320),
                                    (37, 512), (16384, 640), (3, 4096), (70, 1024)])
def test_layernorm(cuda, rows, C):
    torch.manual_seed(0)
    x = (torch.randn(rows, C, device=cuda) * 2 + 0.5).to(torch.bfloat16)
    w = torch.randn(C, device=cuda).to(torch.bfloat16)
    b = torch.randn(C, device=cuda).to(torch.bfloat16)
    y = ops.layer_norm(x, w, b, 1e-5)
    ref = F.layer_norm(x.float(), (C,), w.float(), b.float(), 1e-5)
    assert ops.stats().get(("layernorm", "hip"), 0) == 1
    assert _rel(y, ref) < 1e-2


@pytest.mark.parametrize("B,H,Sq,Sk,D", [(2, 10, 256, 256, 64), (2, 20, 100, 77, 64), (1, 8, 300, 300, 40),
                                         (2, 8, 128, 77, 80), (1, 8, 64, 64, 160), (1, 4, 96, 200, 128)])
def test_flash_attention(cuda, B, H, Sq, Sk, D):
    torch.manual_seed(0)
    q = torch.randn(B, Sq, H * D, device=cuda).to(torch.bfloat16)
    k = torch.randn(B, Sk, H * D, device=cuda).to(torch.bfloat16)
    v = torch.randn(B, Sk, H * D, device=cuda).to(torch.bfloat16)
    o = ops.attention(q, k, v, H)
    ref = core.attention_reference(q.float(), k.float(), v.float(), H)
    assert ops.stats().get(("attention", "hip"), 0) == 1
    assert _rel(o, ref) < 2e-2


def test_flash_attention_strided_qkv(cuda):
    """q, k, v as views of one fused QKV projection (stride 3C), as the UNet uses them."""
    torch.manual_seed(1)
    B, S, H, D = 2, 200, 5, 64
    qkv = torch.randn(B, S, 3 * H * D, device=cuda).to(torch.bfloat16)
    C = H * D
    q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
    o = ops.attention(q, k, v, H)
    ref = core.attention_reference(q.float(), k.float(), v.float(), H)
    assert _rel(o, ref) < 2e-2


def test_flash_attention_causal_and_spike(cuda):
    """Causal CLIP mask + a spiked key forcing large running-max jumps (rescale path)."""
    torch.manual_seed(2)
    B, S, H, D = 2, 77, 12, 64
    q = torch.randn(B, S, H * D, device=cuda)
    k = torch.randn(B, S, H * D, device=cuda)
    k[:, 70, :] *= 8.0
    v = torch.randn(B, S, H * D, device=cuda)
    q, k, v = (t.to(torch.bfloat16) for t in (q, k, v))
    o = ops.attention(q, k, v, H, causal=True)
    ref = core.attention_reference(q.float(), k.float(), v.float(), H, causal=True)
    assert _rel(o, ref) < 2e-2


@pytest.mark.parametrize("Bw,H,Sq,Sk,D,nW,kind", [
    (32, 6, 64, 64, 30, 4, "float"),       # SwinIR / HAT: 8x8 windows, head dim 30 (zero-padded), shift mask
    (8, 6, 256, 576, 30, 0, "none"),       # HAT overlapping cross-attention: 16x16 queries, 24x24 keys
    (16, 4, 64, 64, 32, 8, "bool"),        # SCUNet: -inf blocks from a bool mask
    (6, 3, 64, 64, 60, 2, "v2"),           # Swin2SR: cosine scores x per-head logit scale
    (2, 2, 130, 130, 64, 0, "none"),       # ragged query / key tiles
])
def test_attention_bias(cuda, Bw, H, Sq, Sk, D, nW, kind):
    """Additive bias + window mask in the flash kernel's softmax vs the fp32 math of the Swin models."""
    torch.manual_seed(3)
    q = torch.randn(Bw, H, Sq, D, device=cuda)
    k = torch.randn(Bw, H, Sk, D, device=cuda)
    v = torch.randn(Bw, H, Sk, D, device=cuda)
    bias = torch.randn(H, Sq, Sk, device=cuda) * 2
    hs = None
    if kind == "v2":
        q, k = F.normalize(q, dim=-1), F.normalize(k, dim=-1)
        hs = torch.tensor([10.0, 25.0, 100.0], device=cuda)
    q, k, v = (t.to(torch.bfloat16) for t in (q, k, v))
    mask = None
    if kind == "float":
        mask = torch.where(torch.rand(nW, Sq, Sk, device=cuda) < 0.3, -100.0, 0.0)
    elif kind == "bool":
        mask = torch.rand(nW, Sq, Sk, device=cuda) < 0.4
        mask[..., 0] = False                                  # every query keeps a key
    scale = 1.0 if kind == "v2" else D ** -0.5
    o = ops.attention_bias(q, k, v, bias, mask, scale=scale, head_scale=hs)
    assert ops.stats().get(("attention", "hip"), 0) == 1
    s = (q.float() @ k.float().transpose(-2, -1)) * scale
    if hs is not None:
        s = s * hs[:, None, None]
    s = s + bias
    if mask is not None:
        m = mask if mask.dtype != torch.bool else torch.zeros(mask.shape, device=cuda).masked_fill(mask, -math.inf)
        s = (s.view(Bw // nW, nW, H, Sq, Sk) + m[None, :, None]).view(Bw, H, Sq, Sk)
    ref = torch.softmax(s, -1) @ v.float()
    assert o.shape == ref.shape
    assert _rel(o, ref) < 2e-2


@pytest.mark.parametrize("N,H,W,C,k,rep", [(2, 24, 24, 64, 3, False), (1, 17, 9, 2048, 3, False),
                                            (1, 32, 31, 192, 3, True), (2, 8, 8, 16, 5, False),
                                            (1, 4, 8, 2048, 3, False), (3, 5, 12, 8, 3, False),
                                            (1, 1, 4, 24, 3, False), (2, 24, 24, 2048, 3, True),
                                            (2, 6, 6, 64, 3, False)])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_depthwise_conv_nhwc(cuda, N, H, W, C, k, rep, dt):
    """W % 4 == 0 zero-padded 3 x 3 maps run the four-pixel kernel, the rest the one-pixel kernel."""
    torch.manual_seed(0)
    x = torch.randn(N, H, W, C, device=cuda).to(dt)
    w = torch.randn(C, 1, k, k, device=cuda).to(dt)
    b = torch.randn(C, device=cuda).to(dt)
    y = ops.depthwise_conv2d_nhwc(x, w.reshape(C, k * k).t().contiguous(), b, k, replicate=rep)
    xn = x.float().permute(0, 3, 1, 2)
    if rep:
        ref = F.conv2d(F.pad(xn, (k // 2,) * 4, mode="replicate"), w.float(), b.float(), groups=C)
    else:
        ref = F.conv2d(xn, w.float(), b.float(), padding=k // 2, groups=C)
    assert ops.stats().get(("dwconv", "hip"), 0) == 1
    assert _rel(y.permute(0, 3, 1, 2), ref) < 1e-2


def test_depthwise_conv_pixels_per_thread_knob(cuda):
    """The 2 / 4 output-pixels-per-thread forms of the 3 x 3 depthwise kernel agree bit for bit (the same fma
    order per output) and with the one-pixel kernel to bf16 rounding."""
    from comfy_gen_server_amd import _native
    lib = _native.load_kernels()
    torch.manual_seed(0)
    x = torch.randn(2, 12, 16, 256, device=cuda).to(torch.bfloat16)
    w = torch.randn(9, 256, device=cuda).to(torch.bfloat16)
    b = torch.randn(256, device=cuda).to(torch.bfloat16)
    outs = []
    try:
        for p in (1, 2, 4):
            lib.cgs_dwconv_set_px(p)
            outs.append(ops.depthwise_conv2d_nhwc(x, w, b, 3))
    finally:
        lib.cgs_dwconv_set_px(4)
    assert torch.equal(outs[1], outs[2])
    assert _rel(outs[0], outs[2]) < 1e-2


@pytest.mark.parametrize("ks", ["d64ks2", "d64ks4"])
@pytest.mark.parametrize("B,H,Sq,Sk,fused", [(2, 20, 1024, 1024, True), (2, 10, 4096, 4096, True),
                                             (1, 8, 700, 1000, False), (2, 8, 333, 1100, False)])
def test_attention_key_split(cuda, B, H, Sq, Sk, fused, ks, monkeypatch):
    """D = 64 self-attention with the keys split 2 / 4 ways and the partials merged by log-sum-exp (the
    small-grid candidates of ops.attention), forced through the tuning override, vs the fp32 reference;
    q / k / v as column views of one fused QKV projection where Sq == Sk."""
    import json
    torch.manual_seed(4)
    C = H * 64
    if fused:
        qkv = torch.randn(B, Sq, 3 * C, device=cuda).to(torch.bfloat16)
        q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
    else:
        q = torch.randn(B, Sq, C, device=cuda).to(torch.bfloat16)
        k = torch.randn(B, Sk, C, device=cuda).to(torch.bfloat16)
        v = torch.randn(B, Sk, C, device=cuda).to(torch.bfloat16)
    monkeypatch.setenv("CGS_AUTOTUNE", "1")
    monkeypatch.setenv("CGS_TUNE_OVERRIDE", json.dumps({f"attention_grid2|{B}|{H}|{Sq}|{Sk}|64": ks}))
    calls = []
    lib = _native.load_kernels()
    real = lib.cgs_flash_attn_fwd_ks
    monkeypatch.setattr(lib, "cgs_flash_attn_fwd_ks", lambda *a: calls.append(a[17]) or real(*a))
    o = ops.attention(q, k, v, H)
    assert calls == [int(ks[-1])]
    assert _rel(o, core.attention_reference(q.float(), k.float(), v.float(), H)) < 2e-2


def test_layernorm_no_affine(cuda):
    x = torch.randn(300, 2048, device=cuda).to(torch.bfloat16)
    y = ops.layer_norm(x, None, None, 1e-6)
    assert ops.stats().get(("layernorm", "hip"), 0) == 1
    assert _rel(y, F.layer_norm(x.float(), (2048,), eps=1e-6)) < 1e-2


@pytest.fixture(params=[1, 2, 3, 4], ids=["generic", "d64fast", "shortkv", "d64r2"])
def attn_variant(request):
    lib = _native.load_kernels()
    lib.cgs_attn_set_variant(request.param)
    yield request.param
    lib.cgs_attn_set_variant(0)


@pytest.mark.parametrize("B,H,Sq,Sk", [(2, 10, 256, 256), (1, 3, 300, 77), (2, 2, 1000, 1000), (1, 2, 4096, 4096),
                                       (1, 1, 64, 1), (2, 3, 513, 130), (2, 5, 1024, 77), (1, 4, 129, 96),
                                       (3, 2, 200, 33), (1, 2, 77, 128), (2, 2, 130, 4)])
@pytest.mark.parametrize("spike", [False, True])
def test_attention_d64_variants(cuda, attn_variant, B, H, Sq, Sk, spike):
    """D=64 fast kernel vs the generic kernel vs fp32 reference: tails in Sq (256-row blocks) and Sk
    (64-key tiles), and spiked late keys that force running-max rescales mid-sequence."""
    if attn_variant == 3 and Sk > 128:
        pytest.skip("short-KV kernel covers Sk <= 128")
    torch.manual_seed(3)
    D = 64
    q = torch.randn(B, Sq, H * D, device=cuda)
    k = torch.randn(B, Sk, H * D, device=cuda)
    v = torch.randn(B, Sk, H * D, device=cuda)
    if spike:
        q *= 3.0
        for j in range(Sk // 3, Sk, max(1, Sk // 5)):
            k[:, j, :] *= 1.0 + 0.5 * (j * 7 % 11)
    q, k, v = (t.to(torch.bfloat16) for t in (q, k, v))
    o = ops.attention(q, k, v, H)
    ref = core.attention_reference(q.float(), k.float(), v.float(), H)
    assert ops.stats().get(("attention", "hip"), 0) == 1
    assert torch.isfinite(o).all()
    assert _rel(o, ref) < 2e-2


@pytest.fixture(params=[1, 2, 3, 4, 5, 6, 7, 8, 10, 11, 12, 13, 14],
                ids=["v1", "v2", "v3w4", "v3w8", "v5pp", "v6pp160", "v7ppk", "v8t128", "v10t64x128", "v11t128x64",
                     "v12t64x128s6", "v13t128x64s6", "v14t128s5"])
def gemm_variant(request):
    lib = _native.load_kernels()
    lib.cgs_gemm_set_variant(request.param)
    yield request.param
    lib.cgs_gemm_set_variant(-1)


@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (300, 320, 640), (154, 1280, 2048), (4096, 1280, 1280),
                                   (77, 768, 768), (2, 1280, 2816), (1000, 640, 320), (512, 3840, 1280),
                                   (1100, 328, 96), (513, 2560, 32), (700, 1280, 640), (2048, 2048, 2048)])
@pytest.mark.parametrize("epi", ["none", "bias", "bias_res"])
def test_gemm(cuda, M, N, K, epi, gemm_variant):
    torch.manual_seed(0)
    a = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    w = (torch.randn(N, K, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    b = torch.randn(N, device=cuda).to(torch.bfloat16) if epi != "none" else None
    r = torch.randn(M, N, device=cuda).to(torch.bfloat16) if epi == "bias_res" else None
    y = ops.linear(a, w, b, residual=r)
    ref = a.float() @ w.float().t()
    if b is not None:
        ref = ref + b.float()
    if r is not None:
        ref = ref + r.float()
    assert ops.stats().get(("gemm", "hip"), 0) == 1
    assert _rel(y, ref) < 1e-2


@pytest.mark.parametrize("M,N2,K", [(256, 512, 128), (333, 2560, 320), (64, 10240, 1280), (600, 10240, 1280)])
def test_gemm_geglu(cuda, M, N2, K, gemm_variant):
    torch.manual_seed(0)
    a = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    w = (torch.randn(N2, K, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    b = torch.randn(N2, device=cuda).to(torch.bfloat16)
    y = ops.linear_geglu(a, core.geglu_interleave(w), core.geglu_interleave(b))
    h = a.float() @ w.float().t() + b.float()
    x1, g = h.chunk(2, dim=-1)
    ref = x1 * F.gelu(g)
    assert ops.stats().get(("gemm_geglu", "hip"), 0) == 1
    assert _rel(y, ref) < 1e-2


def test_elementwise(cuda):
    torch.manual_seed(0)
    x = torch.randn(1000, 40, device=cuda).to(torch.bfloat16)
    assert _rel(ops.silu(x), F.silu(x.float())) < 1e-2
    t = torch.tensor([1.0, 500.0, 999.0], device=cuda)
    e = ops.timestep_embedding(t, 320)
    half = 160
    freqs = torch.exp(-math.log(10000.0) * torch.arange(half, device=cuda) / half)
    args = t[:, None] * freqs[None]
    ref = torch.cat([torch.cos(args), torch.sin(args)], -1)
    assert (e - ref).abs().max().item() < 2e-3
    c = torch.randn(2, 4, 16, 16, device=cuda)
    u = torch.randn(2, 4, 16, 16, device=cuda)
    assert torch.allclose(ops.cfg_combine(c, u, 7.5), u + (c - u) * 7.5, atol=1e-5)
    xx = torch.randn(2, 4, 16, 16, device=cuda)
    den = torch.randn(2, 4, 16, 16, device=cuda)
    nz = torch.randn(2, 4, 16, 16, device=cuda)
    out = ops.euler_step(xx, den, nz, 3.0, 2.0, 0.5)
    ref = xx + (xx - den) / 3.0 * (2.0 - 3.0) + nz * 0.5
    assert torch.allclose(out, ref, atol=1e-5)
    im = torch.randn(2, 64, 8, 8, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    up = ops.upsample_nearest2x(im)
    assert torch.equal(up, F.interpolate(im, scale_factor=2.0, mode="nearest"))


@pytest.fixture(params=[2, 3, 4, 5, 6, 7, 8, 18, 21],
                ids=["cv2", "cv3w4", "cv3w8", "cv5pp", "cv6pp160", "cv7ppk", "cv8t128", "cv6n128", "cv6w4"])
def conv_variant(request):
    lib = _native.load_kernels()
    lib.cgs_conv_set_variant(request.param)
    yield request.param
    lib.cgs_conv_set_variant(-1)


@pytest.mark.parametrize("N,Cin,H,W,Cout,k,s,p", [(2, 64, 16, 16, 64, 3, 1, 1), (2, 320, 32, 32, 320, 3, 1, 1),
                                                  (1, 640, 16, 16, 1280, 3, 1, 1), (2, 320, 32, 32, 320, 3, 2, 1),
                                                  (1, 128, 7, 9, 256, 1, 1, 0), (3, 256, 11, 5, 4, 3, 1, 1),
                                                  (1, 1920, 8, 8, 1280, 1, 1, 0), (2, 512, 12, 12, 3, 3, 1, 1),
                                                  (2, 96, 20, 20, 160, 3, 1, 1), (1, 320, 33, 17, 640, 3, 2, 1)])
@pytest.mark.parametrize("epi", ["bias", "bias_res", "none"])
def test_conv2d(cuda, N, Cin, H, W, Cout, k, s, p, epi, conv_variant):
    if conv_variant in (2, 5, 6, 18, 21) and Cin % 64:
        pytest.skip("v2/v5/v6 need Cin % 64")
    torch.manual_seed(0)
    x = torch.randn(N, Cin, H, W, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Cout, Cin, k, k, device=cuda) / math.sqrt(Cin * k * k)).to(torch.bfloat16)
    b = torch.randn(Cout, device=cuda).to(torch.bfloat16) if epi != "none" else None
    ref = F.conv2d(x.float(), w.float(), None if b is None else b.float(), s, p)
    r = None
    if epi == "bias_res":
        r = torch.randn_like(ref).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        ref = ref + r.float()
    y = ops.conv2d(x, w, b, s, p, residual=r, weight_nhwc=w.permute(0, 2, 3, 1).contiguous())
    assert ops.stats().get(("conv", "hip"), 0) == 1
    assert y.shape == ref.shape
    assert _rel(y, ref) < 1e-2


# The SDXL VAE decoder's largest convs at 1024^2 (the bench runs 8 images; 1 here): 128 / 256 channels at
# full resolution, the 256-channel upsample conv (nearest 2x fused into the gather) and the 512 -> 256 one.
@pytest.mark.parametrize("Cin,H,Cout,up", [(128, 1024, 128, False), (256, 1024, 128, False), (256, 512, 256, True),
                                           (512, 512, 256, False)])
def test_conv2d_vae_production_shapes(cuda, Cin, H, Cout, up):
    torch.manual_seed(1)
    x = torch.randn(1, Cin, H, H, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Cout, Cin, 3, 3, device=cuda) / math.sqrt(Cin * 9)).to(torch.bfloat16)
    b = torch.randn(Cout, device=cuda).to(torch.bfloat16)
    xr = F.interpolate(x.float(), scale_factor=2.0, mode="nearest") if up else x.float()
    ref = F.conv2d(xr, w.float(), b.float(), 1, 1)
    y = ops.conv2d(x, w, b, 1, 1, weight_nhwc=w.permute(0, 2, 3, 1).contiguous(), upsample2x=up)
    assert ops.stats().get(("conv", "hip"), 0) == 1 and ops.stats().get(("conv", "lib"), 0) == 0
    assert y.shape == ref.shape
    assert _rel(y, ref) < 1e-2


@pytest.mark.parametrize("N,C,H,W,Cout", [(2, 320, 8, 8, 320), (1, 640, 5, 7, 640), (2, 128, 16, 16, 128)])
def test_conv2d_fused_upsample(cuda, N, C, H, W, Cout, conv_variant):
    torch.manual_seed(0)
    x = torch.randn(N, C, H, W, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Cout, C, 3, 3, device=cuda) / math.sqrt(C * 9)).to(torch.bfloat16)
    b = torch.randn(Cout, device=cuda).to(torch.bfloat16)
    ref = F.conv2d(F.interpolate(x.float(), scale_factor=2.0, mode="nearest"), w.float(), b.float(), 1, 1)
    y = ops.conv2d(x, w, b, 1, 1, weight_nhwc=w.permute(0, 2, 3, 1).contiguous(), upsample2x=True)
    assert ops.stats().get(("conv", "hip"), 0) == 1
    assert y.shape == ref.shape
    assert _rel(y, ref) < 1e-2


def test_autotuned_ops_match_reference(cuda, monkeypatch):
    """With the measured dispatch on, whatever candidate wins must still be numerically right."""
    from comfy_gen_server_amd.ops import autotune
    monkeypatch.setenv("CGS_AUTOTUNE", "1")
    autotune.reset()
    torch.manual_seed(0)
    M, N, K = 4096, 1280, 1280
    a = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    w = (torch.randn(N, K, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    b = torch.randn(N, device=cuda).to(torch.bfloat16)
    r = torch.randn(M, N, device=cuda).to(torch.bfloat16)
    y = ops.linear(a, w, b, residual=r)
    assert _rel(y, a.float() @ w.float().t() + b.float() + r.float()) < 1e-2
    x = torch.randn(4, 320, 64, 64, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    cw = (torch.randn(320, 320, 3, 3, device=cuda) / math.sqrt(320 * 9)).to(torch.bfloat16)
    yc = ops.conv2d(x, cw, None, 1, 1, weight_nhwc=cw.permute(0, 2, 3, 1).contiguous())
    assert _rel(yc, F.conv2d(x.float(), cw.float(), None, 1, 1)) < 1e-2
    q = torch.randn(4, 1024, 640, device=cuda).to(torch.bfloat16)
    o = ops.attention(q, q, q, 10)
    assert _rel(o, core.attention_reference(q.float(), q.float(), q.float(), 10)) < 2e-2
    t = autotune.table()
    assert any(k.startswith("gemm|") for k in t) and any(k.startswith("conv|") for k in t)


@pytest.mark.parametrize("B,S,Sk", [(1, 1024, 1024), (2, 300, 300), (1, 64, 4096), (3, 33, 77), (1, 4096, 4096)])
def test_attention_wide_d512(cuda, B, S, Sk):
    """K22: single-head D=512 VAE mid-block attention (head dim split over 4 waves, partial scores
    summed through LDS) vs the fp32 reference, incl. query/key tails and a spiked key."""
    torch.manual_seed(5)
    D = 512
    q = torch.randn(B, S, D, device=cuda) * 0.5
    k = torch.randn(B, Sk, D, device=cuda) * 0.5
    v = torch.randn(B, Sk, D, device=cuda)
    k[:, Sk // 2, :] *= 3.0
    q, k, v = (t.to(torch.bfloat16) for t in (q, k, v))
    o = ops.attention(q, k, v, 1)
    ref = core.attention_reference(q.float(), k.float(), v.float(), 1)
    assert ops.stats().get(("attention", "hip"), 0) == 1
    assert torch.isfinite(o).all()
    assert _rel(o, ref) < 2e-2


@pytest.mark.parametrize("B,S,chunk", [(2, 4096, 1 << 28), (1, 4096, 1000 * 4096), (1, 16384, 1 << 28)])
def test_attention_wide_materialised(cuda, B, S, chunk, monkeypatch):
    """K22 v2: fp32 scores on the v7 GEMM (MC_EPI_F32OUT) -> one-pass softmax2 -> P (V^T)^T on the
    v7 GEMM, over q/k/v that are strided views of one fused QKV tensor (the VAE AttnBlock layout),
    with query chunks (incl. a partial last chunk) vs the fp32 reference."""
    monkeypatch.setattr(core, "_WIDE_CHUNK_ELEMS", chunk)
    torch.manual_seed(9)
    D = 512
    qkv = (torch.randn(B, S, 3 * D, device=cuda) * 0.6).to(torch.bfloat16)
    qkv[:, S // 3, D:2 * D] *= 4.0          # a spiked key
    q, k, v = qkv[..., :D], qkv[..., D:2 * D], qkv[..., 2 * D:]
    o = ops.attention(q, k, v, 1)
    assert ops.stats().get(("attention", "hip"), 0) == 1
    rows = torch.arange(0, S, 7, device=cuda)[:512]      # reference on a row subset (S x S fp32 per image)
    ref = core.attention_reference(q[:, rows].float(), k.float(), v.float(), 1)
    assert torch.isfinite(o).all()
    assert _rel(o[:, rows], ref) < 2e-2


@pytest.mark.parametrize("B,H,S,Sk,D", [(2, 10, 1024, 1024, 64), (1, 4, 300, 77, 64), (2, 5, 200, 333, 80),
                                        (1, 2, 130, 64, 40)])
def test_attention_lse_and_ring_merge(cuda, B, H, S, Sk, D):
    """Flash kernels with the LSE output (ring attention partials): o and lse vs fp32 torch, and two
    K/V halves merged by parallel/sp.py's log-sum-exp rule == attention over the whole K/V."""
    from comfy_gen_server_amd.parallel import sp
    torch.manual_seed(11)
    q = torch.randn(B, S, H * D, device=cuda).to(torch.bfloat16)
    k = torch.randn(B, Sk, H * D, device=cuda).to(torch.bfloat16)
    v = torch.randn(B, Sk, H * D, device=cuda).to(torch.bfloat16)
    o, lse = ops.attention_lse(q, k, v, H)
    assert ops.stats().get(("attention", "hip"), 0) == 1
    qh = q.float().view(B, S, H, D).transpose(1, 2)
    kh = k.float().view(B, Sk, H, D).transpose(1, 2)
    s = (qh @ kh.transpose(-1, -2)) * D ** -0.5
    assert (lse - torch.logsumexp(s, -1)).abs().max().item() < 2e-2
    assert _rel(o, core.attention_reference(q.float(), k.float(), v.float(), H)) < 2e-2
    h = Sk // 2
    o1, l1 = sp._partial_attention(q, k[:, :h], v[:, :h], H)
    o2, l2 = sp._partial_attention(q, k[:, h:], v[:, h:], H)
    m = torch.maximum(l1, l2)
    wa, wb = torch.exp(l1 - m), torch.exp(l2 - m)
    merged = ((o1 * wa + o2 * wb) / (wa + wb)).reshape(B, S, H * D)
    assert _rel(merged, core.attention_reference(q.float(), k.float(), v.float(), H)) < 2e-2


@pytest.mark.parametrize("B,H,S,Sk", [(1, 20, 1024, 1024), (2, 10, 4096, 4096), (1, 3, 300, 77), (1, 5, 1000, 333),
                                      (2, 2, 129, 1000)])
@pytest.mark.parametrize("variant", [2, 5])
def test_attention_d64_q_block_forms(cuda, B, H, S, Sk, variant):
    """D = 64 fast kernel with 256-row (variant 2, 8 waves) and 128-row (variant 5, 4 waves, two WGs
    per CU: the batch-1 form) Q blocks vs the fp32 reference."""
    torch.manual_seed(5)
    D = 64
    q = torch.randn(B, S, H * D, device=cuda).to(torch.bfloat16)
    k = torch.randn(B, Sk, H * D, device=cuda).to(torch.bfloat16)
    v = torch.randn(B, Sk, H * D, device=cuda).to(torch.bfloat16)
    o = torch.empty_like(q)
    lib = core._lib()
    st = lambda t, L: (L * H * D, H * D, D)   # noqa: E731  (batch, seq, head) strides in elements
    rc = lib.cgs_flash_attn_fwd_v(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), B, H, S, Sk, D,
                                  *st(q, S), *st(k, Sk), *st(v, Sk), *st(o, S), D ** -0.5, variant, core._stream())
    assert rc == 0
    assert _rel(o, core.attention_reference(q.float(), k.float(), v.float(), H)) < 2e-2


def test_softmax2_and_transpose_kernels(cuda):
    lib = core._lib()
    x = torch.randn(37, 5000, device=cuda) * 6
    y = torch.empty(37, 5000, device=cuda, dtype=torch.bfloat16)
    assert lib.cgs_softmax2_f32_bf16(x.data_ptr(), y.data_ptr(), 37, 5000, 5000, 5000, core._stream()) == 0
    ref = torch.softmax(x * math.log(2.0), dim=-1)
    assert (y.float() - ref).abs().max().item() < 4e-3 * ref.max().item() + 1e-6
    assert torch.allclose(y.float().sum(-1), torch.ones(37, device=cuda), atol=2e-2)
    a = torch.randn(200, 72, device=cuda).to(torch.bfloat16)
    t = torch.empty(72, 200, device=cuda, dtype=torch.bfloat16)
    assert lib.cgs_transpose_bf16(a.data_ptr(), t.data_ptr(), 200, 72, 72, 200, core._stream()) == 0
    assert torch.equal(t, a.t())


def test_vae_mid_attention_block_native(cuda):
    """The VAE AttnBlock runs fused-QKV GEMM + the D=512 kernel + out-proj GEMM (no SDPA)."""
    from comfy_gen_server_amd.models.layers import init_random_
    from comfy_gen_server_amd.models.vae import AttnBlock
    m = AttnBlock(512)
    init_random_(m, seed=3)
    x = torch.randn(2, 512, 24, 24)
    with torch.no_grad():
        ref = m(x)
        md = AttnBlock(512, dtype=torch.bfloat16, device=cuda)
        md.load_state_dict(m.state_dict())
        out = md(x.to(cuda, torch.bfloat16).contiguous(memory_format=torch.channels_last))
    st = ops.stats()
    assert st.get(("attention", "hip"), 0) == 1 and st.get(("attention", "lib"), 0) == 0, st
    assert _rel(out.cpu(), ref) < 2e-2


@pytest.mark.parametrize("M,N,K", [(256, 640, 640), (77, 1280, 2048), (1000, 333 * 8, 96)])
@pytest.mark.parametrize("epi", ["none", "bias", "bias_res"])
def test_gemm_fp8_weights(cuda, M, N, K, epi):
    """K21: bf16 activations x fp8-e4m3fn weights; the kernel's in-register widening is exact, so the
    result matches the GEMM on the upcast weights (fp32 reference)."""
    torch.manual_seed(4)
    x = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    w8 = (torch.randn(N, K, device=cuda) * 0.5).to(torch.float8_e4m3fn)
    b = torch.randn(N, device=cuda).to(torch.bfloat16) if epi != "none" else None
    r = torch.randn(M, N, device=cuda).to(torch.bfloat16) if epi == "bias_res" else None
    y = ops.linear(x, w8, b, residual=r)
    assert ops.stats().get(("gemm_w8", "hip"), 0) == 1
    ref = x.float() @ w8.float().t()
    if b is not None:
        ref = ref + b.float()
    if r is not None:
        ref = ref + r.float()
    assert _rel(y, ref) < 1e-2


def test_fp8_e4m3_decode_rule_is_exact():
    """The kernel's e4m3fn -> bf16 bit rule reproduces torch's own cast for every non-NaN byte."""
    idx = torch.arange(256)
    ref = torch.arange(256, dtype=torch.uint8).view(torch.float8_e4m3fn).float().to(torch.bfloat16)
    ref = ref.view(torch.int16).int() & 0xFFFF
    s, e, m = (idx & 0x80) << 8, (idx >> 3) & 15, idx & 7
    mag = torch.where(e > 0, ((e + 120) << 7) | (m << 4), (m.float() * 0.001953125).view(torch.int32) >> 16)
    nan = (idx & 0x7F) == 0x7F
    assert torch.equal((s | mag)[~nan], ref[~nan])


# The SDXL bench shapes (UNet batch 16 at 1024^2): 64x64 tokens x 640 ch and 32x32 x 1280 ch.
@pytest.mark.parametrize("M,N,K,epi", [(65536, 1920, 640, "none"), (65536, 640, 640, "bias_res"),
                                       (16384, 3840, 1280, "none"), (16384, 1280, 1280, "bias_res"),
                                       (16384, 1280, 5120, "bias_res"), (1232, 2560, 2048, "none")])
@pytest.mark.parametrize("variant", [5, 6, 7])
def test_gemm_bench_shapes(cuda, M, N, K, epi, variant):
    lib = _native.load_kernels()
    lib.cgs_gemm_set_variant(variant)
    try:
        torch.manual_seed(0)
        a = torch.randn(M, K, device=cuda).to(torch.bfloat16)
        w = (torch.randn(N, K, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
        b = torch.randn(N, device=cuda).to(torch.bfloat16) if epi != "none" else None
        r = torch.randn(M, N, device=cuda).to(torch.bfloat16) if epi == "bias_res" else None
        y = ops.linear(a, w, b, residual=r)
        ref = a.float() @ w.float().t()
        if b is not None:
            ref += b.float()
        if r is not None:
            ref += r.float()
        assert ops.stats().get(("gemm", "hip"), 0) == 1
        assert _rel(y, ref) < 1e-2
    finally:
        lib.cgs_gemm_set_variant(-1)


@pytest.mark.parametrize("M,N2,K", [(65536, 5120, 640), (16384, 10240, 1280)])
@pytest.mark.parametrize("variant", [5, 7])
def test_gemm_geglu_bench_shapes(cuda, M, N2, K, variant):
    lib = _native.load_kernels()
    lib.cgs_gemm_set_variant(variant)
    try:
        torch.manual_seed(0)
        a = torch.randn(M, K, device=cuda).to(torch.bfloat16)
        w = (torch.randn(N2, K, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
        b = torch.randn(N2, device=cuda).to(torch.bfloat16)
        y = ops.linear_geglu(a, core.geglu_interleave(w), core.geglu_interleave(b))
        h = a.float() @ w.float().t() + b.float()
        x1, g = h.chunk(2, dim=-1)
        ref = x1 * F.gelu(g)
        assert ops.stats().get(("gemm_geglu", "hip"), 0) == 1
        assert _rel(y, ref) < 1e-2
    finally:
        lib.cgs_gemm_set_variant(-1)


@pytest.mark.parametrize("N,C1,C2,H,W", [(2, 1280, 1280, 16, 16), (2, 1280, 640, 16, 16), (1, 640, 320, 32, 24),
                                         (3, 320, 320, 8, 8)])
def test_groupnorm_dual_source(cuda, N, C1, C2, H, W):
    """GroupNorm of cat([a, b], 1) read from both tensors (K14), groups straddling the seam included."""
    torch.manual_seed(0)
    a = (torch.randn(N, C1, H, W, device=cuda) * 2 + 0.5).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    b = (torch.randn(N, C2, H, W, device=cuda) - 1).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = torch.randn(C1 + C2, device=cuda).to(torch.bfloat16)
    bb = torch.randn(C1 + C2, device=cuda).to(torch.bfloat16)
    y = ops.group_norm(a, 32, w, bb, 1e-5, silu=True, x2=b)
    ref = F.silu(F.group_norm(torch.cat([a, b], 1).float(), 32, w.float(), bb.float(), 1e-5))
    assert ops.stats().get(("groupnorm", "hip"), 0) == 1
    assert _rel(y, ref) < 1e-2


@pytest.mark.parametrize("C1,C2,Cout,k", [(1280, 1280, 1280, 3), (1280, 640, 640, 1), (640, 320, 320, 3), (320, 320, 320, 1)])
def test_conv_dual_source(cuda, C1, C2, Cout, k, conv_variant):
    torch.manual_seed(0)
    a = torch.randn(2, C1, 16, 16, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    b = torch.randn(2, C2, 16, 16, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Cout, C1 + C2, k, k, device=cuda) / math.sqrt((C1 + C2) * k * k)).to(torch.bfloat16)
    bias = torch.randn(Cout, device=cuda).to(torch.bfloat16)
    y = ops.conv2d(a, w, bias, 1, k // 2, weight_nhwc=w.permute(0, 2, 3, 1).contiguous(), x2=b)
    ref = F.conv2d(torch.cat([a, b], 1).float(), w.float(), bias.float(), 1, k // 2)
    assert ops.stats().get(("conv", "hip"), 0) == 1
    assert _rel(y, ref) < 1e-2


def test_unet_skip_concat_never_materialised(cuda):
    """The decoder ResBlocks consume the skip concat as two tensors (SkipCat): the device forward
    matches the fp32 CPU forward of the same weights (which concatenates)."""
    import copy
    from comfy_gen_server_amd.models.layers import init_random_fast_
    from comfy_gen_server_amd.models.unet import UNetModel
    cfg = dict(in_channels=4, model_channels=128, out_channels=4, num_res_blocks=[1, 1], channel_mult=[1, 2],
               transformer_depth=[0, 1], transformer_depth_output=[0, 0, 1, 1], transformer_depth_middle=1,
               num_heads=-1, num_head_channels=64, use_linear_in_transformer=True, context_dim=128)
    with torch.inference_mode():
        m = UNetModel(**cfg, dtype=torch.bfloat16, device=cuda)
        init_random_fast_(m, seed=4)
        cpu = copy.deepcopy(m).float().cpu()
        g = torch.Generator().manual_seed(0)
        x = torch.randn(2, 4, 16, 16, generator=g)
        t = torch.tensor([700.0, 30.0])
        c = torch.randn(2, 12, 128, generator=g)
        yd = m(x.to(cuda, torch.bfloat16).contiguous(memory_format=torch.channels_last), t.to(cuda),
               context=c.to(cuda, torch.bfloat16), transformer_options={})
        yc = cpu(x, t, context=c, transformer_options={})
    assert _rel(yd.float().cpu(), yc) < 3e-2


# v7 split-K tail (mfma_ppk.h): shapes whose last round of 256x256 tiles is at most half full get
# their tail tiles cut into K ranges, reduced by the last-arriving unit of each tile.
@pytest.mark.parametrize("M,N,K,epi", [(16384, 1280, 5120, "bias_res"), (16384, 1280, 5120, "bias"),
                                       (1024, 1024, 8192, "none"), (4096, 1280, 5120, "bias"),
                                       (16200, 1288, 5120, "bias_res")])
def test_gemm_v7_split_tail(cuda, M, N, K, epi):
    lib = _native.load_kernels()
    ws_bytes = lib.cgs_v7_ws_bytes(M, N, K)
    assert ws_bytes > 0, "shape chosen to exercise the split tail"
    torch.manual_seed(0)
    a = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    w = (torch.randn(N, K, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    b = torch.randn(N, device=cuda).to(torch.bfloat16) if epi != "none" else None
    r = torch.randn(M, N, device=cuda).to(torch.bfloat16) if epi == "bias_res" else None
    flags = (1 if b is not None else 0) | (2 if r is not None else 0)
    ws = torch.full((ws_bytes,), 0x7F, dtype=torch.uint8, device=cuda)   # garbage counters / partials
    outs = []
    for _ in range(2):                                                   # counters self-consistent on reuse
        y = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
        assert lib.cgs_gemm_bf16_v7ws(a.data_ptr(), w.data_ptr(), y.data_ptr(), None if b is None else b.data_ptr(),
                                      None if r is None else r.data_ptr(), M, N, K, K, K, N, N if r is not None else 0,
                                      flags, 1.0, ws.data_ptr(), ws_bytes, core._stream()) == 0
        outs.append(y)
    torch.cuda.synchronize()
    ref = a.float() @ w.float().t()
    if b is not None:
        ref += b.float()
    if r is not None:
        ref += r.float()
    assert _rel(outs[0], ref) < 1e-2
    assert torch.equal(outs[0], outs[1]) or _rel(outs[1], ref) < 1e-2


@pytest.mark.parametrize("M,N2,K", [(16384, 2560, 5120), (1024, 5120, 5120)])
def test_gemm_v7_split_tail_geglu(cuda, M, N2, K):
    lib = _native.load_kernels()
    ws_bytes = lib.cgs_v7_ws_bytes(M, N2, K)
    assert ws_bytes > 0
    torch.manual_seed(0)
    a = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    w = (torch.randn(N2, K, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    b = torch.randn(N2, device=cuda).to(torch.bfloat16)
    wi, bi = core.geglu_interleave(w), core.geglu_interleave(b)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=cuda)
    y = torch.empty(M, N2 // 2, device=cuda, dtype=torch.bfloat16)
    assert lib.cgs_gemm_bf16_v7ws(a.data_ptr(), wi.data_ptr(), y.data_ptr(), bi.data_ptr(), None, M, N2, K, K, K,
                                  N2 // 2, 0, 1 | core.EPI_GEGLU, 1.0, ws.data_ptr(), ws_bytes, core._stream()) == 0
    h = a.float() @ w.float().t() + b.float()
    x1, g = h.chunk(2, dim=-1)
    assert _rel(y, x1 * F.gelu(g)) < 1e-2


@pytest.mark.parametrize("N,C1,C2,H,W,Cout,k,res", [(4, 1280, 0, 32, 32, 1280, 3, True), (4, 1280, 1280, 32, 32, 1280, 3, False),
                                                    (2, 640, 0, 64, 48, 640, 3, True), (4, 2560, 2560, 32, 32, 1280, 1, False)])
def test_conv_v7_split_tail(cuda, N, C1, C2, H, W, Cout, k, res):
    """v7 conv with the buffer-load gather (ConvGatherKB) and the split-K tail, dual source included."""
    lib = _native.load_kernels()
    Cin = C1 + C2
    ws_bytes = lib.cgs_v7_ws_bytes(N * H * W, Cout, k * k * Cin)
    assert ws_bytes > 0
    torch.manual_seed(0)
    a = torch.randn(N, C1, H, W, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x2 = (torch.randn(N, C2, H, W, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
          if C2 else None)
    w = (torch.randn(Cout, Cin, k, k, device=cuda) / math.sqrt(Cin * k * k)).to(torch.bfloat16)
    bias = torch.randn(Cout, device=cuda).to(torch.bfloat16)
    full = a if x2 is None else torch.cat([a, x2], 1)
    ref = F.conv2d(full.float(), w.float(), bias.float(), 1, k // 2)
    r = None
    if res:
        r = torch.randn_like(ref).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        ref = ref + r.float()
    wn = w.permute(0, 2, 3, 1).contiguous()
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=cuda)
    y = torch.empty(N, Cout, H, W, device=cuda, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    assert lib.cgs_conv2d_nhwc_v7ws(a.data_ptr(), None if x2 is None else x2.data_ptr(), C1, wn.data_ptr(),
                                    bias.data_ptr(), None if r is None else r.data_ptr(), y.data_ptr(), N, H, W, Cin,
                                    Cout, k, k, 1, k // 2, H, W, 0, ws.data_ptr(), ws_bytes, core._stream()) == 0
    assert _rel(y, ref) < 1e-2


@pytest.mark.parametrize("M,C,N,geglu", [(4096, 640, 1920, False), (1000, 1280, 3840, False), (2048, 640, 5120, True),
                                         (16384, 1280, 10240, True), (4096, 640, 640, False), (2000, 1280, 1280, False)])
def test_layernorm_folded_gemm(cuda, M, C, N, geglu):
    """K07 folded: LN(x) @ W^T + b from the raw rows + (mean, rstd) -- fp32 reference of LN then GEMM."""
    torch.manual_seed(0)
    x = (torch.randn(M, C, device=cuda) * 3 + 1.5).to(torch.bfloat16)
    gamma = (torch.rand(C, device=cuda) + 0.5).to(torch.bfloat16)
    beta = (torch.randn(C, device=cuda) * 0.2).to(torch.bfloat16)
    w = (torch.randn(N, C, device=cuda) / math.sqrt(C)).to(torch.bfloat16)
    b = torch.randn(N, device=cuda).to(torch.bfloat16) if geglu else None
    rs = ops.layernorm_stats(x, 1e-5)
    ref_ln = F.layer_norm(x.float(), (C,), gamma.float(), beta.float(), 1e-5)
    assert torch.allclose(rs[:, 0], x.float().mean(1), atol=1e-3)
    h = ref_ln @ w.float().t() + (b.float() if b is not None else 0)
    if geglu:
        wi, bi = core.geglu_interleave(w), core.geglu_interleave(b)
        w2, cs, b2 = ops.lnfold_weights(wi, bi, gamma, beta)
        y = ops.linear_lnfold(x, rs, w2, cs, b2, geglu=True)
        a, g = h.chunk(2, dim=-1)
        ref = a * F.gelu(g)
    else:
        w2, cs, b2 = ops.lnfold_weights(w, None, gamma, beta)
        y = ops.linear_lnfold(x, rs, w2, cs, b2)
        ref = h
    assert _rel(y, ref) < 1.5e-2


@pytest.mark.parametrize("M,C,N,geglu", [(2048, 1280, 3840, False), (2048, 1280, 10240, True), (8192, 640, 1920, False),
                                         (300, 640, 1280, False), (1152, 2048, 4096, True)])
@pytest.mark.parametrize("variant", [8, 10, 11, 12, 13, 14])
def test_layernorm_folded_gemm_small_tiles(cuda, M, C, N, geglu, variant):
    """The LayerNorm fold on the small-tile kernels (128x128 / 64x128 / 128x64) the batch-1 UNet's
    under-filled grids autotune to: same fp32 reference as test_layernorm_folded_gemm."""
    torch.manual_seed(1)
    x = (torch.randn(M, C, device=cuda) * 3 + 1.5).to(torch.bfloat16)
    gamma = (torch.rand(C, device=cuda) + 0.5).to(torch.bfloat16)
    beta = (torch.randn(C, device=cuda) * 0.2).to(torch.bfloat16)
    w = (torch.randn(N, C, device=cuda) / math.sqrt(C)).to(torch.bfloat16)
    b = torch.randn(N, device=cuda).to(torch.bfloat16)
    rs = ops.layernorm_stats(x, 1e-5)
    h = F.layer_norm(x.float(), (C,), gamma.float(), beta.float(), 1e-5) @ w.float().t() + b.float()
    if geglu:
        w2, cs, b2 = ops.lnfold_weights(core.geglu_interleave(w), core.geglu_interleave(b), gamma, beta)
        a, g = h.chunk(2, dim=-1)
        ref = a * F.gelu(g)
    else:
        w2, cs, b2 = ops.lnfold_weights(w, b, gamma, beta)
        ref = h
    nout = N // 2 if geglu else N
    y = torch.empty(M, nout, device=cuda, dtype=torch.bfloat16)
    lib = _native.load_kernels()
    assert lib.cgs_gemm_bf16_lnfold_v(x.data_ptr(), w2.data_ptr(), y.data_ptr(), b2.data_ptr(), rs.data_ptr(),
                                      cs.data_ptr(), M, N, C, C, C, nout,
                                      core.EPI_BIAS | (core.EPI_GEGLU if geglu else 0), None, 0, variant,
                                      core._stream()) == 0
    assert _rel(y, ref) < 1.5e-2


def test_transformer_block_lnfold_matches_unfolded(cuda, monkeypatch):
    from comfy_gen_server_amd.models.attention import BasicTransformerBlock
    from comfy_gen_server_amd.models.layers import init_random_fast_
    torch.manual_seed(0)
    with torch.inference_mode():
        blk = BasicTransformerBlock(640, 10, 64, context_dim=2048, dtype=torch.bfloat16, device=cuda)
        init_random_fast_(blk, seed=2)
        x = torch.randn(2, 1024, 640, device=cuda).to(torch.bfloat16)
        ctx = torch.randn(2, 77, 2048, device=cuda).to(torch.bfloat16)
        ops.reset_stats()
        y_fold = blk(x, context=ctx, transformer_options={})
        assert blk._lnfold_ok(x)
        monkeypatch.setattr(core, "_LNFOLD", False)
        y_ref = blk(x, context=ctx, transformer_options={})
    assert _rel(y_fold, y_ref) < 2e-2


@pytest.mark.parametrize("M,N,K", [(77, 3840, 1280), (16, 1280, 1280), (1, 320, 1280), (77, 768, 3072), (128, 200, 96),
                                   (100, 5120, 1280), (33, 8, 64), (77, 1280, 5120), (77, 1280, 1280)])
@pytest.mark.parametrize("epi", ["none", "bias", "bias_res", "bias_gelu"])
def test_gemm_skinny(cuda, M, N, K, epi):
    """Skinny-M GEMM (one prompt through CLIP, time-embedding projections): one workgroup per 16
    columns, K split over the 8 waves -- and, where N / 16 workgroups underfill the chip, over S K-slices
    (fp32 partials + a reduce/epilogue kernel: cgs_gemm_skinny_ws) -- vs fp32 torch."""
    torch.manual_seed(2)
    a = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    w = (torch.randn(N, K, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    b = torch.randn(N, device=cuda).to(torch.bfloat16) if epi != "none" else None
    r = torch.randn(M, N, device=cuda).to(torch.bfloat16) if epi == "bias_res" else None
    gelu = epi == "bias_gelu"
    y = ops.linear(a, w, b, residual=r, act="gelu" if gelu else None)
    ref = a.float() @ w.float().t()
    if b is not None:
        ref = ref + b.float()
    if gelu:
        ref = torch.nn.functional.gelu(ref)
    if r is not None:
        ref = ref + r.float()
    assert ops.stats().get(("gemm", "hip"), 0) == 1
    assert _rel(y, ref) < 1e-2
    if (M, N, K) == (77, 1280, 5120):
        assert core._SKWS.get((M, N, K), 0) > 0     # takes the split-K form


def test_attention_underfilled_grid_autotuned(cuda, monkeypatch):
    """Batch-2 level-2 SDXL self-attention (2 x 20 heads x 1024 tokens: 160 workgroups of the D=64
    kernel) goes through the per-call d64 / generic choice; both candidates match fp32."""
    monkeypatch.setenv("CGS_AUTOTUNE", "1")
    torch.manual_seed(8)
    B, H, S, D = 2, 20, 1024, 64
    q = torch.randn(B, S, H * D, device=cuda).to(torch.bfloat16)
    ref = core.attention_reference(q.float(), q.float(), q.float(), H)
    o = ops.attention(q, q, q, H)
    assert ops.stats().get(("attention", "hip"), 0) == 1
    assert _rel(o, ref) < 2e-2
    lib = core._lib()
    for var in (0, 1):
        ov = torch.empty_like(q)
        assert lib.cgs_flash_attn_fwd_v(q.data_ptr(), q.data_ptr(), q.data_ptr(), ov.data_ptr(), B, H, S, S, D,
                                        q.stride(0), q.stride(1), D, q.stride(0), q.stride(1), D, q.stride(0),
                                        q.stride(1), D, ov.stride(0), ov.stride(1), D, D ** -0.5, var,
                                        core._stream()) == 0
        assert _rel(ov, ref) < 2e-2


# Narrow-output convs (Cout <= 16: UNet conv_out 320 -> 4, VAE conv_out 128 -> 3): the dedicated
# kernel (conv_nhwc_smalln_kernel) for every variant but an explicit v2; includes Cin % 64 != 0,
# stride 2, the fused 2x upsample, a residual and the dual-source (skip-concat) input.
@pytest.mark.parametrize("N,Cin,H,W,Cout,k,s,up,res", [(2, 320, 128, 128, 4, 3, 1, False, False),
                                                       (1, 128, 1024, 1024, 3, 3, 1, False, False),
                                                       (3, 96, 13, 11, 3, 3, 1, False, True),
                                                       (2, 32, 9, 17, 16, 3, 2, False, False),
                                                       (1, 64, 10, 6, 8, 1, 1, False, True),
                                                       (2, 160, 7, 9, 5, 3, 1, True, False)])
def test_conv2d_narrow_output(cuda, N, Cin, H, W, Cout, k, s, up, res):
    torch.manual_seed(3)
    p = k // 2
    x = torch.randn(N, Cin, H, W, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Cout, Cin, k, k, device=cuda) / math.sqrt(Cin * k * k)).to(torch.bfloat16)
    b = torch.randn(Cout, device=cuda).to(torch.bfloat16)
    xr = F.interpolate(x.float(), scale_factor=2.0, mode="nearest") if up else x.float()
    ref = F.conv2d(xr, w.float(), b.float(), s, p)
    r = None
    if res:
        r = torch.randn_like(ref).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        ref = ref + r.float()
    wn = w.permute(0, 2, 3, 1).contiguous()
    y = ops.conv2d(x, w, b, s, p, residual=r, weight_nhwc=wn, upsample2x=up)
    assert ops.stats().get(("conv", "hip"), 0) == 1 and ops.stats().get(("conv", "lib"), 0) == 0
    assert y.shape == ref.shape
    assert _rel(y, ref) < 1e-2
    if H >= 128 and Cin % 64 == 0:      # production shape: time it against the 256-row v2 tile
        lib = _native.load_kernels()

        def t(variant):
            lib.cgs_conv_set_variant(variant)
            try:
                for _ in range(2):
                    ops.conv2d(x, w, b, s, p, weight_nhwc=wn)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    ops.conv2d(x, w, b, s, p, weight_nhwc=wn)
                e1.record()
                torch.cuda.synchronize()
                return e0.elapsed_time(e1) / 5
            finally:
                lib.cgs_conv_set_variant(-1)
        t_new, t_v2 = t(-1), t(2)
        print(f"narrow conv N={N} Cin={Cin} {H}x{W} Cout={Cout}: smalln {t_new * 1e3:.1f} us, v2 {t_v2 * 1e3:.1f} us")
        assert t_new < t_v2


def test_conv2d_narrow_output_dual_source(cuda):
    torch.manual_seed(4)
    a = torch.randn(2, 128, 12, 10, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    b2 = torch.randn(2, 64, 12, 10, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(16, 192, 3, 3, device=cuda) / math.sqrt(192 * 9)).to(torch.bfloat16)
    bias = torch.randn(16, device=cuda).to(torch.bfloat16)
    ref = F.conv2d(torch.cat([a, b2], 1).float(), w.float(), bias.float(), 1, 1)
    y = ops.conv2d(a, w, bias, 1, 1, weight_nhwc=w.permute(0, 2, 3, 1).contiguous(), x2=b2)
    assert ops.stats().get(("conv", "hip"), 0) == 1
    assert _rel(y, ref) < 1e-2


# ConvTranspose2d(4, 2, 1) (Stable Cascade Stage A decoder upsampler) as four sub-pixel phase convs on
# the HIP conv kernel; includes the production shape (384 -> 192 at 256^2, batch 1).
@pytest.mark.parametrize("N,Cin,H,W,Cout", [(1, 384, 256, 256, 192), (2, 64, 7, 9, 32), (1, 96, 12, 10, 8)])
def test_conv_transpose2d_phases(cuda, N, Cin, H, W, Cout):
    torch.manual_seed(5)
    x = torch.randn(N, Cin, H, W, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Cin, Cout, 4, 4, device=cuda) / math.sqrt(Cin * 4)).to(torch.bfloat16)
    b = torch.randn(Cout, device=cuda).to(torch.bfloat16)
    ref = F.conv_transpose2d(x.float(), w.float(), b.float(), 2, 1)
    y = ops.conv_transpose2d(x, w, b, 2, 1)
    assert ops.stats().get(("conv", "hip"), 0) == 4 and ops.stats().get(("conv", "lib"), 0) == 0
    assert y.shape == ref.shape
    assert _rel(y, ref) < 1e-2


def test_cascade_stage_a_decode_on_hip(cuda):
    """Stage A decode (ResBlockA stack + 4x4/s2 transposed conv + pixel shuffle) runs without any
    library conv and matches the same module in fp32 on the CPU."""
    from comfy_gen_server_amd.models.cascade import StageA
    from comfy_gen_server_amd.models.layers import init_random_fast_
    torch.manual_seed(6)
    m = StageA(bottleneck_blocks=2, dtype=torch.float32)
    init_random_fast_(m, seed=3)
    z = torch.randn(1, 4, 32, 32)
    with torch.inference_mode():
        ref = m.decode(z)
        md = m.to(device=cuda, dtype=torch.bfloat16)
        ops.reset_stats()
        y = md.decode(z.to(cuda))
    st = ops.stats()
    assert st.get(("conv", "lib"), 0) == 0 and st.get(("conv", "hip"), 0) >= 4 and st.get(("gemm", "lib"), 0) == 0, st
    assert y.shape == ref.shape
    assert _rel(y.float().cpu(), ref) < 3e-2


@pytest.mark.parametrize("N,H,W,C", [(2, 24, 24, 2048), (1, 16, 16, 1280), (4, 7, 9, 64)])
def test_channel_affine_nhwc(cuda, N, H, W, C):
    """Cascade TimestepBlock: x * (1 + a) + b with a, b the halves of one [N, 2C] mapper output."""
    torch.manual_seed(2)
    x = torch.randn(N, H, W, C, device=cuda).to(torch.bfloat16)
    ab = torch.randn(N, 2 * C, device=cuda).to(torch.bfloat16)
    a, b = ab.chunk(2, dim=-1)
    ops.reset_stats()
    y = ops.channel_affine_nhwc(x, a, b, add=1.0)
    assert ops.stats().get(("channel_affine", "hip"), 0) == 1
    ref = x.float() * (1 + a.float()[:, None, None, :]) + b.float()[:, None, None, :]
    assert _rel(y, ref) < 1e-2


@pytest.mark.parametrize("N,H,W,Cin,Cout,pre", [(2, 32, 32, 320, 320, True), (1, 16, 16, 640, 640, False),
                                                 (2, 16, 32, 128, 160, True)])
def test_conv_gn_stats_epilogue(cuda, N, H, W, Cin, Cout, pre):
    """K06 second half (wired for the UNet ResBlock since r04: profiles/r04/gn_convstats_ab_r04ax.log): the v6 conv's
    epilogue writes the GroupNorm partials of its bf16 output; finalize + apply from them == the GroupNorm
    of the stored conv output (pre-add shift included)."""
    torch.manual_seed(3)
    lib = _native.load_kernels()
    x = (torch.rand(N, H, W, Cin, device=cuda) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(Cout, 3, 3, Cin, device=cuda) * 2 - 1) / math.sqrt(Cin * 9)).to(torch.bfloat16)
    b = (torch.randn(Cout, device=cuda) + 2).to(torch.bfloat16)
    g = torch.randn(Cout, device=cuda).to(torch.bfloat16)
    be = torch.randn(Cout, device=cuda).to(torch.bfloat16)
    p = torch.randn(N, Cout, device=cuda).to(torch.bfloat16) if pre else None
    out = torch.empty(N, H, W, Cout, device=cuda, dtype=torch.bfloat16)
    HW = H * W
    gnp = torch.full((N * (HW // 64) * Cout * 2,), float("nan"), device=cuda)
    ab = torch.empty(N * Cout * 2, device=cuda)
    y = torch.empty_like(out)
    st = core._stream()
    assert lib.cgs_conv2d_nhwc_gns(x.data_ptr(), None, Cin, w.data_ptr(), b.data_ptr(), None, out.data_ptr(), N, H, W,
                                   Cin, Cout, 3, 3, 1, 1, H, W, 0, gnp.data_ptr(), st) == 0
    assert lib.cgs_groupnorm_nhwc_part(out.data_ptr(), y.data_ptr(), g.data_ptr(), be.data_ptr(),
                                       None if p is None else p.data_ptr(), gnp.data_ptr(), ab.data_ptr(), N, HW, Cout,
                                       32, 64, 1e-5, 1, 1, st) == 0
    torch.cuda.synchronize()
    assert torch.isfinite(gnp).all()
    conv_ref = F.conv2d(x.permute(0, 3, 1, 2).float(), w.permute(0, 3, 1, 2).float(), b.float(), 1, 1)
    assert _rel(out.permute(0, 3, 1, 2), conv_ref) < 1e-2
    xf = out.permute(0, 3, 1, 2).float() + (p.float()[:, :, None, None] if pre else 0.0)
    ref = F.silu(F.group_norm(xf, 32, g.float(), be.float(), 1e-5))
    assert _rel(y.permute(0, 3, 1, 2), ref) < 1e-2


def test_conv_gn_stats_wired(cuda, monkeypatch):
    """ops.conv2d(gn_stats=True) -> ops.group_norm (the UNet ResBlock's in_layers conv -> out_layers GroupNorm,
    models/unet.py): the statistics come from the conv epilogue and the result equals the two-pass GroupNorm.
    The shape is a packaged-table key whose tuned kernel is v6 (the only one with the statistics epilogue)."""
    monkeypatch.setenv("CGS_AUTOTUNE", "1")
    torch.manual_seed(5)
    N, H, W, Cin, Cout = 2, 128, 128, 320, 320
    x = torch.randn(N, Cin, H, W, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Cout, Cin, 3, 3, device=cuda) / math.sqrt(Cin * 9)).to(torch.bfloat16)
    b = torch.randn(Cout, device=cuda).to(torch.bfloat16)
    wn = w.permute(0, 2, 3, 1).contiguous()
    g = (1 + 0.1 * torch.randn(Cout, device=cuda)).to(torch.bfloat16)
    be = (0.1 * torch.randn(Cout, device=cuda)).to(torch.bfloat16)
    pre = torch.randn(N, Cout, device=cuda).to(torch.bfloat16)
    h = ops.conv2d(x, w, b, 1, 1, weight_nhwc=wn, gn_stats=True)
    assert getattr(h, "_cgs_gnpart", None) is not None, "tuned v6 conv did not take the statistics epilogue"
    y = ops.group_norm(h, 32, g, be, 1e-5, silu=True, pre_add=pre)
    h_plain = ops.conv2d(x, w, b, 1, 1, weight_nhwc=wn)
    assert getattr(h_plain, "_cgs_gnpart", None) is None
    y_ref = ops.group_norm(h_plain, 32, g, be, 1e-5, silu=True, pre_add=pre)
    torch.cuda.synchronize()
    assert torch.equal(h, h_plain)
    assert (y.float() - y_ref.float()).abs().max().item() < 0.05
    ref = F.silu(F.group_norm(h.float() + pre.float()[:, :, None, None], 32, g.float(), be.float(), 1e-5))
    assert _rel(y, ref) < 1e-2


@pytest.mark.parametrize("B,H,Sq,S2", [(2, 32, 576, 85), (1, 8, 300, 77), (2, 4, 1024, 8)])
def test_attention_two_kv_sources(cuda, B, H, Sq, S2):
    """Stable Cascade self-attention over cat([x, kv]) with the keys read from two (strided) sources:
    == attention over the materialised concat; the HIP two-source kernel runs."""
    torch.manual_seed(5)
    C = H * 64
    qkv = torch.randn(B, Sq, 3 * C, device=cuda).to(torch.bfloat16)
    kv2 = torch.randn(B, S2, 2 * C, device=cuda).to(torch.bfloat16)
    q, k1, v1 = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
    k2, v2 = kv2[..., :C], kv2[..., C:]
    o = ops.attention_kv2(q, k1, v1, k2, v2, H)
    assert ops.stats().get(("attention", "hip"), 0) == 1
    ref = core.attention_reference(q.float(), torch.cat([k1, k2], 1).float(), torch.cat([v1, v2], 1).float(), H)
    assert _rel(o, ref) < 1e-2


def test_cascade_self_attention_two_source_path(cuda, monkeypatch):
    """Stable Cascade Stage C (head dim 64) on the device: self-attention through the fused QKV / KV
    projections and the two-source kernel == the concat path (cat([x, kv]) -> to_q / to_k / to_v)."""
    from comfy_gen_server_amd.models import cascade as SC
    from comfy_gen_server_amd.models.layers import init_random_
    cfg = dict(c_in=16, c_out=16, c_r=64, c_cond=128, c_hidden=[128, 128], nhead=[2, 2], blocks=[[1, 1], [1, 1]],
               block_repeat=[[1, 1], [1, 1]], level_config=["CTA", "CTA"], c_clip_text=64, c_clip_text_pooled=64,
               c_clip_img=768, c_clip_seq=2, switch_level=[False])
    m = SC.StageC(**cfg)
    init_random_(m, seed=11)
    m = m.to(device=cuda, dtype=torch.bfloat16)
    g = torch.Generator().manual_seed(1)
    args = (torch.randn(2, 16, 12, 12, generator=g), torch.tensor([0.3, 0.7]), torch.randn(2, 7, 64, generator=g),
            torch.randn(2, 1, 64, generator=g), torch.randn(2, 1, 768, generator=g))
    args = tuple(a.to(cuda, torch.bfloat16 if a.dim() > 1 else torch.float32) for a in args)
    with torch.inference_mode():
        ops.reset_stats()
        fast = m(*args).float()
        n_fast = ops.stats().get(("attention", "hip"), 0)
        monkeypatch.setattr(SC.OptimizedAttention, "forward_self",
                            lambda self, xs, kv, residual=None, kvp=None: self.forward(
                                xs, torch.cat([xs, kv.to(xs.dtype)], 1), torch.cat([xs, kv.to(xs.dtype)], 1),
                                residual=residual))
        slow = m(*args).float()
    assert n_fast > 0
    assert _rel(fast, slow) < 2e-2


@pytest.mark.parametrize("M,N2,K,ln", [(2048, 10240, 1280, False), (600, 5120, 640, False), (333, 2560, 320, False),
                                       (2048, 10240, 1280, True), (1000, 5120, 640, True)])
def test_gemm_geglu_v6(cuda, M, N2, K, ln):
    """GEGLU on the 256x160 kernel (pq::run GG: 16-row-interleaved weights staged so that one
    v_permlane32_swap pairs a / g), plain and with the LayerNorm fold, vs the fp32 reference."""
    torch.manual_seed(2)
    lib = _native.load_kernels()
    a = (torch.randn(M, K, device=cuda) * (3 if ln else 1) + (1.5 if ln else 0)).to(torch.bfloat16)
    w = (torch.randn(N2, K, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    b = torch.randn(N2, device=cuda).to(torch.bfloat16)
    if ln:
        gamma = (torch.rand(K, device=cuda) + 0.5).to(torch.bfloat16)
        beta = (torch.randn(K, device=cuda) * 0.2).to(torch.bfloat16)
        rs = ops.layernorm_stats(a, 1e-5)
        w2, cs, b2 = ops.lnfold_weights(core.geglu_interleave(w), core.geglu_interleave(b), gamma, beta)
        y = torch.empty(M, N2 // 2, device=cuda, dtype=torch.bfloat16)
        assert lib.cgs_gemm_bf16_lnfold_v(a.data_ptr(), w2.data_ptr(), y.data_ptr(), b2.data_ptr(), rs.data_ptr(),
                                          cs.data_ptr(), M, N2, K, K, K, N2 // 2, core.EPI_BIAS | core.EPI_GEGLU,
                                          None, 0, 6, core._stream()) == 0
        h = F.layer_norm(a.float(), (K,), gamma.float(), beta.float(), 1e-5) @ w.float().t() + b.float()
    else:
        lib.cgs_gemm_set_variant(6)
        try:
            y = ops.linear_geglu(a, core.geglu_interleave(w), core.geglu_interleave(b))
        finally:
            lib.cgs_gemm_set_variant(-1)
        h = a.float() @ w.float().t() + b.float()
    x1, g = h.chunk(2, dim=-1)
    ref = x1 * F.gelu(g)
    assert _rel(y, ref) < 1.5e-2


@pytest.mark.parametrize("M,N,K,variant", [(1000, 320, 128, 6), (4096, 1280, 320, 6), (1152, 8192, 256, 8),
                                           (300, 640, 96, 10), (64, 512, 256, -1), (2048, 256, 512, 4),
                                           (577, 264, 64, 14)])
@pytest.mark.parametrize("res", [False, True])
def test_gemm_gelu_epilogue(cuda, M, N, K, variant, res):
    """EPI_GELU: out = gelu(A W^T + b) (+ R) in the v6 ACT kernel, the mc::tile family and skinny."""
    torch.manual_seed(5)
    a = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    w = (torch.randn(N, K, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    b = torch.randn(N, device=cuda).to(torch.bfloat16)
    r = torch.randn(M, N, device=cuda).to(torch.bfloat16) if res else None
    out = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    epi = core.EPI_BIAS | core.EPI_GELU | (core.EPI_RESIDUAL if res else 0)
    rc = _native.load_kernels().cgs_gemm_bf16_v(a.data_ptr(), w.data_ptr(), out.data_ptr(), b.data_ptr(),
                                                 None if r is None else r.data_ptr(), M, N, K, K, K, N,
                                                 N if res else 0, epi, 1.0, variant, core._stream())
    assert rc == 0
    ref = F.gelu(a.float() @ w.float().t() + b.float()) + (r.float() if res else 0.0)
    assert _rel(out, ref) < 1e-2
    # the op-level entry point (autotuned kernel choice) agrees
    y = ops.linear(a, w, b, residual=r, act="gelu")
    assert _rel(y, ref) < 1e-2


@pytest.mark.parametrize("N,H,W,c", [(2, 16, 16, 64), (2, 6, 6, 64), (1, 32, 24, 128)])
def test_cascade_channel_mlp_grn_fold(cuda, N, H, W, c, monkeypatch):
    """Cascade ChannelMLP on the device -- GELU epilogue, then the GRN either as a pass over h (H W <= c)
    or folded into per-image second-GEMM weights (H W > c) -- vs the fp32 NCHW reference math."""
    from comfy_gen_server_amd.models import cascade as SC
    from comfy_gen_server_amd.models.layers import init_random_
    for k in ("GELU_EPI", "GRNFOLD"):
        monkeypatch.setenv(f"CGS_CASCADE_{k}", "1")
    torch.manual_seed(6)
    m = SC._ChannelMLP(c, 4 * c, c)
    init_random_(m, seed=3)
    with torch.no_grad():
        m[2].gamma.normal_(0, 0.5)
        m[2].beta.normal_(0, 0.5)
    x = torch.randn(N, H, W, c)
    res = torch.randn(N, H, W, c)
    h = F.gelu(F.linear(x, m[0].weight, m[0].bias))
    gx = torch.norm(h, p=2, dim=(1, 2), keepdim=True)
    nx = gx / (gx.mean(dim=-1, keepdim=True) + 1e-6)
    h = m[2].gamma * (h * nx) + m[2].beta + h
    ref = F.linear(h, m[4].weight, m[4].bias) + res
    g = m.to(device=cuda, dtype=torch.bfloat16)
    with torch.no_grad():
        y = g(x.to(cuda, torch.bfloat16), residual=res.to(cuda, torch.bfloat16))
    assert ops.stats().get(("grn", "hip"), 0) == 1 and ops.stats().get(("gemm", "hip"), 0) >= 2
    assert _rel(y.cpu(), ref) < 2e-2


@pytest.mark.parametrize("N,H,W,C", [(2, 24, 24, 2048), (3, 5, 7, 64), (1, 8, 8, 1280), (2, 4, 4, 4096)])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_channel_affine_layernorm(cuda, N, H, W, C, dt):
    """One-pass x * (1 + a[n]) + b[n] and LayerNorm of it (Cascade TimestepBlock -> AttnBlock): xa bit-equal
    to channel_affine_nhwc, LN(xa) vs the fp32 LayerNorm of xa."""
    torch.manual_seed(1)
    x = (torch.randn(N, H, W, C, device=cuda) * 2 + 0.5).to(dt)
    ab = (torch.randn(N, 2 * C, device=cuda) * 0.5).to(dt)
    a, b = ab.chunk(2, dim=-1)
    ops.reset_stats()
    xa, y = ops.channel_affine_layernorm_nhwc(x, a, b, add=1.0, eps=1e-6)
    assert ops.stats().get(("channel_affine", "hip"), 0) == 1
    assert torch.equal(xa, ops.channel_affine_nhwc(x, a, b, add=1.0))
    ref = F.layer_norm(xa.float(), (C,), eps=1e-6)
    assert _rel(y, ref) < 1e-2


@pytest.mark.parametrize("batched", ["1", "0"])
def test_cascade_timestep_mappers_one_gemm(cuda, batched, monkeypatch):
    """Stage C with every TimestepBlock's mapper pair from one GEMM per call (TSBATCH) == the per-block
    mapper GEMMs, vs the fp32 CPU model."""
    from comfy_gen_server_amd.models import cascade as SC
    from comfy_gen_server_amd.models.layers import init_random_
    monkeypatch.setenv("CGS_CASCADE_TSBATCH", batched)
    cfg = dict(c_in=16, c_out=16, c_r=64, c_cond=128, c_hidden=[128, 256], nhead=[2, 4], blocks=[[1, 2], [2, 1]],
               block_repeat=[[1, 1], [1, 1]], level_config=["CT", "CTA"], c_clip_text=64, c_clip_text_pooled=64,
               c_clip_img=768, c_clip_seq=2, switch_level=[False])
    m = SC.StageC(**cfg)
    init_random_(m, seed=12)
    g = torch.Generator().manual_seed(2)
    args = (torch.randn(2, 16, 8, 8, generator=g), torch.tensor([0.2, 0.9]), torch.randn(2, 7, 64, generator=g),
            torch.randn(2, 1, 64, generator=g), torch.randn(2, 1, 768, generator=g))
    with torch.inference_mode():
        ref = m(*args).float()
        m = m.to(device=cuda, dtype=torch.bfloat16)
        out = m(*tuple(a.to(cuda, torch.bfloat16 if a.dim() > 1 else torch.float32) for a in args)).float().cpu()
    assert ("_ts_fused" in m.__dict__) == (batched == "1")
    assert _rel(out, ref) < 3e-2


@pytest.mark.parametrize("fused", ["1", "0"])
def test_cascade_stage_affine_layernorm_path(cuda, fused, monkeypatch):
    """Stage C (C-T-A blocks) with the TimestepBlock writing the next AttnBlock's LayerNorm (AFFLN) == the
    separate affine + LayerNorm passes."""
    from comfy_gen_server_amd.models import cascade as SC
    from comfy_gen_server_amd.models.layers import init_random_
    monkeypatch.setenv("CGS_CASCADE_AFFLN", fused)
    calls = []
    real = ops.channel_affine_layernorm_nhwc
    monkeypatch.setattr(ops, "channel_affine_layernorm_nhwc", lambda *a, **k: calls.append(1) or real(*a, **k))
    cfg = dict(c_in=16, c_out=16, c_r=64, c_cond=128, c_hidden=[128, 128], nhead=[2, 2], blocks=[[1, 1], [1, 1]],
               block_repeat=[[1, 1], [1, 1]], level_config=["CTA", "CTA"], c_clip_text=64, c_clip_text_pooled=64,
               c_clip_img=768, c_clip_seq=2, switch_level=[False])
    m = SC.StageC(**cfg)
    init_random_(m, seed=11)
    g = torch.Generator().manual_seed(1)
    args = (torch.randn(2, 16, 12, 12, generator=g), torch.tensor([0.3, 0.7]), torch.randn(2, 7, 64, generator=g),
            torch.randn(2, 1, 64, generator=g), torch.randn(2, 1, 768, generator=g))
    with torch.inference_mode():
        ref = m(*args).float()
        m = m.to(device=cuda, dtype=torch.bfloat16)
        out = m(*tuple(a.to(cuda, torch.bfloat16 if a.dim() > 1 else torch.float32) for a in args)).float().cpu()
    assert (len(calls) > 0) == (fused == "1")
    assert _rel(out, ref) < 3e-2


@pytest.mark.parametrize("fold", ["1", "0"])
@pytest.mark.parametrize("N,H,W,c", [(2, 6, 6, 128), (1, 16, 8, 256)])
def test_cascade_attnblock_lnfold(cuda, N, H, W, c, fold, monkeypatch):
    """Cascade AttnBlock on the device with its LayerNorm folded into the fused QKV GEMM (ATTNLN=1:
    statistics pass + ops.linear_lnfold) or materialised (0), plain and with the static conditioning K/V
    of a captured step, vs the fp32 CPU block."""
    from comfy_gen_server_amd.models import cascade as SC
    from comfy_gen_server_amd.models.layers import init_random_
    monkeypatch.setenv("CGS_CASCADE_ATTNLN", fold)
    calls = []
    real = ops.linear_lnfold
    monkeypatch.setattr(ops, "linear_lnfold", lambda *a, **k: calls.append(1) or real(*a, **k))
    torch.manual_seed(3)
    blk = SC.AttnBlock(c, 64, c // 64, self_attn=True)
    init_random_(blk, seed=5)
    x = torch.randn(N, H, W, c)
    kv = torch.randn(N, 5, 64)
    with torch.no_grad():
        ref = blk(x, kv)
        g = blk.to(device=cuda, dtype=torch.bfloat16)
        xg, kvg = x.to(cuda, torch.bfloat16), kv.to(cuda, torch.bfloat16)
        y = g(xg, kvg).float().cpu()
        y2 = g(xg, {id(g): g.static_kv(kvg)}).float().cpu()
    assert len(calls) == (2 if fold == "1" else 0)
    assert _rel(y, ref) < 2e-2 and _rel(y2, ref) < 2e-2


@pytest.mark.parametrize("N,H,W,c", [(2, 16, 16, 128), (2, 6, 6, 128), (1, 8, 8, 256)])
def test_cascade_resblock_lnfold(cuda, N, H, W, c, monkeypatch):
    """Cascade ResBlock / FeedForwardBlock on the device: LayerNorm folded into the first GEMM together with
    the GELU epilogue (ops.linear_lnfold act="gelu"), GRN pass or GRN weight fold, vs the fp32 CPU blocks."""
    from comfy_gen_server_amd.models import cascade as SC
    from comfy_gen_server_amd.models.layers import init_random_
    for k in ("GELU_EPI", "LNFOLD", "GRNFOLD", "DWLN"):
        monkeypatch.setenv(f"CGS_CASCADE_{k}", "1")
    torch.manual_seed(7)
    for blk in (SC.ResBlock(c), SC.FeedForwardBlock(c)):
        init_random_(blk, seed=4)
        grn = blk.channelwise[2]
        with torch.no_grad():
            grn.gamma.normal_(0, 0.5)
            grn.beta.normal_(0, 0.5)
        x = torch.randn(N, H, W, c)
        with torch.no_grad():
            ref = blk(x)
            g = blk.to(device=cuda, dtype=torch.bfloat16)
            ops.reset_stats()
            y = g(x.to(cuda, torch.bfloat16)).float().cpu()
        # ResBlock: the statistics come out of the depthwise kernel; FeedForwardBlock: one statistics pass
        assert ops.stats().get(("layernorm", "hip"), 0) == (0 if isinstance(blk, SC.ResBlock) else 1)
        assert _rel(y, ref) < 2e-2


@pytest.mark.parametrize("N,H,W,c", [(2, 8, 8, 320), (2, 24, 24, 320), (3, 16, 8, 640)])
def test_cascade_grn_stats_from_gemm_epilogue(cuda, N, H, W, c, monkeypatch):
    """The GELU GEMM's epilogue writes per-(image, 64-row block, column) (mean, M2) partials and the GRN (pass
    over h, or the weight fold) takes sum_HW h^2 from them instead of its statistics pass: same output as
    with the pass (CGS_GRN_GNS off) and as the fp32 CPU block."""
    from comfy_gen_server_amd.models import cascade as SC
    from comfy_gen_server_amd.models.layers import init_random_
    from comfy_gen_server_amd.ops import core as C
    for k in ("GELU_EPI", "LNFOLD", "GRNFOLD", "DWLN"):
        monkeypatch.setenv(f"CGS_CASCADE_{k}", "1")
    used = []
    real = C._grn_part

    def spy(*a):
        r = real(*a)
        used.append(r is not None)
        return r
    monkeypatch.setattr(C, "_grn_part", spy)
    torch.manual_seed(8)
    blk = SC.ResBlock(c)
    init_random_(blk, seed=5)
    with torch.no_grad():
        blk.channelwise[2].gamma.normal_(0, 0.5)
        blk.channelwise[2].beta.normal_(0, 0.5)
    x = torch.randn(N, H, W, c)
    with torch.no_grad():
        ref = blk(x)
        g = blk.to(device=cuda, dtype=torch.bfloat16)
        xd = x.to(cuda, torch.bfloat16)
        y = g(xd).float().cpu()
        assert used and all(used), used
        monkeypatch.setattr(C, "_GRN_GNS", False)
        used.clear()
        y0 = g(xd).float().cpu()
        assert not any(used)
    assert _rel(y, ref) < 2e-2
    assert _rel(y, y0) < 5e-3


@pytest.mark.parametrize("N,H,W,C,k,rep", [(2, 24, 24, 2048, 3, False), (1, 17, 9, 320, 3, False),
                                           (2, 8, 8, 1280, 7, True), (1, 5, 6, 64, 3, False)])
def test_dwconv_ln_stats(cuda, N, H, W, C, k, rep):
    """Depthwise conv with the per-pixel LayerNorm statistics of its (rounded) output in the same pass."""
    torch.manual_seed(8)
    x = (torch.randn(N, H, W, C, device=cuda) + 0.5).to(torch.bfloat16)
    w = (torch.randn(k * k, C, device=cuda) / k).to(torch.bfloat16)
    b = torch.randn(C, device=cuda).to(torch.bfloat16)
    y, rs = ops.depthwise_conv2d_nhwc_lnstats(x, w, b, k, 1e-6, rep)
    xn = x.float().permute(0, 3, 1, 2)
    if rep:
        xn = F.pad(xn, (k // 2,) * 4, mode="replicate")
    ref = F.conv2d(xn, w.float().t().reshape(C, 1, k, k), b.float(), 1, 0 if rep else k // 2, 1, C).permute(0, 2, 3, 1)
    assert ops.stats().get(("dwconv", "hip"), 0) == 1
    assert _rel(y, ref) < 1e-2
    yf = y.float().reshape(-1, C)                   # statistics of the stored bf16 values
    assert torch.allclose(rs[:, 0], yf.mean(1), atol=1e-3, rtol=1e-3)
    assert torch.allclose(rs[:, 1], torch.rsqrt(yf.var(1, unbiased=False) + 1e-6), rtol=2e-3)


@pytest.mark.parametrize("M,N,K,res", [(65536, 640, 640, True), (16384, 1280, 5120, True), (4100, 1280, 1280, False)])
def test_gemm_rowstats_epilogue(cuda, M, N, K, res):
    """v6 GEMM whose epilogue also writes per-row LayerNorm statistics partials (pq::run RSO): the output is
    bitwise the plain v6 output, and the partials (Chan-combined by cgs_ln_rs_from_partials) give the
    (mean, rstd) of the stored rows that the statistics pass computes."""
    torch.manual_seed(5)
    lib = core._lib()
    a = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    w = (torch.randn(N, K, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    b = torch.randn(N, device=cuda).to(torch.bfloat16)
    r = (torch.randn(M, N, device=cuda) * 3 + 2).to(torch.bfloat16) if res else None
    epi = 1 | (2 if res else 0)
    y0 = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    y1 = torch.empty_like(y0)
    part = torch.empty(M, N // 80, 2, device=cuda, dtype=torch.float32)
    s = core._stream()
    assert lib.cgs_gemm_bf16_v(a.data_ptr(), w.data_ptr(), y0.data_ptr(), b.data_ptr(), core._ptr(r), M, N, K, K, K, N,
                               N if res else 0, epi, 1.0, 6, s) == 0
    assert lib.cgs_gemm_bf16_rowstats(a.data_ptr(), w.data_ptr(), y1.data_ptr(), b.data_ptr(), core._ptr(r), M, N, K,
                                      K, K, N, N if res else 0, epi, 1.0, part.data_ptr(), s) == 0
    rs = torch.empty(M, 2, device=cuda, dtype=torch.float32)
    assert lib.cgs_ln_rs_from_partials(part.data_ptr(), rs.data_ptr(), M, N // 80, 1e-5, s) == 0
    torch.cuda.synchronize()
    assert torch.equal(y0, y1)
    yf = y1.float()
    mean = yf.mean(1)
    rstd = torch.rsqrt(yf.var(1, unbiased=False) + 1e-5)
    assert (rs[:, 0] - mean).abs().max().item() < 1e-3 * (mean.abs().max().item() + 1)
    assert ((rs[:, 1] - rstd).abs() / rstd).max().item() < 1e-3


# v6 with 128 x 160 tiles (variant 19, pq::run NI = 2) and its one-wave-group 128 x 80 form (variant 20, NW = 4):
# partial M tiles, every epilogue they carry (bias, residual, LayerNorm fold, row-statistics partials) against fp32.
@pytest.mark.parametrize("M,N,K", [(300, 160, 128), (2048, 1280, 1280), (8200, 640, 640), (129, 320, 2560)])
@pytest.mark.parametrize("epi", ["none", "bias", "bias_res", "ln", "rowstats"])
@pytest.mark.parametrize("variant", [19, 20], ids=["v6m128", "v6w4"])
def test_gemm_v6_m128(cuda, M, N, K, epi, variant):
    torch.manual_seed(11)
    lib = core._lib()
    s = core._stream()
    a = (torch.randn(M, K, device=cuda) * (2 if epi == "ln" else 1) + (1 if epi == "ln" else 0)).to(torch.bfloat16)
    w = (torch.randn(N, K, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    b = torch.randn(N, device=cuda).to(torch.bfloat16) if epi != "none" else None
    r = torch.randn(M, N, device=cuda).to(torch.bfloat16) if epi in ("bias_res", "rowstats") else None
    y = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    if epi == "ln":
        mu = a.float().mean(1)
        rstd = torch.rsqrt(a.float().var(1, unbiased=False) + 1e-5)
        rs = torch.stack([mu, rstd], 1).contiguous()
        cs = w.float().sum(1).contiguous()
        assert lib.cgs_gemm_bf16_lnfold_v(a.data_ptr(), w.data_ptr(), y.data_ptr(), b.data_ptr(), rs.data_ptr(),
                                          cs.data_ptr(), M, N, K, K, K, N, 1, None, 0, variant, s) == 0
        ref = ((a.float() - mu[:, None]) * rstd[:, None]) @ w.float().t() + b.float()
    else:
        e = (1 if b is not None else 0) | (2 if r is not None else 0)
        if epi == "rowstats":
            part = torch.empty(M, N // 80, 2, device=cuda, dtype=torch.float32)
            assert lib.cgs_gemm_bf16_rowstats_v(a.data_ptr(), w.data_ptr(), y.data_ptr(), b.data_ptr(), r.data_ptr(),
                                                M, N, K, K, K, N, N, e, 1.0, part.data_ptr(), variant, s) == 0
            y6 = torch.empty_like(y)
            assert lib.cgs_gemm_bf16_v(a.data_ptr(), w.data_ptr(), y6.data_ptr(), b.data_ptr(), r.data_ptr(), M, N, K,
                                       K, K, N, N, e, 1.0, variant, s) == 0
            rsp = torch.empty(M, 2, device=cuda, dtype=torch.float32)
            assert lib.cgs_ln_rs_from_partials(part.data_ptr(), rsp.data_ptr(), M, N // 80, 1e-5, s) == 0
        else:
            assert lib.cgs_gemm_bf16_v(a.data_ptr(), w.data_ptr(), y.data_ptr(), core._ptr(b), core._ptr(r), M, N, K,
                                       K, K, N, N if r is not None else 0, e, 1.0, variant, s) == 0
        ref = a.float() @ w.float().t() + (b.float() if b is not None else 0) + (r.float() if r is not None else 0)
    torch.cuda.synchronize()
    assert _rel(y, ref) < 1e-2
    if epi == "rowstats":
        assert torch.equal(y, y6)
        yf = y.float()
        assert torch.allclose(rsp[:, 0], yf.mean(1), atol=1e-3, rtol=1e-3)
        assert torch.allclose(rsp[:, 1], torch.rsqrt(yf.var(1, unbiased=False) + 1e-5), rtol=2e-3)


def test_transformer_block_rowstats_matches(cuda, monkeypatch):
    """SDXL transformer block with the LayerNorm statistics taken from the producing GEMMs' epilogues vs the
    statistics pass (CGS_LN_ROWSTATS off): same output; the block output carries its partials."""
    from comfy_gen_server_amd.models.attention import BasicTransformerBlock
    from comfy_gen_server_amd.models.layers import init_random_fast_
    monkeypatch.setenv("CGS_AUTOTUNE", "1")     # the tuned table (v6 on these shapes) decides the kernel
    torch.manual_seed(6)
    blk = BasicTransformerBlock(640, 10, 64, context_dim=2048, dtype=torch.bfloat16, device=cuda)
    init_random_fast_(blk, seed=3)
    # the SDXL level-1 shapes at UNet batch 16 (the tuned table runs their GEMMs on v6)
    x = torch.randn(16, 4096, 640, device=cuda).to(torch.bfloat16)
    ctx = torch.randn(16, 77, 2048, device=cuda).to(torch.bfloat16)
    with torch.inference_mode():
        y1 = blk(x, context=ctx, transformer_options={})
        assert getattr(y1, "_cgs_rowpart", None) is not None
        monkeypatch.setattr(core, "_RSO", False)
        y0 = blk(x, context=ctx, transformer_options={})
        assert getattr(y0, "_cgs_rowpart", None) is None
    assert _rel(y1, y0) < 5e-3


# w6 (gemm_w6.hip, variant 16): one wave per SIMD, 64-deep full-line LDS-DMA K-tiles, persistent with the
# next unit's first K-tiles prefetched under the current one; partial M / N tiles, several units per
# workgroup (M x N >> 256 tiles), every epilogue (bias, residual, GEGLU, LayerNorm fold, LN + GEGLU).
@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (300, 336, 640), (4096, 1280, 1280), (16384, 3840, 1280),
                                   (1232, 2560, 2048), (65536, 640, 640), (777, 4096, 256)])
@pytest.mark.parametrize("epi", ["none", "bias", "bias_res", "geglu", "ln", "ln_geglu"])
@pytest.mark.parametrize("variant", [16, 17], ids=["w6", "w6n160"])
def test_gemm_w6(cuda, M, N, K, epi, variant):
    lib = _native.load_kernels()
    torch.manual_seed(3)
    geglu, ln = "geglu" in epi, epi.startswith("ln")
    if geglu and (N % 32 or variant == 17):
        pytest.skip("GEGLU needs N % 32 == 0 and 256-wide tiles")
    x = (torch.randn(M, K, device=cuda) * (3 if ln else 1) + (1.5 if ln else 0)).to(torch.bfloat16)
    w = (torch.randn(N, K, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    b = torch.randn(N, device=cuda).to(torch.bfloat16) if epi != "none" else None
    nout = N // 2 if geglu else N
    r = torch.randn(M, N, device=cuda).to(torch.bfloat16) if epi == "bias_res" else None
    flags = (core.EPI_BIAS if b is not None else 0) | (core.EPI_RESIDUAL if r is not None else 0) | \
        (core.EPI_GEGLU if geglu else 0)
    if ln:
        gamma = (torch.rand(K, device=cuda) + 0.5).to(torch.bfloat16)
        beta = (torch.randn(K, device=cuda) * 0.2).to(torch.bfloat16)
        xf = F.layer_norm(x.float(), (K,), gamma.float(), beta.float(), 1e-5)
        rs = ops.layernorm_stats(x, 1e-5)
    else:
        xf = x.float()
    h = xf @ w.float().t() + (b.float() if b is not None else 0)
    if geglu:
        a_, g_ = h.chunk(2, dim=-1)
        ref = a_ * F.gelu(g_)
        wk, bk = core.geglu_interleave(w), core.geglu_interleave(b)
    else:
        ref = h + (r.float() if r is not None else 0)
        wk, bk = w, b
    y = torch.empty(M, nout, device=cuda, dtype=torch.bfloat16)
    if ln:
        w2, cs, b2 = ops.lnfold_weights(wk, bk, gamma, beta)
        assert lib.cgs_gemm_bf16_lnfold_v(x.data_ptr(), w2.data_ptr(), y.data_ptr(), b2.data_ptr(), rs.data_ptr(),
                                          cs.data_ptr(), M, N, K, K, K, nout, flags | core.EPI_BIAS, None, 0, variant,
                                          core._stream()) == 0
    else:
        assert lib.cgs_gemm_bf16_v(x.data_ptr(), wk.data_ptr(), y.data_ptr(), 0 if bk is None else bk.data_ptr(),
                                   0 if r is None else r.data_ptr(), M, N, K, K, K, nout, N if r is not None else 0,
                                   flags, 1.0, variant, core._stream()) == 0
    torch.cuda.synchronize()
    assert torch.isfinite(y).all()
    assert _rel(y, ref) < (1.5e-2 if ln else 1e-2), _rel(y, ref)


@pytest.mark.parametrize("C,C2,G,silu,pre", [(640, 0, 32, True, True), (1280, 0, 32, False, False),
                                              (640, 320, 32, True, False), (320, 0, 32, True, True)])
def test_row_sharded_groupnorm_native(cuda, C, C2, G, silu, pre):
    """Latency mode's row-sharded GroupNorm (parallel/spatial.py) on the native kernels: each band's
    (mean, M2) from cgs_groupnorm_band_stats, Chan-combined, applied by cgs_groupnorm_apply_stats -- two
    bands of one image reproduce the fp32 GroupNorm of the whole image; no ATen GroupNorm runs."""
    from comfy_gen_server_amd.parallel.spatial import SpatialShard
    torch.manual_seed(5)
    H, W = 32, 24
    x = (torch.randn(1, C, H, W, device=cuda) * 2 + 0.5).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    x2 = (torch.randn(1, C2, H, W, device=cuda)).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last) if C2 else None
    Ct = C + C2
    w = (torch.rand(Ct, device=cuda) + 0.5).to(torch.bfloat16)
    b = (torch.randn(Ct, device=cuda) * 0.1).to(torch.bfloat16)
    pa = torch.randn(1, Ct, device=cuda).to(torch.bfloat16) if pre else None
    xf = x.float() if x2 is None else torch.cat([x.float(), x2.float()], 1)
    if pa is not None:
        xf = xf + pa.float()[:, :, None, None]
    ref = F.group_norm(xf, G, w.float(), b.float(), 1e-5)
    if silu:
        ref = F.silu(ref)
    bands = []
    for r in range(2):
        sc = SpatialShard(None, 2, r, [0, 1])
        other = SpatialShard(None, 1, 0, [0])

        def gather(st, sc=sc, r=r):
            lo, hi = sc.band(H)
            olo, ohi = (hi, H) if r == 0 else (0, lo)
            xo = x[:, :, olo:ohi]
            x2o = None if x2 is None else x2[:, :, olo:ohi]
            # the other band's statistics through the same native kernel (a 1-rank shard of its rows)
            cap = {}
            other._gather_stats = lambda s2: cap.setdefault("s", s2)[None]
            other.group_norm(xo, G, w, b, 1e-5, silu=silu, pre_add=pa, x2=x2o)
            parts = [st, cap["s"]] if r == 0 else [cap["s"], st]
            return torch.stack(parts)
        sc._gather_stats = gather
        ops.reset_stats()
        lo, hi = sc.band(H)
        yb = sc.group_norm(x[:, :, lo:hi], G, w, b, 1e-5, silu=silu, pre_add=pa,
                           x2=None if x2 is None else x2[:, :, lo:hi])
        assert sc.stats.get("gn_native", 0) == 1
        assert ops.stats().get(("groupnorm", "hip"), 0) >= 1 and not any(k[1] == "lib" for k in ops.stats())
        bands.append(yb)
    y = torch.cat(bands, dim=2)
    assert _rel(y, ref) < 1e-2, _rel(y, ref)


@pytest.mark.parametrize("M,N,K", [(2048, 1280, 5120), (2048, 1280, 1280), (1000, 640, 2560), (333, 320, 1024)])
@pytest.mark.parametrize("epi", ["bias_res", "bias", "gelu", "ln"])
@pytest.mark.parametrize("name", ["sk2v8", "sk4v10", "sk2v11"])
def test_gemm_splitk(cuda, M, N, K, epi, name):
    """Split-K GEMM (K slices into fp32 partials, one reduce pass with the epilogue) vs fp32 torch."""
    if epi == "ln" and K > 2048:
        pytest.skip("LayerNorm statistics kernel: C <= 2048 (the LN-folded GEMMs have K <= 2048)")
    torch.manual_seed(11)
    x = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    w = (torch.randn(N, K, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    b = torch.randn(N, device=cuda).to(torch.bfloat16)
    r = torch.randn(M, N, device=cuda).to(torch.bfloat16) if epi == "bias_res" else None
    o = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    if epi == "ln":
        rs = core.layernorm_stats(x, 1e-5)
        w2, cs, b2 = core.lnfold_weights(w, b, None, None)
        core._splitk_run(x, w2, o, b2, None, rs, cs, M, N, K, core.EPI_BIAS | core.EPI_LNFOLD, name)
        ref = F.linear(F.layer_norm(x.float(), (K,), eps=1e-5), w.float(), b.float())
    else:
        e = core.EPI_BIAS | (core.EPI_RESIDUAL if r is not None else 0) | (core.EPI_GELU if epi == "gelu" else 0)
        core._splitk_run(x, w, o, b, r, None, None, M, N, K, e, name)
        ref = F.linear(x.float(), w.float(), b.float())
        if epi == "gelu":
            ref = F.gelu(ref)
        if r is not None:
            ref = ref + r.float()
    assert _rel(o, ref) < 1e-2


def test_gemm_splitk_is_a_linear_candidate(cuda, monkeypatch):
    """ops.linear on a batch-1 shape runs the split-K form when the tuning override picks it."""
    monkeypatch.setenv("CGS_AUTOTUNE", "1")
    monkeypatch.setenv("CGS_SPLITK", "1")                      # opt-in candidates (profiles/r05/splitk.md)
    monkeypatch.setenv("CGS_TUNE_OVERRIDE", '{"gemm|2048|1280|5120|3": "sk4v8"}')
    torch.manual_seed(12)
    x = torch.randn(2048, 5120, device=cuda).to(torch.bfloat16)
    w = (torch.randn(1280, 5120, device=cuda) / 64).to(torch.bfloat16)
    b = torch.randn(1280, device=cuda).to(torch.bfloat16)
    r = torch.randn(2048, 1280, device=cuda).to(torch.bfloat16)
    calls = []
    real = core._splitk_run
    monkeypatch.setattr(core, "_splitk_run", lambda *a: calls.append(a[-1]) or real(*a))
    y = ops.linear(x, w, b, residual=r)
    assert calls == ["sk4v8"]
    assert _rel(y, F.linear(x.float(), w.float(), b.float()) + r.float()) < 1e-2
