"""fp32-I/O device paths (csrc/kernels/f32.hip) for ``--force-fp32`` / ``--fp32-vae``.

The reference runs fp32 models on the vendor libraries (``comfy/cli_args.py:55`` ``--force-fp32``,
``:66`` ``--fp32-vae``; ROCm's default VAE dtype is fp32, ``comfy/model_management.py:169-197``).
Here an fp32 tensor reaching ``ops.linear`` / ``conv2d`` / ``group_norm`` / ``layer_norm`` /
``attention`` runs on the f32-input MFMA kernels instead: exact fp32 products (the fp32 GEMM's
numerics), fused bias / residual / GELU epilogues, the conv's channel concat and nearest-2x upsample
read in place. Each function returns None when the operands do not fit the kernels (the caller then
takes its existing fallback, which is counted as such).
"""
from __future__ import annotations

import math

import torch

from .. import _native

F32 = torch.float32
_BIAS, _RES, _GELU = 1, 2, 4
SCORE_BUDGET = 1 << 28          # fp32 elements of one attention score chunk (1 GiB)


def _lib():
    return _native.load_kernels()


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _check(rc, name):
    if rc != 0:
        raise RuntimeError(f"{name} failed: hip error {rc}")


def _ptr(t):
    return 0 if t is None else t.data_ptr()


def _vec_ok(t: torch.Tensor) -> bool:
    return t.data_ptr() % 16 == 0


def available(name: str = "cgs_gemm_f32") -> bool:
    return _native.has_kernel(name)


def _f32(t, device):
    if t is None:
        return None
    if t.dtype != F32 or t.device != device or not t.is_contiguous():
        t = t.to(device=device, dtype=F32).contiguous()
    return t


def gemm(a: torch.Tensor, w: torch.Tensor, out: torch.Tensor, *, bias=None, residual=None, gelu=False,
         alpha=1.0, bkn=False, batch=1, sab=0, sbb=0, scb=0, M=None, N=None, K=None,
         lda=None, ldb=None, ldc=None, ldr=0):
    """Raw launch of ``cgs_gemm_f32`` on fp32 operands (strides in elements)."""
    epi = (_BIAS if bias is not None else 0) | (_RES if residual is not None else 0) | (_GELU if gelu else 0)
    _check(_lib().cgs_gemm_f32(a.data_ptr(), w.data_ptr(), out.data_ptr(), _ptr(bias), _ptr(residual),
                               M, N, K, lda, ldb, ldc, ldr, epi, float(alpha), 1 if bkn else 0, batch, sab, sbb,
                               scb, _stream()), "cgs_gemm_f32")
    return out


def linear(x: torch.Tensor, weight: torch.Tensor, bias, residual, act, out):
    K = x.shape[-1]
    N = weight.shape[0]
    if weight.dtype != F32 or x.numel() == 0:
        return None
    a = x.reshape(-1, K)
    if a.stride(-1) != 1 or (a.shape[0] > 1 and a.stride(0) < K) or a.stride(0) % 4 or not _vec_ok(a):
        a = a.contiguous()
    if K % 4:         # row strides must be float4-aligned: pad K (the kernel zero-fills the K tail)
        Kp = (K + 3) // 4 * 4
        a = torch.nn.functional.pad(a, (0, Kp - K))
        weight = torch.nn.functional.pad(weight, (0, Kp - K))
    M = a.shape[0]
    w = weight if weight.is_contiguous() and _vec_ok(weight) else weight.contiguous()
    b = _f32(bias, x.device)
    r = None
    if residual is not None:
        r = residual.reshape(M, N).to(F32)
        if not r.is_contiguous():
            r = r.contiguous()
    y = out if out is not None else torch.empty((M, N), device=x.device, dtype=F32)
    gemm(a, w, y, bias=b, residual=r, gelu=act == "gelu", M=M, N=N, K=K, lda=a.stride(0), ldb=w.stride(0), ldc=N,
         ldr=N if r is not None else 0)
    return y.view(*x.shape[:-1], N)


def conv2d(x, weight, bias, stride, padding, residual, weight_nhwc, upsample2x, x2):
    """NHWC implicit-GEMM conv (groups = 1). Input channel counts that are not multiples of 4 (RGB
    stems) are zero-padded to 4 here; a concat partner whose split is not 4-aligned is materialised."""
    Cout, Cin_w, kh, kw = weight.shape
    if weight.dtype != F32 or x.dim() != 4:
        return None
    if x2 is not None and (x.shape[1] % 4 or x2.shape[1] % 4 or x2.dtype != F32):
        x = torch.cat([x, x2.to(F32)], dim=1)
        x2 = None
    N, C1, H, W = x.shape
    C2 = 0 if x2 is None else x2.shape[1]
    if C1 + C2 != Cin_w:
        return None
    wn = weight_nhwc if (weight_nhwc is not None and weight_nhwc.dtype == F32
                         and tuple(weight_nhwc.shape) == (Cout, kh, kw, Cin_w)
                         and weight_nhwc.is_contiguous()) else weight.permute(0, 2, 3, 1).contiguous()
    if x2 is None and C1 % 4:
        cp = (C1 + 3) // 4 * 4
        xp = torch.empty((N, cp, H, W), device=x.device, dtype=F32, memory_format=torch.channels_last)
        xp[:, C1:].zero_()
        xp[:, :C1] = x
        x, C1 = xp, cp
        wn = torch.nn.functional.pad(wn, (0, cp - Cin_w))
    xc = x.contiguous(memory_format=torch.channels_last)
    x2c = None if x2 is None else x2.contiguous(memory_format=torch.channels_last)
    if not _vec_ok(xc) or (x2c is not None and not _vec_ok(x2c)) or not _vec_ok(wn):
        return None
    Hl, Wl = (2 * H, 2 * W) if upsample2x else (H, W)
    Ho = (Hl + 2 * padding - kh) // stride + 1
    Wo = (Wl + 2 * padding - kw) // stride + 1
    y = torch.empty((N, Cout, Ho, Wo), device=x.device, dtype=F32, memory_format=torch.channels_last)
    r = None
    if residual is not None:
        r = residual.to(F32).contiguous(memory_format=torch.channels_last)
    _check(_lib().cgs_conv_f32(xc.data_ptr(), _ptr(x2c), wn.data_ptr(), _ptr(_f32(bias, x.device)), _ptr(r),
                               y.data_ptr(), N, H, W, C1, C2, Cout, kh, kw, stride, padding, 1 if upsample2x else 0,
                               Ho, Wo, _stream()), "cgs_conv_f32")
    return y


def group_norm(x, groups, weight, bias, eps, silu, x2, pre_add):
    N, C1, H, W = x.shape
    C = C1 + (0 if x2 is None else x2.shape[1])
    if C % groups or C % 4 or x.dim() != 4:
        return None
    if x2 is not None and (C1 % 4 or x2.dtype != F32):
        x = torch.cat([x, x2.to(F32)], dim=1)
        x2, C1 = None, C
    xc = x.contiguous(memory_format=torch.channels_last)
    x2c = None if x2 is None else x2.contiguous(memory_format=torch.channels_last)
    pa = None
    if pre_add is not None:
        pa = pre_add.to(F32).reshape(N, C).contiguous()
    if not _vec_ok(xc) or (x2c is not None and not _vec_ok(x2c)) or (pa is not None and not _vec_ok(pa)):
        return None
    y = torch.empty((N, C, H, W), device=x.device, dtype=F32, memory_format=torch.channels_last)
    ws = torch.empty(int(_lib().cgs_groupnorm_f32_ws(N, H * W, C)), device=x.device, dtype=F32)
    _check(_lib().cgs_groupnorm_f32(xc.data_ptr(), _ptr(x2c), C1, y.data_ptr(), _ptr(_f32(weight, x.device)),
                                    _ptr(_f32(bias, x.device)), _ptr(pa), ws.data_ptr(), N, H * W, C, groups,
                                    float(eps), 1 if silu else 0, _stream()), "cgs_groupnorm_f32")
    return y


def layer_norm(x, weight, bias, eps):
    C = x.shape[-1]
    if C % 4:
        return None
    xc = x.contiguous()
    if not _vec_ok(xc):
        return None
    y = torch.empty_like(xc)
    _check(_lib().cgs_layernorm_f32(xc.data_ptr(), y.data_ptr(), _ptr(_f32(weight, x.device)),
                                    _ptr(_f32(bias, x.device)), xc.numel() // C, C, float(eps), _stream()),
           "cgs_layernorm_f32")
    return y


def attention(q, k, v, heads, mask=None, causal=False, key_padding=None):
    """Exact fp32 attention: per image, chunks of query rows -> scores S = Q K^T / sqrt(d) for all heads
    in one batched launch (batch = heads, per-head views straight from [B, S, H*D]), masks applied to
    the chunk, row softmax in place (``cgs_softmax_rows``), O = P V in one batched launch (V read as
    [K, N]). Scores are bounded to ``SCORE_BUDGET`` elements per chunk."""
    B, Sq, HD = q.shape
    Sk = k.shape[1]
    D = HD // heads
    if D % 4 or k.dtype != F32 or v.dtype != F32:
        return None
    for t in (q, k, v):
        if t.stride(-1) != 1 or t.stride(1) % 4 or t.stride(0) % 4 or not _vec_ok(t):
            return None
    lib, st = _lib(), _stream()
    o = torch.empty((B, Sq, HD), device=q.device, dtype=F32)
    ld = (Sk + 3) // 4 * 4      # score row stride: float4-aligned rows for the PV GEMM's A loads
    rows = max(1, min(Sq, SCORE_BUDGET // max(1, heads * ld)))
    s = torch.empty((heads, rows, ld), device=q.device, dtype=F32)
    full_mask = None
    if mask is not None:     # normalised as attention_reference does: bool keep-mask -> 0 / -inf,
        m = mask               # [Sq, Sk] -> [1, 1, Sq, Sk], [B, Sq, Sk] -> [B, 1, Sq, Sk]
        if m.dtype == torch.bool:
            m = torch.zeros(m.shape, device=m.device, dtype=F32).masked_fill(~m, float("-inf"))
        full_mask = m.to(F32)
        while full_mask.dim() < 4:
            full_mask = full_mask.unsqueeze(0) if full_mask.dim() < 3 else full_mask.unsqueeze(1)
        try:
            full_mask = full_mask.expand(B, heads, Sq, Sk)
        except RuntimeError:
            return None
    scale = 1.0 / math.sqrt(D)
    for b in range(B):
        for r0 in range(0, Sq, rows):
            n = min(rows, Sq - r0)
            sc = s[:, :n, :Sk]
            if ld != Sk:    # pad columns join the row softmax as exp(-inf) = 0
                s[:, :, Sk:].fill_(float("-inf"))
            qb = q[b, r0:r0 + n]
            gemm(qb, k[b], s, alpha=scale, batch=heads, sab=D, sbb=D, scb=rows * ld, M=n, N=Sk, K=D,
                 lda=q.stride(1), ldb=k.stride(1), ldc=ld)
            if full_mask is not None:
                sc.add_(full_mask[b, :, r0:r0 + n])
            if causal:
                idx = torch.arange(r0, r0 + n, device=q.device)[:, None]
                sc.masked_fill_(torch.arange(Sk, device=q.device)[None, :] > idx, float("-inf"))
            if key_padding is not None:
                sc.masked_fill_(~key_padding[b].to(torch.bool)[None, None, :], float("-inf"))
            _check(lib.cgs_softmax_rows(s.data_ptr(), s.data_ptr(), heads * rows, ld, 1.0, 0, st), "cgs_softmax_rows")
            ob = o[b, r0:r0 + n]
            gemm(s, v[b], ob, bkn=True, batch=heads, sab=rows * ld, sbb=D, scb=D, M=n, N=D, K=Sk,
                 lda=ld, ldb=v.stride(1), ldc=HD)
    return o
