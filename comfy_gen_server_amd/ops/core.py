"""Op implementations: HIP launchers (device) and fp32 torch references (CPU / oracle).

Tensor conventions
  * token tensors: ``[B, S, C]`` with unit stride on C.
  * image tensors on the device: logical NCHW, physically NHWC (``torch.channels_last``), so a
    SpatialTransformer's ``b c h w -> b (h w) c`` is a free view and GroupNorm / conv kernels read
    rows of C contiguously.
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn.functional as F

from .. import _native
from . import autotune
from . import f32 as _f32
from .dispatch import backend_for, count, vendor_fallback

_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}

EPI_BIAS = 1
EPI_RESIDUAL = 2
EPI_GEGLU = 4
EPI_SILU_IN = 8   # reserved
EPI_LNFOLD = 8    # (C side: MC_EPI_LNFOLD; the LN-folded entry points add it themselves)
EPI_GELU = 32     # GELU(acc + bias) before the residual (v6 ACT kernel, mc::tile family, skinny)

# hipBLASLt (through ATen) as a GEMM autotune candidate: off unless explicitly requested -- the
# hand-written MFMA kernels (v5/v6/v7) are the device GEMMs; profiles/r02_gemm_table_v7.md has the
# per-shape comparison.
_LIB_GEMM = os.environ.get("CGS_GEMM_LIB", "0") == "1"


def _stream():
    return ctypes_stream(torch.cuda.current_stream())


def ctypes_stream(s):
    return s.cuda_stream


def _lib():
    return _native.load_kernels()


def _check(err: int, name: str):
    if err != 0:
        raise RuntimeError(f"{name} failed with hipError {err}")


def _ptr(t):
    return None if t is None else t.data_ptr()


# ----------------------------------------------------------------------------------------------
# GEMM family
# ----------------------------------------------------------------------------------------------
_V7WS: dict = {}
_V7_SPLIT = os.environ.get("CGS_V7_SPLIT", "1") != "0"


def _v7_ws(M: int, N: int, K: int, device):
    """Split-K tail workspace of the v7 GEMM / conv (mfma_ppk.h), from the caching allocator so it
    follows stream and graph-pool semantics; None when the shape's last round is full."""
    n = _V7WS.get((M, N, K))
    if n is None:
        n = int(_lib().cgs_v7_ws_bytes(M, N, K)) if _V7_SPLIT and _native.has_kernel("cgs_v7_ws_bytes") else 0
        _V7WS[(M, N, K)] = n
    return torch.empty(n, dtype=torch.uint8, device=device) if n else None


_SKWS: dict = {}


def _skinny_ws(M: int, N: int, K: int, device):
    """Split-K workspace of the skinny (M <= 128) GEMM, from the caching allocator; None = no split."""
    n = _SKWS.get((M, N, K))
    if n is None:
        n = int(_lib().cgs_gemm_skinny_ws_bytes(M, N, K)) if _native.has_kernel("cgs_gemm_skinny_ws_bytes") \
            and os.environ.get("CGS_SKINNY_SPLIT", "1") != "0" else 0
        _SKWS[(M, N, K)] = n
    return torch.empty(n, dtype=torch.uint8, device=device) if n else None


# D = 64 self-attention grids below this many 256-row workgroups are tuned among the small-grid forms
# (128-row blocks, key split): up to two rounds of the CUs (batch-1 SDXL level 1 is 320)
_ATTN_SMALL_WG = int(os.environ.get("CGS_ATTN_SMALL_WG", "512"))


def linear(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None = None,
           residual: torch.Tensor | None = None, act: str | None = None,
           out: torch.Tensor | None = None, row_stats: bool = False) -> torch.Tensor:
    """y = act(x @ weight^T (+ bias)) (+ residual). ``residual`` has y's shape (fused epilogue add);
    ``act="gelu"`` fuses the GELU into the epilogue (Cascade ChannelMLP Linear -> GELU); ``out``: a
    contiguous [rows, N] destination for the device path (e.g. one image's slice of a batch).
    ``row_stats``: when the shape runs on the v6 kernel, its epilogue also writes per-row LayerNorm
    statistics partials of y, attached as ``y._cgs_rowpart`` (see ``layernorm_stats_for``) -- the next
    LayerNorm-folded GEMM then skips the statistics pass over y.

    Device path: the HIP GEMM family (v7 persistent ping-pong 256x256x64 with a register epilogue,
    v6 persistent 256x160, v5 ping-pong 256x256, v3 8-wave 32x32 MFMA, v1 128x128), the kernel picked
    per shape by ``ops.autotune`` (hipBLASLt joins the candidates only with ``CGS_GEMM_LIB=1``)."""
    assert act in (None, "gelu"), act
    if weight.dtype == torch.float8_e4m3fn:
        if act is not None:
            return linear(x, weight.to(x.dtype), None if bias is None else bias.to(x.dtype), residual, act, out)
        return _linear_w8(x, weight, bias, residual)
    be = backend_for("gemm", x, "cgs_gemm_bf16")
    if be == "hip" and x.dtype == torch.float32 and weight.dtype == torch.float32 and _f32.available():
        y = _f32.linear(x, weight, bias, residual, act, out)     # --force-fp32 / --fp32-vae (f32.hip)
        if y is not None:
            count("gemm", "hip")
            return y
    # K % 8: the kernels' 16-byte row loads (a K=2 coordinate MLP is not GEMM-shaped work anyway)
    if be == "hip" and x.dtype == torch.bfloat16 and weight.dtype == torch.bfloat16 and x.shape[-1] % 8 == 0:
        K = x.shape[-1]
        N = weight.shape[0]
        a = x.reshape(-1, K)
        if a.stride(-1) != 1 or (a.shape[0] > 1 and a.stride(0) < K) or a.stride(0) % 8:
            a = a.contiguous()
        M = a.shape[0]
        epi = 0
        r = None
        if bias is not None:
            epi |= EPI_BIAS
        if residual is not None:
            epi |= EPI_RESIDUAL
            r = residual.reshape(M, N)
            if not r.is_contiguous():
                r = r.contiguous()
        gelu = act == "gelu"
        if gelu:
            epi |= EPI_GELU
        w = weight if weight.is_contiguous() else weight.contiguous()
        dst = out
        if dst is not None:
            assert dst.is_contiguous() and dst.numel() == M * N and dst.dtype == x.dtype, "out: contiguous [M, N]"

        rs_part = []

        def run_hip(variant, final=False):
            o = dst if dst is not None else torch.empty((M, N), device=x.device, dtype=x.dtype)
            if isinstance(variant, str):                       # split-K (batch-1 grids)
                return _splitk_run(a, w, o, bias, r, None, None, M, N, K, epi, variant)
            if (final and row_stats and variant in (6, 19, 20) and not gelu and N % 160 == 0 and K % 64 == 0
                    and K >= 128 and _RSO and _native.has_kernel("cgs_gemm_bf16_rowstats_v")):
                part = torch.empty((M, N // 80, 2), device=x.device, dtype=torch.float32)
                _check(_lib().cgs_gemm_bf16_rowstats_v(a.data_ptr(), w.data_ptr(), o.data_ptr(), _ptr(bias), _ptr(r),
                                                       M, N, K, a.stride(0), K, N, N if r is not None else 0, epi,
                                                       1.0, part.data_ptr(), variant, _stream()),
                       "cgs_gemm_bf16_rowstats_v")
                rs_part.append(part)
                return o
            if M <= 128 and variant in (-1, -2) and K % 32 == 0 and (a.data_ptr() | w.data_ptr()) % 16 == 0:
                ws = _skinny_ws(M, N, K, x.device)     # split-K slices when N / 16 workgroups underfill
                if ws is not None:
                    _check(_lib().cgs_gemm_skinny_ws(a.data_ptr(), w.data_ptr(), o.data_ptr(), _ptr(bias), _ptr(r),
                                                     M, N, K, a.stride(0), K, N, N if r is not None else 0, epi, 1.0,
                                                     ws.data_ptr(), ws.numel(), _stream()), "cgs_gemm_skinny_ws")
                    return o
            ws = _v7_ws(M, N, K, x.device) if variant == 7 else None
            if ws is not None:
                _check(_lib().cgs_gemm_bf16_v7ws(a.data_ptr(), w.data_ptr(), o.data_ptr(), _ptr(bias), _ptr(r),
                                                 M, N, K, a.stride(0), K, N, N if r is not None else 0, epi, 1.0,
                                                 ws.data_ptr(), ws.numel(), _stream()), "cgs_gemm_bf16_v7ws")
                return o
            _check(_lib().cgs_gemm_bf16_v(a.data_ptr(), w.data_ptr(), o.data_ptr(), _ptr(bias), _ptr(r),
                                          M, N, K, a.stride(0), K, N, N if r is not None else 0, epi, 1.0,
                                          variant, _stream()), "cgs_gemm_bf16")
            return o

        def run_lib():
            y = F.linear(a, w, bias)
            return y if r is None else y.add_(r)

        choice = "hip"
        # M <= 128 (one prompt through CLIP, time-embedding projections): the skinny kernel ("hip" ->
        # auto), weight-bandwidth bound; the big-tile kernels are not candidates there
        if M * N * K >= (1 << 27) and (M > 128 or K % 32):
            cands = []
            if K % 64 == 0 and N % 8 == 0:
                if K >= 128 and not gelu:
                    cands.append(("v7", lambda: run_hip(7)))
                if not gelu:
                    cands.append(("v5", lambda: run_hip(5)))
                if K >= 128 or not gelu:
                    cands.append(("v6", lambda: run_hip(6)))
            cands += _w6_cands(M, N, K, epi, run_hip)     # one wave per SIMD, full-line DMA, persistent
            if K % 32 == 0 and N % 8 == 0:
                cands.append(("v4", lambda: run_hip(4)))
                cands.append(("v8", lambda: run_hip(8)))      # 128 x 128 tiles (short M / N grids)
                if _underfilled(M, N):    # 64x128 / 128x64 tiles, 4- and 6-stage rings (batch-1 grids)
                    cands += [(f"v{v}", (lambda v=v: run_hip(v))) for v in _SMALL_TILE]
                    if K % 64 == 0 and K >= 128 and N % 160 == 0 and not gelu:   # 128 x 160 v6 tiles
                        cands.append(("v6m128", lambda: run_hip(V6_M128)))
                    if K % 64 == 0 and K >= 128 and N % 80 == 0 and not gelu:    # 128 x 80, 4-wave v6
                        cands.append(("v6w4", lambda: run_hip(V6_W4)))
                    if (a.stride(0) % 8 == 0 and (bias is None or bias.data_ptr() % 16 == 0)
                            and (r is None or r.data_ptr() % 16 == 0)):
                        cands += _splitk_cands(M, N, K, epi, run_hip)
            cands.append(("hip", lambda: run_hip(-1)))
            if _LIB_GEMM and not gelu and dst is None:     # vendor GEMM only as an explicit opt-in
                cands.append(("lib", run_lib))
            choice = autotune.choose(("gemm", M, N, K, epi), cands, default="hip")
        if choice == "lib" and (gelu or dst is not None):
            choice = "hip"
        if choice == "lib":
            count("gemm", "lib")     # explicit opt-in (CGS_GEMM_LIB=1)
            return run_lib().view(*x.shape[:-1], N)
        count("gemm", "hip")
        variant = choice if choice in _SPLITK else {"v7": 7, "v6": 6, "v5": 5, "v4": 4, "v8": 8, "w6": W6,
                                                    "w6n160": W6_160, "v6m128": V6_M128, "v6w4": V6_W4,
                                                    **_SMALL_NAMES}.get(choice, -2)
        y = run_hip(variant, final=True).view(*x.shape[:-1], N)
        if rs_part:
            # (no version counter: inference-mode tensors have none; the consumers take the partials only
            # on the hook-free transformer path, where y is never modified in place)
            y._cgs_rowpart = (rs_part[0], y.data_ptr())
        return y
    if be == "torch":
        count("gemm", "torch")
    else:
        vendor_fallback("gemm", f"dtype {x.dtype}/{weight.dtype}, K={x.shape[-1]}")
    if be == "torch":
        y = F.linear(x.float(), weight.float(), None if bias is None else bias.float())
        if act == "gelu":
            y = F.gelu(y)
        if residual is not None:
            y = y + residual.float()
        y = y.to(x.dtype)
    else:
        y = F.linear(x, weight, bias)
        if act == "gelu":
            y = F.gelu(y)
        if residual is not None:
            y = y + residual
    if out is not None:
        out.view(y.shape).copy_(y)
        return out.view(y.shape)
    return y


def _linear_w8(x, weight, bias, residual):
    """fp8-e4m3fn stored weights (K21, ``--fp8_e4m3fn-unet``): the device kernel widens the weight
    tiles to bf16 while staging them (exact), so HBM streams half the weight bytes; elsewhere the
    weight is cast up front (reference ``comfy/ops.py`` manual cast)."""
    be = backend_for("gemm", x, "cgs_gemm_bf16_w8")
    K = x.shape[-1]
    N = weight.shape[0]
    if be == "hip" and x.dtype == torch.bfloat16 and K % 8 == 0:
        count("gemm_w8", "hip")
        a = x.reshape(-1, K)
        if a.stride(-1) != 1 or (a.shape[0] > 1 and a.stride(0) < K) or a.stride(0) % 8 or a.data_ptr() % 16:
            a = a.contiguous()
        M = a.shape[0]
        w = weight.contiguous()
        epi = (EPI_BIAS if bias is not None else 0) | (EPI_RESIDUAL if residual is not None else 0)
        r = None if residual is None else residual.reshape(M, N).contiguous()
        b = None if bias is None else bias.to(torch.bfloat16).contiguous()
        out = torch.empty((M, N), device=x.device, dtype=x.dtype)
        _check(_lib().cgs_gemm_bf16_w8(a.data_ptr(), w.data_ptr(), out.data_ptr(), _ptr(b), _ptr(r), M, N, K,
                                       a.stride(0), K, N, N if r is not None else 0, epi, 1.0, _stream()),
               "cgs_gemm_bf16_w8")
        return out.view(*x.shape[:-1], N)
    return linear(x, weight.to(x.dtype), None if bias is None else bias.to(x.dtype), residual)


def linear_geglu(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None) -> torch.Tensor:
    """GEGLU (comfy/ldm/modules/attention.py:56-63): [a | g] = x W^T + b ; out = a * gelu(g).

    The device path fuses the gate into the GEMM epilogue; it needs the weight rows interleaved
    in 16-row groups [a0..a15, g0..g15, a16..] (``geglu_interleave``) — models keep that copy.
    """
    be = backend_for("gemm", x, "cgs_gemm_bf16")
    N2 = weight.shape[0]
    if be == "hip" and x.dtype == torch.bfloat16:
        count("gemm_geglu", "hip")
        K = x.shape[-1]
        a = x.reshape(-1, K)
        if not a.is_contiguous():
            a = a.contiguous()
        M = a.shape[0]
        epi = EPI_GEGLU | (EPI_BIAS if bias is not None else 0)

        def run_hip(variant):
            out = torch.empty((M, N2 // 2), device=x.device, dtype=x.dtype)
            ws = _v7_ws(M, N2, K, x.device) if variant == 7 else None
            if ws is not None:
                _check(_lib().cgs_gemm_bf16_v7ws(a.data_ptr(), weight.data_ptr(), out.data_ptr(), _ptr(bias), None,
                                                 M, N2, K, K, K, N2 // 2, 0, epi, 1.0, ws.data_ptr(), ws.numel(),
                                                 _stream()), "cgs_gemm_bf16_v7ws")
                return out
            _check(_lib().cgs_gemm_bf16_v(a.data_ptr(), weight.data_ptr(), out.data_ptr(), _ptr(bias), None,
                                          M, N2, K, K, K, N2 // 2, 0, epi, 1.0, variant, _stream()),
                   "cgs_gemm_bf16")
            return out

        choice = "hip"
        if M * N2 * K >= (1 << 27) and K % 32 == 0:
            cands = []
            if K % 64 == 0:
                if K >= 128:
                    cands.append(("v7", lambda: run_hip(7)))
                    if N2 % 160 == 0:    # 256x160 tiles with the GEGLU epilogue (pq::run GG)
                        cands.append(("v6", lambda: run_hip(6)))
                cands.append(("v5", lambda: run_hip(5)))
            if _w6_ok(M, N2, K, epi):
                cands.append(("w6", lambda: run_hip(W6)))
            cands.append(("v4", lambda: run_hip(4)))
            if _underfilled(M, N2):
                cands += [("v8", lambda: run_hip(8))] + [(f"v{v}", (lambda v=v: run_hip(v))) for v in _SMALL_TILE]
            cands.append(("hip", lambda: run_hip(-1)))
            choice = autotune.choose(("gemm_geglu", M, N2, K, epi), cands, default="hip")
        variant = {"v7": 7, "v6": 6, "v5": 5, "v4": 4, "v8": 8, "w6": W6, **_SMALL_NAMES}.get(choice, -2)
        return run_hip(variant).view(*x.shape[:-1], N2 // 2)
    count("gemm_geglu", be)
    # reference path expects the *interleaved* weight too, undo it
    w = geglu_deinterleave(weight)
    b = None if bias is None else geglu_deinterleave(bias)
    if be == "torch":
        h = F.linear(x.float(), w.float(), None if b is None else b.float())
        a, g = h.chunk(2, dim=-1)
        return (a * F.gelu(g)).to(x.dtype)
    h = F.linear(x, w, b)
    a, g = h.chunk(2, dim=-1)
    return a * F.gelu(g)


GEGLU_GROUP = 16


def geglu_interleave(w: torch.Tensor) -> torch.Tensor:
    """[a ; g] (2N rows) -> rows interleaved in groups of 16: a[0:16], g[0:16], a[16:32], ..."""
    n2 = w.shape[0]
    n = n2 // 2
    a, g = w[:n], w[n:]
    shp = (n // GEGLU_GROUP, GEGLU_GROUP) + tuple(w.shape[1:])
    return torch.stack([a.reshape(shp), g.reshape(shp)], dim=1).reshape(w.shape).contiguous()


def geglu_deinterleave(w: torch.Tensor) -> torch.Tensor:
    n2 = w.shape[0]
    shp = (n2 // (2 * GEGLU_GROUP), 2, GEGLU_GROUP) + tuple(w.shape[1:])
    v = w.reshape(shp)
    a = v[:, 0].reshape((n2 // 2,) + tuple(w.shape[1:]))
    g = v[:, 1].reshape((n2 // 2,) + tuple(w.shape[1:]))
    return torch.cat([a, g], dim=0)


# ----------------------------------------------------------------------------------------------
# Attention
# ----------------------------------------------------------------------------------------------
_FLASH_HEAD_DIMS = (32, 40, 64, 80, 96, 128, 160)
_ATTN_ALLOW_LIB = os.environ.get("CGS_ATTN_ALLOW_LIB", "0") == "1"


def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, heads: int,
              mask: torch.Tensor | None = None, causal: bool = False,
              key_padding: torch.Tensor | None = None) -> torch.Tensor:
    """softmax(q k^T / sqrt(d)) v over ``heads`` heads. q [B,Sq,H*D], k/v [B,Sk,H*D] -> [B,Sq,H*D].

    Softmax is accumulated in fp32 (reference upcast semantics, attention.py:104-107).
    ``mask``: additive float mask broadcastable to [B,H,Sq,Sk] (rare: torch path);
    ``causal``: CLIP causal mask; ``key_padding``: bool [B,Sk] True = attend.
    """
    B, Sq, HD = q.shape
    if k.shape[0] != B:
        # reference semantics when a patch re-batched the queries only (e.g. HyperTile): keys/values
        # are re-viewed with the query batch, i.e. split into contiguous token chunks (attention.py:337-350)
        k = k.reshape(B, -1, k.shape[-1])
        v = v.reshape(B, -1, v.shape[-1])
    Sk = k.shape[1]
    D = HD // heads
    be = backend_for("attention", q, "cgs_flash_attn_fwd")
    if be == "hip" and q.dtype == torch.float32 and _f32.available():
        o = _f32.attention(q, k, v, heads, mask=mask, causal=causal, key_padding=key_padding)
        if o is not None:
            count("attention", "hip")
            return o
    wide_ok = D == 512 and not causal and key_padding is None
    if (be == "hip" and mask is None and (D in _FLASH_HEAD_DIMS or wide_ok) and q.dtype == torch.bfloat16
            and q.stride(-1) == 1 and k.stride(-1) == 1 and v.stride(-1) == 1):
        kp = None
        if key_padding is not None:
            kp = key_padding.to(torch.int8).contiguous()

        def run_hip():
            o = torch.empty((B, Sq, HD), device=q.device, dtype=q.dtype)
            _check(_lib().cgs_flash_attn_fwd(
                q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                B, heads, Sq, Sk, D,
                q.stride(0), q.stride(1), D, k.stride(0), k.stride(1), D, v.stride(0), v.stride(1), D,
                o.stride(0), o.stride(1), D,
                1.0 / math.sqrt(D), _ptr(kp), 1 if causal else 0, _stream()), "cgs_flash_attn_fwd")
            return o

        if (wide_ok and heads == 1 and _WIDE_MAT and kp is None and Sk % 64 == 0 and Sk <= 16384
                and Sq * Sk >= (1 << 22)
                and _native.has_kernel("cgs_softmax2_f32_bf16") and _wide_mat_ok(q, k, v)):
            count("attention", "hip")
            return _attention_wide_mat(q, k, v)
        choice = "hip"
        # D = 64 self-attention whose 256-query blocks leave CUs idle (batch 1-2 at level 2: B*H*Sq/256
        # < 256 workgroups): the 128-row form of the fast kernel and the generic kernel are measured
        # alternatives
        if (kp is None and not causal and D == 64 and Sk > 128 and B * heads * ((Sq + 255) // 256) < _ATTN_SMALL_WG
                and B * heads * Sq * Sk >= (1 << 22) and _native.has_kernel("cgs_flash_attn_fwd_v")):
            def run_v(var):
                o = torch.empty((B, Sq, HD), device=q.device, dtype=q.dtype)
                _check(_lib().cgs_flash_attn_fwd_v(
                    q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), B, heads, Sq, Sk, D,
                    q.stride(0), q.stride(1), D, k.stride(0), k.stride(1), D, v.stride(0), v.stride(1), D,
                    o.stride(0), o.stride(1), D, 1.0 / math.sqrt(D), var, _stream()), "cgs_flash_attn_fwd_v")
                return o
            def run_ks(ks):
                o = torch.empty((B, Sq, HD), device=q.device, dtype=q.dtype)
                ws_o = torch.empty((ks * B * Sq * HD,), device=q.device, dtype=q.dtype)
                ws_l = torch.empty((ks * B * heads * Sq,), device=q.device, dtype=torch.float32)
                _check(_lib().cgs_flash_attn_fwd_ks(
                    q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), B, heads, Sq, Sk, q.stride(0), q.stride(1),
                    k.stride(0), k.stride(1), v.stride(0), v.stride(1), o.stride(0), o.stride(1), 1.0 / math.sqrt(D),
                    ks, ws_o.data_ptr(), ws_l.data_ptr(), _stream()), "cgs_flash_attn_fwd_ks")
                return o
            # d64: 256-row Q blocks (8 waves); d64q128: 128-row blocks, 4 waves, two WGs per CU; d64ks2 / 4: the
            # keys split 2 / 4 ways (KS x the workgroups) and the partials merged by log-sum-exp
            cands = [("d64", lambda: run_v(2)), ("d64q128", lambda: run_v(5)), ("generic", lambda: run_v(1))]
            tiles = (Sk + 63) // 64
            if _native.has_kernel("cgs_flash_attn_fwd_ks") and q.data_ptr() % 16 == 0:
                for ks in (2, 4):
                    if tiles >= 4 * ks and (ks - 1) * ((tiles + ks - 1) // ks) * 64 < Sk:
                        cands.append((f"d64ks{ks}", (lambda ks=ks: run_ks(ks))))
            sel = autotune.choose(("attention_grid2", B, heads, Sq, Sk, D), cands, default="d64q128")
            count("attention", "hip")
            if sel in ("d64ks2", "d64ks4"):
                return run_ks(int(sel[-1]))
            return run_v({"d64": 2, "d64q128": 5}.get(sel, 1))
        # The vendor SDPA is a tuning candidate only on explicit request: the hot path is the
        # hand-written kernel (K02/K03), never an SDPA fallback.
        if kp is None and _ATTN_ALLOW_LIB and B * heads * Sq * Sk >= (1 << 22):
            choice = autotune.choose(("attention", B, heads, Sq, Sk, D, int(causal)),
                                     [("hip", run_hip), ("lib", lambda: _sdpa(q, k, v, heads, causal))],
                                     default="hip")
        if choice == "lib":
            count("attention", "lib")
            return _sdpa(q, k, v, heads, causal)
        count("attention", "hip")
        return run_hip()
    if q.device.type != "cpu":
        vendor_fallback("attention", f"dtype {q.dtype}, head dim {D}, mask={mask is not None}")
        if mask is None and key_padding is None:
            return _sdpa(q, k, v, heads, causal)
    else:
        count("attention", "torch")
    return attention_reference(q, k, v, heads, mask=mask, causal=causal, key_padding=key_padding)


def attention_kv2(q: torch.Tensor, k1: torch.Tensor, v1: torch.Tensor, k2: torch.Tensor, v2: torch.Tensor,
                  heads: int) -> torch.Tensor:
    """``attention(q, cat([k1, k2], 1), cat([v1, v2], 1), heads)`` without materialising either concat:
    the D = 64 kernel reads keys [0, S1) from k1 / v1 and [S1, S1 + S2) from k2 / v2 (Stable Cascade's
    self-attention over cat([x, kv]), cascade/common.py Attention2D). Inputs may be strided views (last
    dim contiguous), e.g. column slices of one fused QKV projection."""
    B, Sq, HD = q.shape
    D = HD // heads
    ok = (D == 64 and q.is_cuda and q.dtype == torch.bfloat16 and all(
        t.dtype == q.dtype and t.dim() == 3 and t.shape[0] == B and t.shape[2] == HD and t.stride(-1) == 1
        for t in (k1, v1, k2, v2)) and k1.shape[1] == v1.shape[1] and k2.shape[1] == v2.shape[1]
        and q.stride(-1) == 1 and backend_for("attention", q, "cgs_flash_attn_fwd_kv2") == "hip")
    if ok:
        o = torch.empty((B, Sq, HD), device=q.device, dtype=q.dtype)
        err = _lib().cgs_flash_attn_fwd_kv2(
            q.data_ptr(), k1.data_ptr(), v1.data_ptr(), k2.data_ptr(), v2.data_ptr(), o.data_ptr(), B, heads, Sq,
            k1.shape[1], k2.shape[1], q.stride(0), q.stride(1), k1.stride(0), k1.stride(1), v1.stride(0), v1.stride(1),
            k2.stride(0), k2.stride(1), v2.stride(0), v2.stride(1), o.stride(0), o.stride(1), 1.0 / math.sqrt(D),
            _stream())
        if err == 0:
            count("attention", "hip")
            return o
    return attention(q, torch.cat([k1, k2.to(k1.dtype)], dim=1), torch.cat([v1, v2.to(v1.dtype)], dim=1), heads)


def attention_bias(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, bias: torch.Tensor,
                   mask: torch.Tensor | None = None, scale: float | None = None,
                   head_scale: torch.Tensor | None = None) -> torch.Tensor:
    """Head-major windowed attention with additive score terms (Swin-family upscalers: SwinIR / Swin2SR /
    HAT / DAT / OmniSR / SCUNet, reference ``comfy_extras/chainner_models/architecture/SwinIR.py:176-186``):

        softmax(scale * head_scale[h] * q k^T + bias[h] + mask[b % nW]) v        (fp32 scores and softmax)

    q [B, H, Sq, D], k / v [B, H, Sk, D] (last dim contiguous), ``bias`` [H, Sq, Sk], ``mask`` [nW, Sq, Sk]
    additive float (or bool, True = blocked) with B % nW == 0 -- the window index of batch entry b is
    b % nW, the (image, window) flattening of ``_partition``. ``head_scale`` [H] (SwinV2's clamped, exponentiated
    logit scale on cosine scores) is applied to the fp32 scores. Returns [B, H, Sq, D] in q's dtype.
    bf16 on the GPU runs the generic flash kernel with the terms added in its softmax loop (no [B, H, Sq,
    Sk] score tensor); head dims that are not a multiple of 8 (Swin's 30) are zero-padded."""
    B, H, Sq, D = q.shape
    Sk = k.shape[2]
    scale = D ** -0.5 if scale is None else float(scale)
    if mask is not None and mask.dtype == torch.bool:
        mask = torch.zeros(mask.shape, device=mask.device, dtype=torch.float32).masked_fill(mask, float("-inf"))
    nW = 1 if mask is None else mask.shape[0]
    ok = (q.is_cuda and q.dtype == torch.bfloat16 and k.dtype == q.dtype and v.dtype == q.dtype and D <= 160
          and B % nW == 0 and tuple(bias.shape) == (H, Sq, Sk)
          and (mask is None or tuple(mask.shape[1:]) == (Sq, Sk))
          and backend_for("attention", q, "cgs_flash_attn_fwd_bias") == "hip")
    if ok:
        Dp = (D + 7) // 8 * 8

        def prep(t):
            if Dp != D:
                return F.pad(t, (0, Dp - D))
            return t if t.stride(-1) == 1 and t.stride(2) % 8 == 0 and t.stride(1) % 8 == 0 and t.stride(0) % 8 == 0 \
                and t.data_ptr() % 16 == 0 else t.contiguous()
        qp, kp, vp = prep(q), prep(k), prep(v)
        bias_f = bias.float().contiguous()
        mask_f = None if mask is None else mask.float().contiguous()
        hs = None if head_scale is None else head_scale.float().reshape(H).contiguous()
        o = torch.empty((B, Sq, H, Dp), device=q.device, dtype=q.dtype)
        _check(_lib().cgs_flash_attn_fwd_bias(
            qp.data_ptr(), kp.data_ptr(), vp.data_ptr(), o.data_ptr(), B, H, Sq, Sk, Dp,
            qp.stride(0), qp.stride(2), qp.stride(1), kp.stride(0), kp.stride(2), kp.stride(1),
            vp.stride(0), vp.stride(2), vp.stride(1), o.stride(0), o.stride(1), o.stride(2),
            scale, bias_f.data_ptr(), _ptr(mask_f), nW, _ptr(hs), _stream()), "cgs_flash_attn_fwd_bias")
        count("attention", "hip")
        return o[..., :D].transpose(1, 2)
    if q.device.type != "cpu":
        vendor_fallback("attention", f"bias attention dtype {q.dtype}, head dim {D}")
    else:
        count("attention", "torch")
    s = ((q * scale) @ k.transpose(-2, -1)).float()                      # the models' own eager math
    if head_scale is not None:
        s = s * head_scale.float().reshape(H, 1, 1)
    s = s + bias.float()
    if mask is not None:
        s = (s.view(B // nW, nW, H, Sq, Sk) + mask.float()[None, :, None]).view(B, H, Sq, Sk)
    return torch.softmax(s, -1).to(v.dtype) @ v


def attention_lse(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, heads: int):
    """Unmasked attention plus the natural-log log-sum-exp of the scaled scores per (b, h, query):
    ``(o [B, Sq, H*D] in q's dtype, lse fp32 [B, H, Sq])`` -- the partial result of one K/V block
    that ring attention (parallel/sp.py) merges across blocks. Device: the flash kernels (D = 64
    fast kernel, generic D <= 160) write the LSE from their running max / sum; else fp32 torch."""
    B, Sq, HD = q.shape
    Sk = k.shape[1]
    D = HD // heads
    be = backend_for("attention", q, "cgs_flash_attn_fwd_lse")
    if (be == "hip" and D in _FLASH_HEAD_DIMS and q.dtype == torch.bfloat16 and k.dtype == q.dtype
            and v.dtype == q.dtype and q.stride(-1) == 1 and k.stride(-1) == 1 and v.stride(-1) == 1 and Sk > 0):
        o = torch.empty((B, Sq, HD), device=q.device, dtype=q.dtype)
        lse = torch.empty((B, heads, Sq), device=q.device, dtype=torch.float32)
        count("attention", "hip")
        _check(_lib().cgs_flash_attn_fwd_lse(
            q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr(), B, heads, Sq, Sk, D,
            q.stride(0), q.stride(1), D, k.stride(0), k.stride(1), D, v.stride(0), v.stride(1), D,
            o.stride(0), o.stride(1), D, 1.0 / math.sqrt(D), _stream()), "cgs_flash_attn_fwd_lse")
        return o, lse
    if q.device.type != "cpu":
        vendor_fallback("attention", f"LSE form: dtype {q.dtype}, head dim {D}")
    else:
        count("attention", "torch")
    qh = q.float().reshape(B, Sq, heads, D).transpose(1, 2)
    kh = k.float().reshape(B, Sk, heads, D).transpose(1, 2)
    vh = v.float().reshape(B, Sk, heads, D).transpose(1, 2)
    s = (qh @ kh.transpose(-2, -1)) * (D ** -0.5)
    lse = torch.logsumexp(s, dim=-1)
    o = (torch.softmax(s, dim=-1) @ vh).transpose(1, 2).reshape(B, Sq, HD)
    return o.to(q.dtype), lse


def fourier_filter(x: torch.Tensor, threshold: int, scale: float) -> torch.Tensor:
    """FreeU's Fourier filter (K29, comfy_extras/nodes_freelunch.py:6-23): scale the 2t x 2t
    low-frequency square of every channel's centred spectrum by ``scale``. Device: the (2t)^2 DFT
    coefficients it touches are reduced directly and the filtered image rebuilt as x + (scale - 1) x
    their inverse transform (exact: the filter is linear and only those modes change); CPU / fp32 /
    t > 4: torch.fft as the reference does."""
    B, C, H, W = x.shape
    t = int(threshold)
    be = backend_for("fourier", x, "cgs_fourier_filter")
    if be == "hip" and x.dtype in (torch.bfloat16, torch.float16) and 1 <= t <= 4 and 2 * t <= min(H, W):
        y = torch.empty_like(x)
        coef = torch.empty((B, C, 4 * t * t, 2), device=x.device, dtype=torch.float32)
        count("fourier", "hip")
        _check(_lib().cgs_fourier_filter(x.data_ptr(), y.data_ptr(), coef.data_ptr(), B, C, H, W, *x.stride(),
                                         *y.stride(), t, float(scale), _DT[x.dtype], _stream()), "cgs_fourier_filter")
        return y
    if x.device.type == "cpu":
        count("fourier", "torch")
    else:
        vendor_fallback("fourier", f"dtype {x.dtype}, threshold {t}, {H}x{W}")
    xf = torch.fft.fftshift(torch.fft.fftn(x.float(), dim=(-2, -1)), dim=(-2, -1))
    mask = torch.ones((B, C, H, W), device=x.device)
    ch, cw = H // 2, W // 2
    mask[..., ch - t:ch + t, cw - t:cw + t] = scale
    out = torch.fft.ifftn(torch.fft.ifftshift(xf * mask, dim=(-2, -1)), dim=(-2, -1)).real
    return out.to(x.dtype)


def tome_match(a: torch.Tensor, b: torch.Tensor):
    """ToMe bipartite matching (K30, comfy_extras/nodes_tomesd.py:22-160): for every src token a_i
    the most cosine-similar dst token, ``(max_j cos(a_i, b_j) fp32 [B, Na], argmax int64 [B, Na])``.
    Device: one fused HIP kernel (row norms, 64x64 fp32 score tiles folded into a running argmax);
    CPU: normalise + matmul + max as the reference does."""
    B, Na, C = a.shape
    Nb = b.shape[1]
    be = backend_for("tome", a, "cgs_tome_match")
    if (be == "hip" and a.dtype in (torch.bfloat16, torch.float16) and b.dtype == a.dtype and a.stride(-1) == 1
            and b.stride(-1) == 1 and Nb > 0):
        ws = torch.empty(B * (Na + Nb), device=a.device, dtype=torch.float32)
        vmax = torch.empty((B, Na), device=a.device, dtype=torch.float32)
        imax = torch.empty((B, Na), device=a.device, dtype=torch.int64)
        count("tome", "hip")
        _check(_lib().cgs_tome_match(a.data_ptr(), b.data_ptr(), ws.data_ptr(), vmax.data_ptr(), imax.data_ptr(), B,
                                     Na, Nb, C, a.stride(0), a.stride(1), b.stride(0), b.stride(1), _DT[a.dtype],
                                     _stream()), "cgs_tome_match")
        return vmax, imax
    if a.device.type == "cpu":
        count("tome", "torch")
    else:
        vendor_fallback("tome", f"dtype {a.dtype}")
    an = a / a.norm(dim=-1, keepdim=True)
    bn = b / b.norm(dim=-1, keepdim=True)
    return (an @ bn.transpose(-1, -2)).max(dim=-1)


EPI_F32OUT = 16
# K22: one-head D=512 attention (KL-VAE mid block) through materialised scores (CGS_WIDE_ATTN=flash
# keeps the flash kernel). S chunks are capped at 2^28 elements (1 GiB fp32).
_WIDE_MAT = os.environ.get("CGS_WIDE_ATTN", "mat") != "flash"
_WIDE_CHUNK_ELEMS = 1 << 28


def _wide_mat_ok(q, k, v) -> bool:
    ts = (q, k, v)
    return (all(t.stride(1) % 8 == 0 and t.stride(0) % 8 == 0 and t.data_ptr() % 16 == 0 for t in ts)
            and q.shape[1] * q.stride(1) * 2 < (1 << 32) and k.shape[1] * k.stride(1) * 2 < (1 << 32))


def _attention_wide_mat(q, k, v):
    """softmax(q k^T / sqrt(d)) v for one head of d = 512, per image and query chunk:
    S = (log2e / sqrt(d)) q k^T on the v7 GEMM with an fp32 epilogue, P = softmax2(S) -> bf16 in one
    pass, O = P V on the v7 GEMM against V^T (transposed once per image). The reference computes the
    same op through a materialised softmax too (comfy/ldm/modules/diffusionmodules/model.py:227-292)."""
    B, Sq, D = q.shape
    Sk = k.shape[1]
    lib, st = _lib(), _stream()
    dev = q.device
    o = torch.empty((B, Sq, D), device=dev, dtype=q.dtype)
    chunk = max(256, min(Sq, _WIDE_CHUNK_ELEMS // Sk))
    s = torch.empty((chunk, Sk), device=dev, dtype=torch.float32)
    p = torch.empty((chunk, Sk), device=dev, dtype=torch.bfloat16)
    vt = torch.empty((D, Sk), device=dev, dtype=torch.bfloat16)
    alpha = 1.4426950408889634 / math.sqrt(D)
    for b in range(B):
        _check(lib.cgs_transpose_bf16(v[b].data_ptr(), vt.data_ptr(), Sk, D, v.stride(1), Sk, st), "cgs_transpose_bf16")
        for r0 in range(0, Sq, chunk):
            m = min(chunk, Sq - r0)
            qa = q.data_ptr() + 2 * (b * q.stride(0) + r0 * q.stride(1))
            ws = _v7_ws(m, Sk, D, dev)
            _check(lib.cgs_gemm_bf16_v7ws(qa, k[b].data_ptr(), s.data_ptr(), None, None, m, Sk, D, q.stride(1),
                                          k.stride(1), Sk, 0, EPI_F32OUT, alpha, _ptr(ws),
                                          0 if ws is None else ws.numel(), st), "cgs_gemm_bf16_v7ws(f32)")
            _check(lib.cgs_softmax2_f32_bf16(s.data_ptr(), p.data_ptr(), m, Sk, Sk, Sk, st), "cgs_softmax2_f32_bf16")
            ws = _v7_ws(m, D, Sk, dev)
            oa = o.data_ptr() + 2 * (b * o.stride(0) + r0 * o.stride(1))
            _check(lib.cgs_gemm_bf16_v7ws(p.data_ptr(), vt.data_ptr(), oa, None, None, m, D, Sk, Sk, Sk, D, 0, 0, 1.0,
                                          _ptr(ws), 0 if ws is None else ws.numel(), st), "cgs_gemm_bf16_v7ws")
    return o


def _sdpa(q, k, v, heads, causal=False):
    """Vendor attention through ATen (ROCm SDPA); layout [B,S,H*D] in and out."""
    B, Sq, HD = q.shape
    Sk = k.shape[1]
    D = HD // heads
    qh = q.view(B, Sq, heads, D).transpose(1, 2)
    kh = k.view(B, Sk, heads, D).transpose(1, 2) if k.is_contiguous() else k.reshape(B, Sk, heads, D).transpose(1, 2)
    vh = v.view(B, Sk, heads, D).transpose(1, 2) if v.is_contiguous() else v.reshape(B, Sk, heads, D).transpose(1, 2)
    o = F.scaled_dot_product_attention(qh, kh, vh, is_causal=causal)
    return o.transpose(1, 2).reshape(B, Sq, HD)


def attention_reference(q, k, v, heads, mask=None, causal=False, key_padding=None):
    B, Sq, HD = q.shape
    Sk = k.shape[1]
    D = HD // heads
    qh = q.reshape(B, Sq, heads, D).transpose(1, 2).float()
    kh = k.reshape(B, Sk, heads, D).transpose(1, 2).float()
    vh = v.reshape(B, Sk, heads, D).transpose(1, 2).float()
    s = torch.matmul(qh, kh.transpose(-1, -2)) * (1.0 / math.sqrt(D))
    if mask is not None:
        m = mask
        if m.dtype == torch.bool:
            m = torch.zeros_like(m, dtype=s.dtype).masked_fill(~m, float("-inf"))
        while m.ndim < 4:
            m = m.unsqueeze(0) if m.ndim < 3 else m.unsqueeze(1)
        s = s + m.float()
    if causal:
        cm = torch.ones(Sq, Sk, dtype=torch.bool, device=q.device).triu(1)
        s = s.masked_fill(cm, float("-inf"))
    if key_padding is not None:
        s = s.masked_fill(~key_padding.bool()[:, None, None, :], float("-inf"))
    p = torch.softmax(s, dim=-1)
    o = torch.matmul(p, vh)
    return o.transpose(1, 2).reshape(B, Sq, HD).to(q.dtype)


# ----------------------------------------------------------------------------------------------
# Normalisation
# ----------------------------------------------------------------------------------------------
def group_norm(x: torch.Tensor, groups: int, weight: torch.Tensor | None, bias: torch.Tensor | None,
               eps: float, silu: bool = False, pre_add: torch.Tensor | None = None,
               x2: torch.Tensor | None = None) -> torch.Tensor:
    """GroupNorm (+ fused SiLU) over a 4-D image tensor (K06).

    ``pre_add`` ([N, C]) is added per (sample, channel) BEFORE normalising — this is how the
    ResBlock timestep-embedding add (openaimodel.py:245-264) is fused into the GroupNorm kernel.
    ``x2``: normalise ``cat([x, x2], 1)`` without materialising the concat (K14, the UNet decoder's
    skip connection, openaimodel.py:879); the kernel reads each 8-channel vector from its source.
    Inside a row-sharded UNet call (parallel/spatial.py) the statistics are summed over the ranks.
    """
    sc = _spatial()
    if sc is not None and x.dim() == 4:
        return sc.group_norm(x, groups, weight, bias, eps, silu=silu, pre_add=pre_add, x2=x2)
    be = backend_for("groupnorm", x, "cgs_groupnorm_nhwc_ws")
    Ct = x.shape[1] + (0 if x2 is None else x2.shape[1])
    if be == "hip" and x.dim() == 4 and x.dtype == torch.float32 and _f32.available("cgs_groupnorm_f32"):
        y = _f32.group_norm(x, groups, weight, bias, eps, silu, x2, pre_add)     # f32.hip
        if y is not None:
            count("groupnorm", "hip")
            return y
    if be == "hip" and x.dim() == 4 and x.dtype in (torch.bfloat16, torch.float16) and \
            weight is not None and Ct % 8 == 0 and Ct % groups == 0 and Ct <= 8192 and \
            Ct % (8 * ((Ct + 2047) // 2048)) == 0 and x.shape[1] % 8 == 0 and \
            (x2 is None or (x2.dtype == x.dtype and x2.shape[0] == x.shape[0] and x2.shape[2:] == x.shape[2:])):
        count("groupnorm", "hip")
        N, C1, H, W = x.shape
        C = Ct
        # the kernel reads gamma/beta in the activation dtype: cast fp8 / offloaded / mixed-dtype params
        if weight.dtype != x.dtype or weight.device != x.device or not weight.is_contiguous():
            weight = weight.to(device=x.device, dtype=x.dtype).contiguous()
        if bias is not None and (bias.dtype != x.dtype or bias.device != x.device or not bias.is_contiguous()):
            bias = bias.to(device=x.device, dtype=x.dtype).contiguous()
        xc = x.contiguous(memory_format=torch.channels_last)
        y = torch.empty((N, C, H, W), device=x.device, dtype=x.dtype, memory_format=torch.channels_last)
        pa, pld = None, C
        if pre_add is not None:
            pa = pre_add.to(x.dtype)
            # a [N, C] column slice of a wider row-major tensor (the UNet's batched time-embedding projection)
            # is read in place through a row stride; anything else is made contiguous
            if not (pa.dim() == 2 and pa.shape == (N, C) and pa.stride(1) == 1 and pa.stride(0) >= C
                    and _native.has_kernel("cgs_groupnorm_nhwc_ws_pld")):
                pa = pa.contiguous()
            pld = pa.stride(0) if pa.dim() == 2 and N > 1 else C
        strided = pa is not None and pld != C
        gp = getattr(x, "_cgs_gnpart", None) if x2 is None else None
        if gp is not None and gp[1] == x.data_ptr() and xc is x and gp[0].numel() == N * (H * W // 64) * C * 2 \
                and _native.has_kernel("cgs_groupnorm_nhwc_part"):
            # statistics from the producing conv's epilogue (conv2d(gn_stats=True)): finalize + apply only
            ab = torch.empty(N * C * 2, device=x.device, dtype=torch.float32)
            if strided:
                _check(_lib().cgs_groupnorm_nhwc_part_pld(xc.data_ptr(), y.data_ptr(), weight.data_ptr(), _ptr(bias),
                                                          pa.data_ptr(), pld, gp[0].data_ptr(), ab.data_ptr(), N,
                                                          H * W, C, groups, 64, float(eps), 1 if silu else 0,
                                                          _DT[x.dtype], _stream()), "cgs_groupnorm_nhwc_part_pld")
            else:
                _check(_lib().cgs_groupnorm_nhwc_part(xc.data_ptr(), y.data_ptr(), weight.data_ptr(), _ptr(bias),
                                                      _ptr(pa), gp[0].data_ptr(), ab.data_ptr(), N, H * W, C, groups,
                                                      64, float(eps), 1 if silu else 0, _DT[x.dtype], _stream()),
                       "cgs_groupnorm_nhwc_part")
            return y
        wsb = int(_lib().cgs_groupnorm_workspace(N, H * W, C))
        ws = torch.empty((wsb + 3) // 4, device=x.device, dtype=torch.float32)
        if x2 is None:
            if strided:
                _check(_lib().cgs_groupnorm_nhwc_ws_pld(xc.data_ptr(), y.data_ptr(), weight.data_ptr(), _ptr(bias),
                                                        pa.data_ptr(), pld, ws.data_ptr(), N, H * W, C, groups,
                                                        float(eps), 1 if silu else 0, _DT[x.dtype], _stream()),
                       "cgs_groupnorm_nhwc_ws_pld")
            else:
                _check(_lib().cgs_groupnorm_nhwc_ws(xc.data_ptr(), y.data_ptr(), weight.data_ptr(),
                                                    _ptr(bias), _ptr(pa), ws.data_ptr(), N, H * W, C, groups,
                                                    float(eps), 1 if silu else 0, _DT[x.dtype], _stream()),
                       "cgs_groupnorm_nhwc_ws")
        else:
            x2c = x2.contiguous(memory_format=torch.channels_last)
            if strided:
                _check(_lib().cgs_groupnorm_nhwc_dual_pld(xc.data_ptr(), x2c.data_ptr(), C1, y.data_ptr(),
                                                          weight.data_ptr(), _ptr(bias), pa.data_ptr(), pld,
                                                          ws.data_ptr(), N, H * W, C, groups, float(eps),
                                                          1 if silu else 0, _DT[x.dtype], _stream()),
                       "cgs_groupnorm_nhwc_dual_pld")
            else:
                _check(_lib().cgs_groupnorm_nhwc_dual(xc.data_ptr(), x2c.data_ptr(), C1, y.data_ptr(),
                                                      weight.data_ptr(), _ptr(bias), _ptr(pa), ws.data_ptr(), N, H * W,
                                                      C, groups, float(eps), 1 if silu else 0, _DT[x.dtype],
                                                      _stream()), "cgs_groupnorm_nhwc_dual")
        return y
    if x2 is not None:
        x = torch.cat([x, x2], dim=1)
    if x.device.type == "cpu":
        count("groupnorm", "torch")
    else:
        vendor_fallback("groupnorm", f"dtype {x.dtype}, C={Ct}, groups={groups}")
    if pre_add is not None:
        x = x + pre_add.to(x.dtype)[:, :, None, None]
    y = F.group_norm(x.float(), groups, None if weight is None else weight.to(x.device, torch.float32),
                     None if bias is None else bias.to(x.device, torch.float32), eps)
    if silu:
        y = F.silu(y)
    return y.to(x.dtype)


def layer_norm(x: torch.Tensor, weight: torch.Tensor | None, bias: torch.Tensor | None,
               eps: float = 1e-5) -> torch.Tensor:
    be = backend_for("layernorm", x, "cgs_layernorm")
    C = x.shape[-1]
    if be == "hip" and x.dtype == torch.float32 and _f32.available("cgs_layernorm_f32"):
        y = _f32.layer_norm(x, weight, bias, eps)
        if y is not None:
            count("layernorm", "hip")
            return y
    if be == "hip" and x.dtype in (torch.bfloat16, torch.float16) and C % 8 == 0:
        count("layernorm", "hip")
        xc = x.contiguous()
        y = torch.empty_like(xc)
        rows = xc.numel() // C
        _check(_lib().cgs_layernorm(xc.data_ptr(), y.data_ptr(), _ptr(weight), _ptr(bias),
                                    rows, C, float(eps), _DT[x.dtype], _stream()), "cgs_layernorm")
        return y
    if x.device.type == "cpu":
        count("layernorm", "torch")
    else:
        vendor_fallback("layernorm", f"dtype {x.dtype}, C={C}")
    return F.layer_norm(x.float(), (C,), None if weight is None else weight.float(),
                        None if bias is None else bias.float(), eps).to(x.dtype)


# ----------------------------------------------------------------------------------------------
# Convolution
# ----------------------------------------------------------------------------------------------
def _spatial():
    from ..parallel import spatial
    return spatial.current()


def conv2d(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None, stride=1, padding=0,
           residual: torch.Tensor | None = None, weight_nhwc: torch.Tensor | None = None,
           groups: int = 1, upsample2x: bool = False, x2: torch.Tensor | None = None,
           gn_stats: bool = False) -> torch.Tensor:
    """2-D convolution; inside a row-sharded UNet call (latency mode, parallel/spatial.py) the halo rows
    come from the neighbouring ranks and the residual is added to the kept interior. ``gn_stats``: when the
    shape runs on the v6 kernel, its epilogue also writes GroupNorm statistics partials of the output
    (per image, 64-pixel block and channel), attached as ``y._cgs_gnpart`` -- ``group_norm`` over y then
    skips its statistics pass."""
    sc = _spatial()
    if sc is None:
        return _conv2d(x, weight, bias, stride, padding, residual, weight_nhwc, groups, upsample2x, x2, gn_stats)
    st = stride[0] if isinstance(stride, (tuple, list)) else stride
    pd = padding[0] if isinstance(padding, (tuple, list)) else padding
    y = sc.conv2d(lambda xx, _: _conv2d(xx, weight, bias, st, pd, None, weight_nhwc, groups, upsample2x, None),
                  x, weight.shape[2], st, pd, upsample2x, x2)
    if residual is not None:
        y = y + residual
    return y.contiguous(memory_format=torch.channels_last) if y.is_cuda else y


def _conv2d(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None, stride=1, padding=0,
            residual: torch.Tensor | None = None, weight_nhwc: torch.Tensor | None = None,
            groups: int = 1, upsample2x: bool = False, x2: torch.Tensor | None = None,
            gn_stats: bool = False) -> torch.Tensor:
    """2-D convolution (K09/K10/K12). Device path: implicit-GEMM NHWC kernel on MFMA
    (csrc/kernels/conv.hip) with fused bias + residual epilogue; ``weight_nhwc`` = weight permuted
    to [Cout, kh, kw, Cin]. ``upsample2x`` reads the input through a nearest-2x upsample inside the
    kernel (openaimodel.py Upsample: interpolate + conv) so the 4x tensor is never written.
    ``x2``: convolve ``cat([x, x2], 1)`` with the concat never materialised (K14; the kernel's A-loader
    picks the source per 64-channel K step, so both channel counts must be multiples of 64)."""
    if isinstance(stride, (tuple, list)):
        stride = stride[0]
    if isinstance(padding, (tuple, list)):
        padding = padding[0]
    be = backend_for("conv", x, "cgs_conv2d_nhwc")
    Cout, Cin_g, kh, kw = weight.shape
    cin_total = x.shape[1] + (0 if x2 is None else x2.shape[1])
    if (be == "hip" and groups == 1 and x.dtype == torch.float32 and weight.dtype == torch.float32
            and _f32.available("cgs_conv_f32")):
        y = _f32.conv2d(x, weight, bias, stride, padding, residual, weight_nhwc, upsample2x, x2)
        if y is not None:
            count("conv", "hip")
            return y
    hip_ok = (be == "hip" and groups == 1 and x.dtype == torch.bfloat16 and weight_nhwc is not None
              and x.dim() == 4 and cin_total % 32 == 0 and (Cout % 8 == 0 or Cout <= 16 or cin_total % 64 == 0))
    dual_ok = x2 is None or (hip_ok and x.shape[1] % 64 == 0 and x2.shape[1] % 64 == 0 and x2.dtype == x.dtype
                             and not upsample2x and Cout % 8 == 0)
    if x2 is not None and not dual_ok:
        # every path other than the dual-source HIP loader convolves the materialised concat
        x = torch.cat([x, x2.to(x.dtype)], dim=1)
        x2 = None
    if hip_ok:
        count("conv", "hip")
        N, C1, H, W = x.shape
        Cin = C1 + (0 if x2 is None else x2.shape[1])
        x2c = None if x2 is None else x2.contiguous(memory_format=torch.channels_last)
        Hl, Wl = (2 * H, 2 * W) if upsample2x else (H, W)
        Ho = (Hl + 2 * padding - kh) // stride + 1
        Wo = (Wl + 2 * padding - kw) // stride + 1
        xc = x.contiguous(memory_format=torch.channels_last)
        r = None
        if residual is not None:
            r = residual.contiguous(memory_format=torch.channels_last)
        flags = 16 if upsample2x else 0

        def run(variant):
            out = torch.empty((N, Cout, Ho, Wo), device=x.device, dtype=x.dtype,
                              memory_format=torch.channels_last)
            ws = _v7_ws(N * Ho * Wo, Cout, kh * kw * Cin, x.device) if variant == 7 else None
            if ws is not None:
                _check(_lib().cgs_conv2d_nhwc_v7ws(xc.data_ptr(), _ptr(x2c), C1, weight_nhwc.data_ptr(), _ptr(bias),
                                                   _ptr(r), out.data_ptr(), N, H, W, Cin, Cout, kh, kw, stride,
                                                   padding, Ho, Wo, flags, ws.data_ptr(), ws.numel(), _stream()),
                       "cgs_conv2d_nhwc_v7ws")
                return out
            _check(_lib().cgs_conv2d_nhwc_v(xc.data_ptr(), _ptr(x2c), C1, weight_nhwc.data_ptr(), _ptr(bias), _ptr(r),
                                            out.data_ptr(), N, H, W, Cin, Cout, kh, kw, stride, padding, Ho, Wo,
                                            flags, variant, _stream()), "cgs_conv2d_nhwc")
            return out

        variant = -2            # process-wide override (cgs_conv_set_variant), default auto
        M = N * Ho * Wo
        # Cout <= 16 (UNet / VAE conv_out): the narrow-output kernel, no tuning (csrc conv_launch)
        if M * Cout * Cin * kh * kw >= (1 << 27) and Cout > 16:
            cands = [("v4", lambda: run(4))]
            if Cout % 8 == 0:
                cands.append(("v8", lambda: run(8)))      # 128 x 128 tiles (short grids)
            if Cin % 64 == 0:
                cands += [("v7", lambda: run(7)), ("v5", lambda: run(5)), ("v6", lambda: run(6)),
                          ("v2", lambda: run(2))]
                if Cout % 128 == 0 and Cout % 160 and kh * kw * Cin >= 128:
                    cands.append(("v6n128", lambda: run(18)))   # 256 x 128 tiles (e.g. the VAE's Cout = 128)
                if Cout % 80 == 0 and kh * kw * Cin >= 128 and M <= 32768:
                    cands.append(("v6w4", lambda: run(21)))      # 128 x 80 tiles, 4 waves (batch-1 grids)
            choice = autotune.choose(("conv", N, H, W, Cin, Cout, kh, stride, padding, flags, int(r is not None))
                                     + ((("dual", C1),) if x2c is not None else ()), cands, default="auto")
            variant = {"v2": 2, "v4": 4, "v5": 5, "v6": 6, "v7": 7, "v8": 8, "v6n128": 18, "v6w4": 21,
                       "auto": -2}[choice]
        if (gn_stats and variant == 6 and _GNS and (Ho * Wo) % 256 == 0 and Cin % 64 == 0 and C1 % 64 == 0
                and Cout % 8 == 0 and kh * kw * Cin >= 128 and (bias is None or bias.data_ptr() % 8 == 0)
                and _native.has_kernel("cgs_conv2d_nhwc_gns")):
            out = torch.empty((N, Cout, Ho, Wo), device=x.device, dtype=x.dtype, memory_format=torch.channels_last)
            part = torch.empty(N * (Ho * Wo // 64) * Cout * 2, device=x.device, dtype=torch.float32)
            _check(_lib().cgs_conv2d_nhwc_gns(xc.data_ptr(), _ptr(x2c), C1, weight_nhwc.data_ptr(), _ptr(bias),
                                              _ptr(r), out.data_ptr(), N, H, W, Cin, Cout, kh, kw, stride, padding,
                                              Ho, Wo, flags, part.data_ptr(), _stream()), "cgs_conv2d_nhwc_gns")
            out._cgs_gnpart = (part, out.data_ptr())
            return out
        return run(variant)
    if upsample2x:
        x = upsample_nearest2x(x)
    if be == "torch":
        count("conv", "torch")
        y = F.conv2d(x.float(), weight.float(), None if bias is None else bias.float(), stride, padding,
                     groups=groups)
        if residual is not None:
            y = y + residual.float()
        return y.to(x.dtype)
    vendor_fallback("conv", f"dtype {x.dtype}, groups={groups}, Cin={x.shape[1]}, Cout={Cout}")
    y = F.conv2d(x, weight, bias, stride, padding, groups=groups)
    if residual is not None:
        y = y + residual
    return y


# ConvTranspose2d(k=4, s=2, p=1) as four sub-pixel phases: output pixel (2y + py, 2x + px) sums the
# 2 x 2 input neighbourhood starting at (y - 1 + py, x - 1 + px) through kernel taps _CT_TAPS[py] x
# _CT_TAPS[px] (tap k of the transposed conv reaches output 2i - 1 + k).
_CT_TAPS = ((3, 1), (2, 0))


def conv_transpose_phase_weights(weight: torch.Tensor):
    """[Cin, Cout, 4, 4] ConvTranspose2d weight -> four ([Cout, Cin, 2, 2], NHWC copy) phase convs."""
    out = []
    for py in range(2):
        for px in range(2):
            wp = weight[:, :, list(_CT_TAPS[py])][:, :, :, list(_CT_TAPS[px])].permute(1, 0, 2, 3).contiguous()
            out.append((wp, wp.permute(0, 2, 3, 1).contiguous()))
    return out


def conv_transpose2d(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None, stride=1, padding=0,
                     phase_weights=None) -> torch.Tensor:
    """ConvTranspose2d (Stable Cascade Stage A decoder's 4x4 / stride-2 upsampler, cascade.py).

    Device path for k = 4, s = 2, p = 1: four 2 x 2 convs (one per output sub-pixel phase, pad 1, on
    the NHWC implicit-GEMM conv kernel) written into the interleaved output -- the overlap-add of
    the transposed conv is never formed and no library kernel runs (MIOpen's backward-data conv
    took ~180 ms per call on this shape). ``phase_weights``: cached conv_transpose_phase_weights()."""
    s = stride[0] if isinstance(stride, (tuple, list)) else stride
    p = padding[0] if isinstance(padding, (tuple, list)) else padding
    Cin, Cout, kh, kw = weight.shape
    be = backend_for("conv", x, "cgs_conv2d_nhwc")
    if (be == "hip" and x.dim() == 4 and x.dtype == torch.bfloat16 and weight.dtype == x.dtype and kh == kw == 4
            and s == 2 and p == 1 and Cin % 32 == 0 and (Cout % 8 == 0 or Cout <= 16)):
        N, _, H, W = x.shape
        pw = phase_weights if phase_weights is not None else conv_transpose_phase_weights(weight)
        out = torch.empty((N, Cout, 2 * H, 2 * W), device=x.device, dtype=x.dtype, memory_format=torch.channels_last)
        for i, (wp, wn) in enumerate(pw):
            py, px = divmod(i, 2)
            y = conv2d(x, wp, bias, 1, 1, weight_nhwc=wn)          # [N, Cout, H + 1, W + 1]
            out[:, :, py::2, px::2] = y[:, :, py:py + H, px:px + W]
        return out
    if be == "torch":
        count("conv", "torch")
        y = F.conv_transpose2d(x.float(), weight.float(), None if bias is None else bias.float(), s, p)
        return y.to(x.dtype)
    vendor_fallback("conv", f"conv_transpose2d k={kh}x{kw} s={s} p={p} dtype {x.dtype}")
    return F.conv_transpose2d(x, weight, bias, s, p)


def upsample_nearest2x(x: torch.Tensor) -> torch.Tensor:
    be = backend_for("upsample", x, "cgs_upsample_nearest2x_nhwc")
    if be == "hip" and x.dim() == 4 and x.dtype in (torch.bfloat16, torch.float16):
        count("upsample", "hip")
        N, C, H, W = x.shape
        xc = x.contiguous(memory_format=torch.channels_last)
        y = torch.empty((N, C, 2 * H, 2 * W), device=x.device, dtype=x.dtype,
                        memory_format=torch.channels_last)
        _check(_lib().cgs_upsample_nearest2x_nhwc(xc.data_ptr(), y.data_ptr(), N, H, W, C,
                                                  _DT[x.dtype], _stream()), "cgs_upsample")
        return y
    count("upsample", "torch" if x.device.type == "cpu" else "lib")
    return F.interpolate(x, scale_factor=2.0, mode="nearest")


def depthwise_conv2d_nhwc(x: torch.Tensor, w_kkc: torch.Tensor, bias: torch.Tensor | None, k: int,
                          replicate: bool = False) -> torch.Tensor:
    """Depthwise kxk conv, stride 1, 'same' padding (zeros, or border replicate) on an NHWC tensor
    [N, H, W, C] (K11: Stable Cascade ResBlocks). ``w_kkc`` = weight [C,1,k,k] laid out [k*k, C]."""
    N, H, W, C = x.shape
    be = backend_for("dwconv", x, "cgs_dwconv_nhwc")
    if be == "hip" and x.dtype in (torch.bfloat16, torch.float16) and C % 8 == 0 and k % 2 == 1:
        count("dwconv", "hip")
        xc = x.contiguous()
        y = torch.empty_like(xc)
        _check(_lib().cgs_dwconv_nhwc(xc.data_ptr(), w_kkc.contiguous().data_ptr(), _ptr(bias), y.data_ptr(),
                                      N, H, W, C, k, int(replicate), _DT[x.dtype], _stream()), "cgs_dwconv")
        return y
    count("dwconv", "torch" if x.device.type == "cpu" else "lib")
    xn = x.permute(0, 3, 1, 2)
    wt = w_kkc.t().reshape(C, 1, k, k).to(x.dtype)
    if replicate:
        xn = F.pad(xn.float(), (k // 2,) * 4, mode="replicate").to(x.dtype)
        y = F.conv2d(xn, wt, bias, 1, 0, 1, C)
    else:
        y = F.conv2d(xn, wt, bias, 1, k // 2, 1, C)
    return y.permute(0, 2, 3, 1).contiguous()


def depthwise_conv2d_nhwc_lnstats(x: torch.Tensor, w_kkc: torch.Tensor, bias: torch.Tensor | None, k: int,
                                  eps: float, replicate: bool = False):
    """``(y, rs)``: the depthwise conv of ``depthwise_conv2d_nhwc`` plus the per-pixel LayerNorm statistics
    of y over C (float32 [pixels, 2] (mean, rstd), the ``layernorm_stats`` layout) from the same pass --
    the Cascade ResBlock's depthwise -> LayerNorm2d feeding a LayerNorm-folded GEMM (no second read of y)."""
    N, H, W, C = x.shape
    be = backend_for("dwconv", x, "cgs_dwconv_ln_stats_nhwc")
    if be == "hip" and x.dtype in (torch.bfloat16, torch.float16) and C % 8 == 0 and C <= 2048 and k % 2 == 1:
        count("dwconv", "hip")
        xc = x.contiguous()
        y = torch.empty_like(xc)
        rs = torch.empty((N * H * W, 2), device=x.device, dtype=torch.float32)
        _check(_lib().cgs_dwconv_ln_stats_nhwc(xc.data_ptr(), w_kkc.contiguous().data_ptr(), _ptr(bias), y.data_ptr(),
                                               rs.data_ptr(), N, H, W, C, k, int(replicate), float(eps),
                                               _DT[x.dtype], _stream()), "cgs_dwconv_ln_stats_nhwc")
        return y, rs
    y = depthwise_conv2d_nhwc(x, w_kkc, bias, k, replicate)
    yf = y.float().reshape(-1, C)
    mean = yf.mean(dim=1)
    rstd = torch.rsqrt(yf.var(dim=1, unbiased=False) + eps)
    return y, torch.stack([mean, rstd], dim=1)


# ----------------------------------------------------------------------------------------------
# Elementwise
# ----------------------------------------------------------------------------------------------
def silu(x: torch.Tensor) -> torch.Tensor:
    be = backend_for("silu", x, "cgs_silu")
    if be == "hip" and x.dtype in (torch.bfloat16, torch.float16) and x.is_contiguous():
        count("silu", "hip")
        y = torch.empty_like(x)
        _check(_lib().cgs_silu(x.data_ptr(), y.data_ptr(), x.numel(), _DT[x.dtype], _stream()), "cgs_silu")
        return y
    return F.silu(x.float()).to(x.dtype) if x.device.type == "cpu" else F.silu(x)


def gelu(x: torch.Tensor, approximate: str = "none") -> torch.Tensor:
    return F.gelu(x, approximate=approximate)


def timestep_embedding(t: torch.Tensor, dim: int, max_period: float = 10000.0,
                       flip_sin_to_cos: bool = True) -> torch.Tensor:
    """Sinusoidal timestep embedding: [cos | sin] (util.py:229-249 semantics), fp32 out."""
    be = backend_for("timestep_embedding", t, "cgs_timestep_embedding")
    if be == "hip" and dim % 2 == 0:
        count("timestep_embedding", "hip")
        tt = t.float().contiguous()
        out = torch.empty((t.shape[0], dim), device=t.device, dtype=torch.float32)
        _check(_lib().cgs_timestep_embedding(tt.data_ptr(), out.data_ptr(), t.shape[0], dim,
                                             float(max_period), 1 if flip_sin_to_cos else 0, _stream()),
               "cgs_timestep_embedding")
        return out
    half = dim // 2
    freqs = torch.exp(-math.log(max_period) * torch.arange(half, dtype=torch.float32, device=t.device) / half)
    args = t[:, None].float() * freqs[None]
    emb = torch.cat([torch.cos(args), torch.sin(args)], dim=-1) if flip_sin_to_cos else \
        torch.cat([torch.sin(args), torch.cos(args)], dim=-1)
    if dim % 2:
        emb = torch.cat([emb, torch.zeros_like(emb[:, :1])], dim=-1)
    return emb


def cfg_combine(cond: torch.Tensor, uncond: torch.Tensor, scale: float) -> torch.Tensor:
    """uncond + (cond - uncond) * scale (samplers.py:240), fused on device."""
    be = backend_for("cfg", cond, "cgs_cfg_combine")
    if be == "hip" and cond.dtype == torch.float32 and cond.is_contiguous() and uncond.is_contiguous():
        out = torch.empty_like(cond)
        _check(_lib().cgs_cfg_combine(cond.data_ptr(), uncond.data_ptr(), out.data_ptr(), cond.numel(),
                                      float(scale), 0, _stream()), "cgs_cfg_combine")
        return out
    return uncond + (cond - uncond) * scale


def euler_step(x: torch.Tensor, denoised: torch.Tensor, noise: torch.Tensor | None, sigma: float,
               sigma_down: float, sigma_up: float) -> torch.Tensor:
    """Fused Euler(-ancestral) update (sampling.py:148-164):
    d = (x - denoised)/sigma ; x = x + d*(sigma_down - sigma) ; x += noise*sigma_up."""
    be = backend_for("euler", x, "cgs_euler_step")
    if be == "hip" and x.dtype == torch.float32 and denoised.dtype == torch.float32 and x.is_contiguous() \
            and denoised.is_contiguous() and (noise is None or noise.is_contiguous()):
        count("euler", "hip")
        x = x.clone()  # the kernel updates in place; keep the caller's tensor intact
        _check(_lib().cgs_euler_step(x.data_ptr(), denoised.data_ptr(),
                                     _ptr(noise) if (noise is not None and sigma_up > 0) else None,
                                     x.numel(), float(sigma), float(sigma_down), float(sigma_up), _stream()),
               "cgs_euler_step")
        return x
    d = (x - denoised) / sigma
    x = x + d * (sigma_down - sigma)
    if noise is not None and sigma_up > 0:
        x = x + noise * sigma_up
    return x


# ----------------------------------------------------------------------------------------------
# Counter-based noise (csrc/kernels/rng.hip; CPU mirror sampling/rng.py)
# ----------------------------------------------------------------------------------------------
def _numel1(shape):
    n = 1
    for d in shape[1:]:
        n *= int(d)
    return n


# Device-resident RNG key (sampling/run_graph.py): while a sampler run is being captured into hipGraphs,
# draws keyed by the run's (seed, index0) read both from this int64 device tensor instead of kernel
# arguments, so replaying the graphs for another job only rewrites the tensor.
import contextvars as _cv
_RNG_KEY: _cv.ContextVar = _cv.ContextVar("cgs_rng_key", default=None)


def rng_key_scope(key: torch.Tensor, seed: int, index0: int):
    """Context manager: draws with (seed, index0) take them from ``key`` = [seed, index0] (device)."""
    class _Scope:
        def __enter__(self_):
            self_.tok = _RNG_KEY.set((key, int(seed) & ((1 << 64) - 1), int(index0)))

        def __exit__(self_, *a):
            _RNG_KEY.reset(self_.tok)
    return _Scope()


def _dev_key(seed, index0):
    k = _RNG_KEY.get()
    if k is not None and k[1] == (int(seed) & ((1 << 64) - 1)) and k[2] == index0:
        return k[0].data_ptr()
    return None


def philox_randn(shape, seed: int, inds, stream: int, device=None, dtype=torch.float32,
                 dev_step: torch.Tensor | None = None) -> torch.Tensor:
    """N(0,1) noise [B, ...] where image b's values depend only on (seed, inds[b], stream).

    ``dev_step`` (device int64 scalar) is added to ``stream`` inside the kernel, so a captured graph
    can advance the stream per replay without re-recording."""
    from ..sampling import rng
    device = torch.device("cpu") if device is None else torch.device(device)
    probe = torch.empty(0, device=device)
    be = backend_for("rng", probe, "cgs_philox_randn")
    index0, contiguous = rng.contiguous_inds(inds)
    if be == "hip" and dtype in (torch.float32, torch.bfloat16) and contiguous:
        count("rng", "hip")
        out = torch.empty(tuple(shape), device=device, dtype=dtype)
        _check(_lib().cgs_philox_randn(out.data_ptr(), int(shape[0]), _numel1(shape), int(seed) & ((1 << 64) - 1),
                                       index0, int(stream), _ptr(dev_step), 1.0, _DT[dtype], _dev_key(seed, index0),
                                       _stream()),
               "cgs_philox_randn")
        return out
    if be == "hip" and dtype in (torch.float32, torch.bfloat16):   # scattered indices: one launch per image
        return torch.cat([philox_randn((1,) + tuple(shape[1:]), seed, [i], stream, device, dtype, dev_step)
                          for i in inds])
    count("rng", "torch")
    if dev_step is not None:
        stream = int(stream) + int(dev_step.item())
    return rng.randn_reference(tuple(shape), seed, inds, stream).to(device=device, dtype=dtype)


def euler_ancestral_philox(x: torch.Tensor, denoised: torch.Tensor, sigma: float, sigma_down: float,
                           sigma_up: float, seed: int, inds, stream: int) -> torch.Tensor:
    """Euler-ancestral update with the step's noise generated in registers (K16+K18): equals
    ``euler_step(x, denoised, philox_randn(x.shape, seed, inds, stream), ...)`` without the noise tensor."""
    from ..sampling import rng
    be = backend_for("euler", x, "cgs_euler_ancestral_philox")
    index0, contiguous = rng.contiguous_inds(inds)
    if be == "hip" and contiguous and x.dtype == torch.float32 and denoised.dtype == torch.float32 \
            and x.is_contiguous() and denoised.is_contiguous() and _numel1(x.shape) % 4 == 0:
        count("euler", "hip")
        x = x.clone()
        _check(_lib().cgs_euler_ancestral_philox(x.data_ptr(), denoised.data_ptr(), int(x.shape[0]), _numel1(x.shape),
                                                 float(sigma), float(sigma_down), float(sigma_up),
                                                 int(seed) & ((1 << 64) - 1), index0, int(stream),
                                                 _dev_key(seed, index0), _stream()),
               "cgs_euler_ancestral_philox")
        return x
    noise = philox_randn(x.shape, seed, inds, stream, device=x.device, dtype=x.dtype) if sigma_up > 0 else None
    return euler_step(x, denoised, noise, sigma, sigma_down, sigma_up)


def brownian_increment(shape, seed: int, inds, t0: float, t1: float, ta: float, tb: float, tol: float,
                       max_depth: int, scale: float, device=None) -> torch.Tensor:
    """(W(tb) - W(ta)) * scale of the per-image virtual Brownian tree on [t0, t1] (fp32)."""
    from ..sampling import rng
    device = torch.device("cpu") if device is None else torch.device(device)
    be = backend_for("rng", torch.empty(0, device=device), "cgs_brownian_increment")
    index0, contiguous = rng.contiguous_inds(inds)
    if be == "hip" and _numel1(shape) % 4 == 0:
        if not contiguous:
            return torch.cat([brownian_increment((1,) + tuple(shape[1:]), seed, [i], t0, t1, ta, tb, tol, max_depth,
                                                 scale, device) for i in inds])
        count("rng", "hip")
        out = torch.empty(tuple(shape), device=device, dtype=torch.float32)
        _check(_lib().cgs_brownian_increment(out.data_ptr(), int(shape[0]), _numel1(shape),
                                             int(seed) & ((1 << 64) - 1), index0, float(t0), float(t1), float(ta),
                                             float(tb), float(tol), int(max_depth), float(scale),
                                             _dev_key(seed, index0), _stream()),
               "cgs_brownian_increment")
        return out
    count("rng", "torch")
    return rng.brownian_reference(tuple(shape), seed, inds, t0, t1, ta, tb, tol, max_depth, scale).to(device)


# ----------------------------------------------------------------------------------------------
# Image / utility ops (csrc/kernels/image.hip)
# ----------------------------------------------------------------------------------------------
_RESIZE_MODES = {"nearest": 0, "nearest-exact": 1, "bilinear": 2, "bicubic": 3, "area": 4}


def interpolate(x: torch.Tensor, size, mode: str = "nearest", align_corners: bool | None = None) -> torch.Tensor:
    """``F.interpolate(x, size=size, mode=mode)`` for 4-D tensors (K25). Device path: one HIP
    kernel over the NC planes (fp32 accumulate); other modes / ranks go to ATen."""
    Ho, Wo = (size, size) if isinstance(size, int) else (int(size[0]), int(size[1]))
    m = _RESIZE_MODES.get(mode)
    be = backend_for("resize", x, "cgs_resize")
    if be == "hip" and m is not None and x.dim() == 4 and x.dtype in _DT and x.numel() > 0:
        count("resize", "hip")
        N, C, H, W = x.shape
        xc = x.contiguous()
        y = torch.empty((N, C, Ho, Wo), device=x.device, dtype=x.dtype)
        _check(_lib().cgs_resize(xc.data_ptr(), y.data_ptr(), N * C, H, W, Ho, Wo, m, int(bool(align_corners)),
                                 _DT[x.dtype], _stream()), "cgs_resize")
        return y
    kw = {"align_corners": align_corners} if mode in ("bilinear", "bicubic") else {}
    return F.interpolate(x, size=(Ho, Wo), mode=mode, **kw)


def clip_embed(ids: torch.Tensor, tok_weight: torch.Tensor, pos_weight: torch.Tensor) -> torch.Tensor:
    """``tok_weight[ids] + pos_weight[:S]`` (K26: CLIP token + position embedding, one kernel)."""
    B, S = ids.shape
    be = backend_for("clip_embed", tok_weight, "cgs_clip_embed")
    if (be == "hip" and tok_weight.dtype in _DT and pos_weight.dtype == tok_weight.dtype and ids.device == tok_weight.device
            and pos_weight.shape[0] >= S):
        count("clip_embed", "hip")
        D = tok_weight.shape[1]
        idc = ids.to(torch.long).contiguous()
        tw, pw = tok_weight.contiguous(), pos_weight.contiguous()
        y = torch.empty((B, S, D), device=tw.device, dtype=tw.dtype)
        _check(_lib().cgs_clip_embed(idc.data_ptr(), tw.data_ptr(), pw.data_ptr(), y.data_ptr(), B, S, D,
                                     tw.shape[0], _DT[tw.dtype], _stream()), "cgs_clip_embed")
        return y
    count("clip_embed", "torch")
    return F.embedding(ids.to(torch.long), tok_weight) + pos_weight[:S].to(tok_weight.dtype)


def pooled_gather(x: torch.Tensor, ids: torch.Tensor) -> torch.Tensor:
    """``x[b, argmax(ids[b])]`` (K26: CLIP pooled output at the end-of-text token)."""
    B, S, D = x.shape
    be = backend_for("clip_embed", x, "cgs_pooled_gather")
    if be == "hip" and x.dtype in _DT and ids.device == x.device:
        count("clip_embed", "hip")
        xc = x.contiguous()
        idc = ids.to(torch.long).contiguous()
        out = torch.empty((B, D), device=x.device, dtype=x.dtype)
        _check(_lib().cgs_pooled_gather(idc.data_ptr(), xc.data_ptr(), out.data_ptr(), B, S, D, _DT[x.dtype],
                                        _stream()), "cgs_pooled_gather")
        return out
    return x[torch.arange(B, device=x.device), ids.to(device=x.device, dtype=torch.long).argmax(dim=-1)]


_LNFOLD = os.environ.get("CGS_LNFOLD", "1") != "0"


def lnfold_available(x: torch.Tensor, K: int) -> bool:
    """The LayerNorm-folded GEMM path applies (device bf16 rows, v7-legal K)."""
    return (_LNFOLD and os.environ.get("CGS_LNFOLD", "1") != "0" and x.is_cuda and x.dtype == torch.bfloat16 and K % 64 == 0 and K >= 128 and K <= 2048
            and backend_for("layernorm", x, "cgs_layernorm_stats") == "hip" and _native.has_kernel("cgs_gemm_bf16_lnfold"))


_RSO = os.environ.get("CGS_LN_ROWSTATS", "1") != "0"
_GNS = os.environ.get("CGS_GN_CONVSTATS", "1") != "0"


def layernorm_stats_for(x: torch.Tensor, eps: float) -> torch.Tensor:
    """``layernorm_stats`` of x, from the partials its producing GEMM wrote (``linear(row_stats=True)``)
    when they are attached to this tensor; else the statistics pass over x."""
    h = getattr(x, "_cgs_rowpart", None)
    if h is not None and h[1] == x.data_ptr() and h[0].shape[0] * 80 * h[0].shape[1] == x.numel() \
            and _native.has_kernel("cgs_ln_rs_from_partials"):
        part = h[0]
        M, P = part.shape[0], part.shape[1]
        rs = torch.empty((M, 2), device=x.device, dtype=torch.float32)
        count("layernorm", "hip")
        _check(_lib().cgs_ln_rs_from_partials(part.data_ptr(), rs.data_ptr(), M, P, float(eps), _stream()),
               "cgs_ln_rs_from_partials")
        return rs
    return layernorm_stats(x, eps)


def layernorm_stats(x: torch.Tensor, eps: float) -> torch.Tensor:
    """Per-row (mean, rstd) of ``x`` [..., C] as float32 [rows, 2] (the statistics half of LayerNorm)."""
    C = x.shape[-1]
    a = x.reshape(-1, C)
    if not a.is_contiguous():
        a = a.contiguous()
    rs = torch.empty((a.shape[0], 2), device=x.device, dtype=torch.float32)
    count("layernorm", "hip")
    _check(_lib().cgs_layernorm_stats(a.data_ptr(), rs.data_ptr(), a.shape[0], C, float(eps), _DT[x.dtype],
                                      _stream()), "cgs_layernorm_stats")
    return rs


def lnfold_weights(weight: torch.Tensor, bias: torch.Tensor | None, gamma: torch.Tensor | None,
                   beta: torch.Tensor | None):
    """(W', colsum(W'), b') with W' = W * gamma (bf16), colsum over the bf16-rounded W' (fp32) and
    b' = b + W beta, so that LN(x) W^T + b = rstd * (x W'^T - mean * colsum(W')) + b'."""
    wf = weight.float()
    w2 = (wf * gamma.float()[None, :]) if gamma is not None else wf
    w2 = w2.to(torch.bfloat16).contiguous()
    cs = w2.float().sum(dim=1).contiguous()
    b = torch.zeros(weight.shape[0], device=weight.device, dtype=torch.float32)
    if bias is not None:
        b = b + bias.float()
    if beta is not None:
        b = b + wf @ beta.float()
    return w2, cs, b.to(torch.bfloat16).contiguous()


_GRN_GNS = os.environ.get("CGS_GRN_GNS", "1") != "0"


def _gelu_gns_ok(M, N, K, hw) -> bool:
    return (_GRN_GNS and os.environ.get("CGS_GRN_GNS", "1") != "0" and hw is not None and hw > 0 and hw % 64 == 0 and M % hw == 0 and M // hw <= 64
            and N % 8 == 0 and K % 64 == 0 and K >= 128 and _native.has_kernel("cgs_gemm_bf16_gelu_gns"))


def _gelu_gns(a, w, b, rs, cs, M, N, K, epi, hw, device, dtype):
    """The v6 GELU (+ LN-fold) GEMM whose epilogue also writes per-(image, 64-row block, column) sums of squares
    partials of its output (returned with it; the caller attaches them to its final view as
    ``y._cgs_grnpart``): the GlobalResponseNorm over y (``grn_nhwc`` / ``grn_fold_weight``) then takes its
    statistics from them instead of a pass over y."""
    out = torch.empty((M, N), device=device, dtype=dtype)
    part = torch.empty((M // 64) * N, device=device, dtype=torch.float32)
    _check(_lib().cgs_gemm_bf16_gelu_gns(a.data_ptr(), w.data_ptr(), out.data_ptr(), b.data_ptr(), _ptr(rs), _ptr(cs),
                                         M, N, K, a.stride(0), K, N, epi, part.data_ptr(), hw, _stream()),
           "cgs_gemm_bf16_gelu_gns")
    return out, part


def linear_lnfold(x: torch.Tensor, rs: torch.Tensor, w2: torch.Tensor, cs: torch.Tensor, b2: torch.Tensor,
                  geglu: bool = False, act: str | None = None, gns_hw: int | None = None) -> torch.Tensor:
    """``LN(x) @ W^T + b`` (or the GEGLU of it, with interleaved W' rows) from the raw rows ``x``, the
    row statistics ``rs`` and ``lnfold_weights`` -- the LayerNorm never materialises (K07 folded
    into the GEMM epilogue of the v7 kernel). ``act="gelu"``: GELU of it (Cascade's LayerNorm ->
    ChannelMLP Linear -> GELU), on the v6 ACT / mc::tile kernels. ``gns_hw`` (rows per image): when the
    v6 kernel runs, its epilogue also leaves the GRN statistics partials of the output (``_gelu_gns``)."""
    K = x.shape[-1]
    a = x.reshape(-1, K)
    if not a.is_contiguous():
        a = a.contiguous()
    M, N = a.shape[0], w2.shape[0]
    nout = N // 2 if geglu else N
    epi = EPI_BIAS | (EPI_GEGLU if geglu else 0)
    count("gemm_geglu" if geglu else "gemm", "hip")
    if act == "gelu":
        assert not geglu
        epi |= EPI_GELU

        def run_g(variant):
            out = torch.empty((M, N), device=x.device, dtype=x.dtype)
            _check(_lib().cgs_gemm_bf16_lnfold_v(a.data_ptr(), w2.data_ptr(), out.data_ptr(), b2.data_ptr(),
                                                 rs.data_ptr(), cs.data_ptr(), M, N, K, K, K, N, epi, None, 0,
                                                 variant, _stream()), "cgs_gemm_bf16_lnfold_v")
            return out
        cands = [("v8", lambda: run_g(8)), ("v6", lambda: run_g(6))]
        if _underfilled(M, N):
            cands += [(f"v{v}", (lambda v=v: run_g(v))) for v in _SMALL_TILE]
        choice = autotune.choose(("gemm_lnfold", M, N, K, epi), cands, default="v6" if N % 160 == 0 else "v8")
        if choice == "v6" and _gelu_gns_ok(M, N, K, gns_hw):
            y, part = _gelu_gns(a, w2, b2, rs, cs, M, N, K, epi | EPI_LNFOLD, gns_hw, x.device, x.dtype)
            y = y.view(*x.shape[:-1], N)
            y._cgs_grnpart = (part, y.data_ptr(), gns_hw)
            return y
        return run_g({"v6": 6, "v8": 8, **_SMALL_NAMES}.get(choice, -1)).view(*x.shape[:-1], N)

    def run(variant):
        out = torch.empty((M, nout), device=x.device, dtype=x.dtype)
        if isinstance(variant, str):                           # split-K (batch-1 grids)
            return _splitk_run(a, w2, out, b2, None, rs, cs, M, N, K, epi | EPI_LNFOLD, variant)
        ws = _v7_ws(M, N, K, x.device) if variant in (-1, 7) else None
        _check(_lib().cgs_gemm_bf16_lnfold_v(a.data_ptr(), w2.data_ptr(), out.data_ptr(), b2.data_ptr(), rs.data_ptr(),
                                             cs.data_ptr(), M, N, K, K, K, nout, epi, _ptr(ws),
                                             0 if ws is None else ws.numel(), variant, _stream()),
               "cgs_gemm_bf16_lnfold_v")
        return out

    variant = -1                  # v6 / v7 by shape
    w6 = _w6_cands(M, N, K, epi | EPI_LNFOLD, run)
    if _underfilled(M, N) and _native.has_kernel("cgs_gemm_bf16_lnfold_v"):
        cands = [("v7", lambda: run(-1)), ("v8", lambda: run(8))] + [(f"v{v}", (lambda v=v: run(v))) for v in _SMALL_TILE]
        if N % 160 == 0:    # 256x160 tiles (plain or GEGLU): whole rounds where 256x256 leaves a partial one
            cands.append(("v6", lambda: run(6)))
            if not geglu:   # 128 x 160 tiles, and 128 x 80 with one wave group
                cands += [("v6m128", lambda: run(V6_M128)), ("v6w4", lambda: run(V6_W4))]
        if not geglu:
            cands += _splitk_cands(M, N, K, epi | EPI_LNFOLD, run)
        choice = autotune.choose(("gemm_lnfold", M, N, K, epi), cands + w6, default="v7")
        variant = choice if choice in _SPLITK else {"v8": 8, "v6": 6, "w6": W6, "w6n160": W6_160,
                                                    "v6m128": V6_M128, "v6w4": V6_W4,
                                                    **_SMALL_NAMES}.get(choice, -1)
    elif geglu and N % 160 == 0 and _native.has_kernel("cgs_gemm_bf16_lnfold_v"):
        choice = autotune.choose(("gemm_lnfold", M, N, K, epi),
                                 [("v7", lambda: run(7)), ("v6", lambda: run(6))] + w6, default="v7")
        variant = {"v6": 6, "w6": W6, "w6n160": W6_160}.get(choice, 7)
    elif not geglu and N % 160 == 0 and N > 1280 and _native.has_kernel("cgs_gemm_bf16_lnfold_v"):
        # wide non-GEGLU projections (fused QKV): 256x160 tiles give whole rounds where 256x256 leave
        # a partial last round (N = 1920 / 3840 at M = 65536 / 16384) -- measured per shape
        choice = autotune.choose(("gemm_lnfold", M, N, K, epi),
                                 [("v7", lambda: run(7)), ("v6", lambda: run(6))] + w6, default="v7")
        variant = {"v6": 6, "w6": W6, "w6n160": W6_160}.get(choice, 7)
    elif w6 and _native.has_kernel("cgs_gemm_bf16_lnfold_v"):
        choice = autotune.choose(("gemm_lnfold", M, N, K, epi), [("v7", lambda: run(-1))] + w6, default="v7")
        variant = {"w6": W6, "w6n160": W6_160}.get(choice, -1)
    return run(variant).view(*x.shape[:-1], nout)


W6, W6_160 = 16, 17      # gemm_w6.hip (256 / 160-wide tiles) through cgs_gemm_bf16_v / _lnfold_v
V6_M128 = 19             # v6 with 128 x 160 tiles (pq::run NI = 2): the short-M grids
V6_W4 = 20               # v6 with 128 x 80 tiles, 4 waves, two workgroups per CU (pq::run NW = 4): batch-1 grids


def _w6_ok(M, N, K, epi, bn=256) -> bool:
    """The w6 kernel's shape / epilogue domain (``cgs_gemm_w6_ok``; contiguous operands: lda = ldw = K)."""
    if M * N * K < (1 << 30) or not _native.has_kernel("cgs_gemm_w6_ok"):
        return False
    nout = N // 2 if epi & EPI_GEGLU else N
    return bool(_lib().cgs_gemm_w6_ok(M, N, K, K, K, nout, nout if epi & EPI_RESIDUAL else 0, epi, bn))


def _w6_cands(M, N, K, epi, run):
    """("w6", ...) / ("w6n160", ...) autotune candidates where the shape is in their domain."""
    out = []
    if _w6_ok(M, N, K, epi):
        out.append(("w6", lambda: run(W6)))
    if N % 160 == 0 and _w6_ok(M, N, K, epi, 160):
        out.append(("w6n160", lambda: run(W6_160)))
    return out


_CUS: list = []
# small-tile GEMM variants (gemm.hip gemm_v8_launch): 10 / 11 = 64x128 / 128x64 with a 4-stage ring,
# 12 / 13 = the same with 6 stages, 14 = 128x128 with 5 stages
_SMALL_TILE = (10, 11, 12, 13, 14)
_SMALL_NAMES = {f"v{v}": v for v in _SMALL_TILE}
# split-K forms of the v8 family (cgs_gemm_bf16_splitk): autotune name -> (tile variant, slices)
_SPLITK = {"sk2v8": (8, 2), "sk4v8": (8, 4), "sk2v10": (10, 2), "sk4v10": (10, 4), "sk2v11": (11, 2),
           "sk4v11": (11, 4), "sk8v8": (8, 8)}


def _splitk_cands(M, N, K, epi, run):
    """Split-K autotune candidates for an under-filled grid (batch-1 shapes: a 128 x 128 grid under two
    workgroups per CU): the K slices multiply the workgroup count, one reduce pass applies the epilogue.
    Candidates by default from K = 4096 (CGS_SPLITK=1: every K, 0: never): slower than the best single-pass
    tile on every SDXL batch-1 shape (profiles/r05/splitk.md -- the fp32 partial round trip costs more than
    the fuller grid gains at K <= 5120), -3.3 % per Cascade batch-1 job on Stage C's K = 8192 ChannelMLP
    projection (profiles/r05/splitk_cascade.md)."""
    mode = os.environ.get("CGS_SPLITK", "auto")
    if (epi & ~(EPI_BIAS | EPI_RESIDUAL | EPI_LNFOLD | EPI_GELU)) or N % 8 or not _underfilled(M, N) \
            or not _native.has_kernel("cgs_gemm_bf16_splitk") or mode == "0" or (mode != "1" and K < 4096):
        return []
    return [(name, (lambda name=name: run(name))) for name, (_, s) in _SPLITK.items()
            if K % (32 * s) == 0 and K // s >= 256]


def _splitk_run(a, w, o, bias, r, rs, cs, M, N, K, epi, name):
    variant, s = _SPLITK[name]
    ws = torch.empty(s * M * N, device=a.device, dtype=torch.float32)
    _check(_lib().cgs_gemm_bf16_splitk(a.data_ptr(), w.data_ptr(), o.data_ptr(), _ptr(bias), _ptr(r), _ptr(rs),
                                       _ptr(cs), M, N, K, a.stride(0), w.stride(0), N, N if r is not None else 0,
                                       epi, 1.0, s, variant, ws.data_ptr(), ws.numel() * 4, _stream()),
           "cgs_gemm_bf16_splitk")
    return o


def _num_cus() -> int:
    if not _CUS:
        try:
            _CUS.append(int(torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count))
        except Exception:
            _CUS.append(256)
    return _CUS[0]


def _underfilled(M: int, N: int) -> bool:
    """A 128 x 128 grid of this output is under two workgroups per CU: the small-tile kernels (v10 /
    v11) join the autotune candidates (batch-1 and Stable Cascade Stage C token counts)."""
    return ((M + 127) // 128) * ((N + 127) // 128) < 2 * _num_cus()


def _feather_mask(h: int, w: int, feather: int, device) -> torch.Tensor:
    """Separable ramp of the reference tiled blend (comfy/utils.py tiled_scale)."""
    def ramp(n):
        t = torch.arange(n, device=device, dtype=torch.float32)
        a = torch.ones(n, device=device)
        a = torch.where(t < feather, a * (t + 1) / feather, a)
        a = torch.where(n - 1 - t < feather, a * (n - t) / feather, a)
        return a
    return ramp(h)[:, None] * ramp(w)[None, :]


def region_accumulate(out: torch.Tensor, div: torch.Tensor | None, piece: torch.Tensor, oy: int, ox: int,
                      mult: torch.Tensor | None = None, feather: int = 0, scale: float = 1.0):
    """In place: ``out[:, :, oy:oy+h, ox:ox+w] += piece * wt`` and ``div[...] += wt`` with
    ``wt = scale * mult (broadcast over channels when it has one) * feather ramp`` -- the area /
    mask cond accumulation of ``calc_cond_batch`` (K17, reference comfy/samplers.py:205-228) and the
    feathered tile blend of ``tiled_scale`` (K24). ``out`` / ``div``: fp32 [B, C, Ho, Wo] contiguous.
    Device path: one HIP kernel (any piece / mult strides and float dtype), no temporaries."""
    B, C, h, w = piece.shape
    be = backend_for("region_acc", out, "cgs_region_accumulate")
    if (be == "hip" and out.dtype == torch.float32 and out.is_contiguous() and piece.dtype in _DT
            and (div is None or (div.shape == out.shape and div.dtype == torch.float32 and div.is_contiguous()))
            and (mult is None or (mult.dim() == 4 and mult.dtype in _DT and mult.shape[1] in (1, C)))):
        count("region_acc", "hip")
        Ho, Wo = out.shape[2], out.shape[3]
        if mult is not None:
            mult = mult.expand(B, mult.shape[1], h, w)
            ms = mult.stride()
        else:
            ms = (0, 0, 0, 0)
        ps = piece.stride()
        _check(_lib().cgs_region_accumulate(out.data_ptr(), _ptr(div), piece.data_ptr(), _DT[piece.dtype],
                                            _ptr(mult), _DT[mult.dtype] if mult is not None else 0, B, C, Ho, Wo,
                                            h, w, int(oy), int(ox), ps[0], ps[1], ps[2], ps[3],
                                            1 if mult is None else mult.shape[1], ms[0], ms[1], ms[2], ms[3],
                                            int(feather), float(scale), _stream()), "cgs_region_accumulate")
        return
    count("region_acc", "torch")
    wt = torch.full((1, 1, h, w), float(scale), device=out.device, dtype=torch.float32)
    if feather > 0:
        wt = wt * _feather_mask(h, w, feather, out.device)
    if mult is not None:
        wt = wt * mult.float()
    hh, ww = min(h, out.shape[2] - oy), min(w, out.shape[3] - ox)
    wt = wt.expand(B, -1, h, w)[:, :, :hh, :ww]
    out[:, :, oy:oy + hh, ox:ox + ww] += piece[:, :, :hh, :ww].float() * wt
    if div is not None:
        div[:, :, oy:oy + hh, ox:ox + ww] += wt.expand(B, C, hh, ww) if wt.shape[1] == 1 else wt


def region_normalize(out: torch.Tensor, div: torch.Tensor, dtype=None) -> torch.Tensor:
    """``(out / div).to(dtype)`` (the final step of both accumulations) in one kernel."""
    dtype = dtype or out.dtype
    be = backend_for("region_acc", out, "cgs_region_normalize")
    if be == "hip" and out.is_contiguous() and div.is_contiguous() and dtype in _DT and div.dtype == torch.float32:
        count("region_acc", "hip")
        y = torch.empty(out.shape, device=out.device, dtype=dtype)
        _check(_lib().cgs_region_normalize(out.data_ptr(), div.data_ptr(), y.data_ptr(), out.numel(), _DT[dtype],
                                           _stream()), "cgs_region_normalize")
        return y
    return (out / div).to(dtype)


def channel_affine_nhwc(x: torch.Tensor, scale: torch.Tensor, shift: torch.Tensor, add: float = 0.0) -> torch.Tensor:
    """y = x * (add + scale[n, c]) + shift[n, c] for NHWC ``x`` [N, H, W, C] and [N, C] coefficient
    views in x's dtype (row stride free: e.g. the two halves of one [N, 2C] GEMM output). Stable
    Cascade TimestepBlock ``x * (1 + a) + b`` (``comfy/ldm/cascade/common.py``) with ``add = 1``."""
    be = backend_for("channel_affine", x, "cgs_channel_affine2")
    N, C = x.shape[0], x.shape[-1]
    if (be == "hip" and x.dtype in (torch.bfloat16, torch.float16) and x.is_contiguous() and C % 8 == 0
            and scale.dtype == shift.dtype == x.dtype and scale.dim() == 2 and shift.dim() == 2
            and scale.stride(1) == 1 and shift.stride(1) == 1 and scale.stride(0) == shift.stride(0)
            and scale.stride(0) % 8 == 0 and scale.data_ptr() % 16 == 0 and shift.data_ptr() % 16 == 0):
        count("channel_affine", "hip")
        y = torch.empty_like(x)
        _check(_lib().cgs_channel_affine2(x.data_ptr(), scale.data_ptr(), shift.data_ptr(), scale.stride(0),
                                          y.data_ptr(), N, x.numel() // (N * C), C, float(add), _DT[x.dtype],
                                          _stream()), "cgs_channel_affine2")
        return y
    count("channel_affine", "torch")
    shp = (N,) + (1,) * (x.dim() - 2) + (C,)
    return (x.float() * (add + scale.reshape(shp).float()) + shift.reshape(shp).float()).to(x.dtype)


def channel_affine_layernorm_nhwc(x: torch.Tensor, scale: torch.Tensor, shift: torch.Tensor, add: float = 0.0,
                                   eps: float = 1e-6):
    """``(xa, LN(xa))`` with xa = ``channel_affine_nhwc(x, scale, shift, add)`` and LN a LayerNorm over C
    without affine, from one read of x (Stable Cascade TimestepBlock -> AttnBlock). Same coefficient
    layout as channel_affine_nhwc."""
    N, C = x.shape[0], x.shape[-1]
    if (x.is_cuda and x.dtype in (torch.bfloat16, torch.float16) and x.is_contiguous() and C % 8 == 0
            and C <= 4096 and _native.has_kernel("cgs_affine_layernorm")
            and backend_for("channel_affine", x, "cgs_affine_layernorm") == "hip"
            and scale.dtype == shift.dtype == x.dtype and scale.dim() == 2 and shift.dim() == 2
            and scale.stride(1) == 1 and shift.stride(1) == 1 and scale.stride(0) == shift.stride(0)
            and scale.stride(0) % 8 == 0 and scale.data_ptr() % 16 == 0 and shift.data_ptr() % 16 == 0):
        count("channel_affine", "hip")
        count("layernorm", "hip")
        xa = torch.empty_like(x)
        y = torch.empty_like(x)
        _check(_lib().cgs_affine_layernorm(x.data_ptr(), scale.data_ptr(), shift.data_ptr(), scale.stride(0),
                                           float(add), xa.data_ptr(), y.data_ptr(), N, x.numel() // (N * C), C,
                                           float(eps), _DT[x.dtype], _stream()), "cgs_affine_layernorm")
        return xa, y
    xa = channel_affine_nhwc(x, scale, shift, add)
    return xa, layer_norm(xa, None, None, eps)


def fused_bias_act(x: torch.Tensor, bias: torch.Tensor | None, negative_slope: float = 0.2,
                   scale: float = 2 ** 0.5) -> torch.Tensor:
    """StyleGAN2 FusedLeakyReLU (K32, ``face/fused_act.py``): leaky_relu(x + bias[c]) * scale,
    bias broadcast along dim 1."""
    be = backend_for("fused_bias_act", x, "cgs_fused_bias_act")
    C = x.shape[1] if x.dim() > 1 else x.shape[0]
    if be == "hip" and x.dtype in _DT and x.numel() > 0:
        count("fused_bias_act", "hip")
        xc = x.contiguous()
        y = torch.empty_like(xc)
        inner = 1
        for d in x.shape[2:]:
            inner *= d
        b = None if bias is None else bias.to(x.dtype).contiguous()
        _check(_lib().cgs_fused_bias_act(xc.data_ptr(), _ptr(b), y.data_ptr(), xc.numel(), C, inner,
                                         float(negative_slope), float(scale), _DT[x.dtype], _stream()),
               "cgs_fused_bias_act")
        return y
    if bias is not None:
        x = x + bias.to(x.dtype).view(1, C, *([1] * (x.dim() - 2)))
    return F.leaky_relu(x, negative_slope) * scale


def upfirdn2d(x: torch.Tensor, kernel: torch.Tensor, up=1, down=1, pad=(0, 0)) -> torch.Tensor:
    """StyleGAN2 upfirdn2d (K32, ``face/upfirdn2d.py``) on NCHW: zero-insert upsample, pad
    (negative crops), FIR with the flipped kernel, decimate. ``pad`` = (p0, p1) for both axes or
    (px0, px1, py0, py1)."""
    ux, uy = (up, up) if isinstance(up, int) else up
    dx, dy = (down, down) if isinstance(down, int) else down
    px0, px1, py0, py1 = (pad[0], pad[1], pad[0], pad[1]) if len(pad) == 2 else pad
    N, C, H, W = x.shape
    kh, kw = kernel.shape
    be = backend_for("upfirdn2d", x, "cgs_upfirdn2d")
    if be == "hip" and x.dtype in _DT and kh * kw <= 1024:
        count("upfirdn2d", "hip")
        Ho = (H * uy + py0 + py1 - kh) // dy + 1
        Wo = (W * ux + px0 + px1 - kw) // dx + 1
        xc = x.contiguous()
        k = kernel.to(device=x.device, dtype=torch.float32).contiguous()
        y = torch.empty((N, C, Ho, Wo), device=x.device, dtype=x.dtype)
        _check(_lib().cgs_upfirdn2d(xc.data_ptr(), k.data_ptr(), y.data_ptr(), N * C, H, W, ux, uy, dx, dy,
                                    px0, px1, py0, py1, kh, kw, _DT[x.dtype], _stream()), "cgs_upfirdn2d")
        return y
    return upfirdn2d_reference(x, kernel, (ux, uy), (dx, dy), (px0, px1, py0, py1))


def upfirdn2d_reference(x, kernel, up, down, pad):
    """Plain PyTorch fp32 upfirdn2d (numerics oracle / CPU path)."""
    (ux, uy), (dx, dy), (px0, px1, py0, py1) = up, down, pad
    N, C, H, W = x.shape
    xf = x.float().reshape(N * C, 1, H, W)
    u = xf.new_zeros(N * C, 1, H * uy, W * ux)
    u[:, :, ::uy, ::ux] = xf
    u = F.pad(u, (max(px0, 0), max(px1, 0), max(py0, 0), max(py1, 0)))
    u = u[:, :, max(-py0, 0):u.shape[2] - max(-py1, 0), max(-px0, 0):u.shape[3] - max(-px1, 0)]
    w = torch.flip(kernel.float().to(x.device), [0, 1])[None, None]
    out = F.conv2d(u, w)[:, :, ::dy, ::dx]
    return out.reshape(N, C, out.shape[2], out.shape[3]).to(x.dtype)


def vq_nearest(z: torch.Tensor, codebook: torch.Tensor):
    """Nearest codebook row for every row of ``z`` [M, D] (K31: Stage A VQ, RestoreFormer /
    CodeFormer quantizers) -> (quantized [M, D], indices int64 [M])."""
    M, D = z.shape
    be = backend_for("vq", z, "cgs_vq_nearest")
    if be == "hip" and z.dtype in _DT and D <= 4096 and M > 0:
        count("vq", "hip")
        zc = z.contiguous()
        cb = codebook.to(z.dtype).contiguous()
        idx = torch.empty(M, device=z.device, dtype=torch.int64)
        q = torch.empty_like(zc)
        _check(_lib().cgs_vq_nearest(zc.data_ptr(), cb.data_ptr(), idx.data_ptr(), q.data_ptr(), M, cb.shape[0], D,
                                     _DT[z.dtype], _stream()), "cgs_vq_nearest")
        return q, idx
    zf, cf = z.float(), codebook.float()
    d = zf.pow(2).sum(1, keepdim=True) + cf.pow(2).sum(1)[None] - 2.0 * zf @ cf.t()
    idx = d.argmin(1)
    return codebook[idx].to(z.dtype), idx


def grn_nhwc(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, pre_gelu: bool = False) -> torch.Tensor:
    """ConvNeXt-V2 GlobalResponseNorm on NHWC [N, H, W, C] (K28, Cascade ``common.py:77-87``):
    beta + a * (1 + gamma * ||a||_HW / mean_C ||a||_HW), a = x, or gelu(x) with ``pre_gelu`` (the
    Linear -> GELU -> GRN of Cascade's ChannelMLP: the GELU is fused into both reads of x)."""
    N, H, W, C = x.shape
    be = backend_for("grn", x, "cgs_grn_nhwc")
    gp = _grn_part(x, N, H * W, C) if not pre_gelu and be == "hip" else None
    if gp is not None:        # statistics from the producing GEMM's epilogue (linear_lnfold gns_hw)
        count("grn", "hip")
        y = torch.empty_like(x)
        ws = torch.empty(N * (C + (C + 255) // 256), device=x.device, dtype=torch.float32)
        g = gamma.to(x.dtype).reshape(-1).contiguous()
        b = beta.to(x.dtype).reshape(-1).contiguous()
        _check(_lib().cgs_grn_apply_gns(x.data_ptr(), gp.data_ptr(), g.data_ptr(), b.data_ptr(), y.data_ptr(),
                                        ws.data_ptr(), N, H * W, C, _stream()), "cgs_grn_apply_gns")
        return y
    if be == "hip" and x.dtype in (torch.bfloat16, torch.float16) and C % 8 == 0 and N <= 64 and \
            _native.has_kernel("cgs_grn_nhwc_v2"):
        count("grn", "hip")
        xc = x.contiguous()
        y = torch.empty_like(xc)
        S = int(_lib().cgs_grn_slices(N, H * W, C))
        ws = torch.empty(N * ((S + 1) * C + (C + 255) // 256), device=x.device, dtype=torch.float32)
        g = gamma.to(x.dtype).reshape(-1).contiguous()
        b = beta.to(x.dtype).reshape(-1).contiguous()
        _check(_lib().cgs_grn_nhwc_v2(xc.data_ptr(), g.data_ptr(), b.data_ptr(), y.data_ptr(), ws.data_ptr(), N,
                                      H * W, C, 1 if pre_gelu else 0, _DT[x.dtype], _stream()), "cgs_grn_nhwc_v2")
        return y
    if pre_gelu:
        x = F.gelu(x)
    if be == "hip" and x.dtype in _DT:
        count("grn", "hip")
        xc = x.contiguous()
        y = torch.empty_like(xc)
        ws = torch.zeros(2 * N * C, device=x.device, dtype=torch.float32)
        _check(_lib().cgs_grn_nhwc(xc.data_ptr(), gamma.to(x.dtype).contiguous().data_ptr(),
                                   beta.to(x.dtype).contiguous().data_ptr(), y.data_ptr(), ws.data_ptr(), N, H * W, C,
                                   _DT[x.dtype], _stream()), "cgs_grn_nhwc")
        return y
    gx = torch.linalg.vector_norm(x, dim=(1, 2), keepdim=True, dtype=torch.float32)
    nx = gx / (gx.mean(dim=-1, keepdim=True) + 1e-6)
    scale = (1.0 + gamma.float().reshape(1, 1, 1, C) * nx).to(x.dtype)
    return torch.addcmul(beta.to(x.dtype).reshape(1, 1, 1, C), x, scale)


def _grn_part(x, N, HW, C):
    """The GNS partials attached by ``_gelu_gns`` when they describe exactly this tensor, else None."""
    h = getattr(x, "_cgs_grnpart", None)
    if (h is None or h[1] != x.data_ptr() or h[2] != HW or not x.is_contiguous() or x.dtype != torch.bfloat16
            or h[0].numel() != N * (HW // 64) * C or N > 64 or C % 8):
        return None
    return h[0]


def grn_fold_weight(h: torch.Tensor, weight: torch.Tensor, gamma: torch.Tensor) -> torch.Tensor:
    """The GlobalResponseNorm over ``h`` [N, H, W, K] (already GELU'd) folded into the next Linear's
    weight [O, K]: returns per-image weights Wn [N, O, K] = W * (1 + gamma * nx_n), nx_n =
    ||h_n||_HW / mean_K ||h_n||_HW, so that GRN(h) W^T = h_n Wn[n]^T + W beta per image (K28 fused with
    the ChannelMLP's second GEMM, Cascade ``common.py:77-87``). Cheaper than rewriting h whenever O < H * W.
    Device path: the GRN statistics passes + one weight-scaling pass (W read once for all images)."""
    N, H, W_, K = h.shape
    O = weight.shape[0]
    be = backend_for("grn", h, "cgs_grn_scale_weight")
    if (be == "hip" and h.dtype == torch.bfloat16 and weight.dtype == h.dtype and K % 8 == 0 and N <= 64
            and weight.shape[1] == K):
        count("grn", "hip")
        hc = h.contiguous()
        S = int(_lib().cgs_grn_slices(N, H * W_, K))
        ws = torch.empty(N * ((S + 1) * K + (K + 255) // 256), device=h.device, dtype=torch.float32)
        gp = _grn_part(h, N, H * W_, K)
        if gp is not None:      # statistics from the producing GEMM's epilogue (linear_lnfold gns_hw)
            _check(_lib().cgs_grn_stats_gns(gp.data_ptr(), ws.data_ptr(), N, H * W_, K, _stream()), "cgs_grn_stats_gns")
        else:
            _check(_lib().cgs_grn_stats(hc.data_ptr(), ws.data_ptr(), N, H * W_, K, 0, _DT[h.dtype], _stream()),
                   "cgs_grn_stats")
        wc = weight.contiguous()
        g = gamma.to(h.dtype).reshape(-1).contiguous()
        out = torch.empty((N, O, K), device=h.device, dtype=h.dtype)
        _check(_lib().cgs_grn_scale_weight(wc.data_ptr(), g.data_ptr(), ws.data_ptr(), N, H * W_, O, K,
                                           out.data_ptr(), _stream()), "cgs_grn_scale_weight")
        return out
    count("grn", "torch")
    gx = torch.linalg.vector_norm(h.float(), dim=(1, 2))                        # [N, K]
    nx = gx / (gx.mean(dim=-1, keepdim=True) + 1e-6)
    s = 1.0 + gamma.float().reshape(1, K) * nx
    return (weight.float()[None] * s[:, None, :]).to(weight.dtype)


def softmax_rows(x: torch.Tensor, scale: float = 1.0) -> torch.Tensor:
    """fp32 softmax over the last dim of ``scale * x`` (K05: the materialised attention map SAG /
    PAG read). Device path: one wave per row."""
    be = backend_for("softmax", x, "cgs_softmax_rows")
    if be == "hip" and x.dtype in _DT and x.numel() > 0:
        count("softmax", "hip")
        xc = x.contiguous()
        y = torch.empty(xc.shape, device=x.device, dtype=torch.float32)
        _check(_lib().cgs_softmax_rows(xc.data_ptr(), y.data_ptr(), xc.numel() // xc.shape[-1], xc.shape[-1],
                                       float(scale), _DT[x.dtype], _stream()), "cgs_softmax_rows")
        return y
    return torch.softmax(x.float() * scale, dim=-1)


def attention_with_probs(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, heads: int):
    """Attention that also returns the probabilities [(b*heads), Sq, Sk] in fp32 (K05: SAG / PAG read
    the map). Device: scores and PV as batched fp32-MFMA GEMMs straight from the strided per-head
    views (``cgs_bgemm_f32``: exact fp32 products, the reference's fp32 bmm precision), the softmax
    writing P in place (``cgs_softmax_rows``); CPU: fp32 torch."""
    b, sq, hd = q.shape
    d = hd // heads
    sk = k.shape[1]
    if (q.is_cuda and q.dtype in (torch.bfloat16, torch.float16) and k.dtype == q.dtype and v.dtype == q.dtype
            and q.stride(-1) == 1 and k.stride(-1) == 1 and v.stride(-1) == 1
            and backend_for("attention", q, "cgs_bgemm_f32") == "hip"
            and backend_for("softmax", q, "cgs_softmax_rows") == "hip"):
        lib, st, dt = _lib(), _stream(), _DT[q.dtype]
        bh = b * heads
        p = torch.empty((bh, sq, sk), device=q.device, dtype=torch.float32)
        # batch index = b * heads + h: per-head base = b*stride(0) + h*d  (sab covers h via the loop)
        for bi in range(b):
            _check(lib.cgs_bgemm_f32(q[bi].data_ptr(), k[bi].data_ptr(), p[bi * heads].data_ptr(), heads, sq, sk, d,
                                     d, q.stride(1), 1, d, 1, k.stride(1), sq * sk, sk, 1.0, dt, dt, st),
                   "cgs_bgemm_f32")
        count("softmax", "hip")
        _check(lib.cgs_softmax_rows(p.data_ptr(), p.data_ptr(), bh * sq, sk, float(d ** -0.5), 0, st),
               "cgs_softmax_rows")
        o = torch.empty((b, sq, hd), device=q.device, dtype=torch.float32)
        for bi in range(b):
            _check(lib.cgs_bgemm_f32(p[bi * heads].data_ptr(), v[bi].data_ptr(), o[bi].data_ptr(), heads, sq, d, sk,
                                     sq * sk, sk, 1, d, v.stride(1), 1, d, hd, 1.0, 0, dt, st), "cgs_bgemm_f32")
        count("attention", "hip")
        return o.to(q.dtype), p
    qh = q.reshape(b, sq, heads, d).permute(0, 2, 1, 3).reshape(b * heads, sq, d).float()
    kh = k.reshape(b, -1, heads, d).permute(0, 2, 1, 3).reshape(b * heads, -1, d).float()
    vh = v.reshape(b, -1, heads, d).permute(0, 2, 1, 3).reshape(b * heads, -1, d).float()
    p = softmax_rows(torch.bmm(qh, kh.transpose(1, 2)), d ** -0.5)
    o = torch.bmm(p, vh).reshape(b, heads, sq, d).permute(0, 2, 1, 3).reshape(b, sq, hd)
    return o.to(q.dtype), p


# ----------------------------------------------------------------------------------------------
# Device-parameterised sampler step (rng.hip): the per-step scalars live in a device table and a
# device step counter, so one captured graph is replayed for every step (sampling/step_graph.py)
# ----------------------------------------------------------------------------------------------
def step_param(out: torch.Tensor, params: torch.Tensor, meta: torch.Tensor, col: int = 0):
    """out[:] = params[meta[0], col] (fp32 device vector)."""
    _check(_lib().cgs_step_param(out.data_ptr(), out.numel(), params.data_ptr(), params.shape[1], col,
                                 meta.data_ptr(), _stream()), "cgs_step_param")
    return out


def sampler_step_dev(x: torch.Tensor, cond_den: torch.Tensor, uncond_den: torch.Tensor | None,
                     den_out: torch.Tensor | None, cfg: float, params: torch.Tensor, meta: torch.Tensor):
    """In place on ``x``: CFG combine + Euler(-ancestral) update + in-register noise, scalars from
    ``params[meta[0]] = (sigma, sigma_down, sigma_up, s_noise)``, seed/index0 from ``meta[1:3]``."""
    count("euler", "hip")
    _check(_lib().cgs_sampler_step_dev(x.data_ptr(), cond_den.data_ptr(), _ptr(uncond_den), _ptr(den_out),
                                       int(x.shape[0]), _numel1(x.shape), float(cfg), params.data_ptr(),
                                       params.shape[1], meta.data_ptr(), _stream()), "cgs_sampler_step_dev")
    return x


def step_advance(meta: torch.Tensor):
    _check(_lib().cgs_step_advance(meta.data_ptr(), _stream()), "cgs_step_advance")


def vae_out_u8(x: torch.Tensor) -> torch.Tensor:
    """VAE decoder output [N, C, H, W] (NHWC in memory) -> uint8 [N, H, W, C]:
    (clamp((x + 1) / 2, 0, 1) * 255 + 0.5).to(uint8) in one pass on the device (K23)."""
    be = backend_for("vae_u8", x, "cgs_vae_out_u8")
    N, C, H, W = x.shape
    if be == "hip" and x.dtype == torch.bfloat16 and x.is_contiguous(memory_format=torch.channels_last):
        count("vae_u8", "hip")
        y = torch.empty((N, H, W, C), device=x.device, dtype=torch.uint8)
        _check(_lib().cgs_vae_out_u8(x.data_ptr(), y.data_ptr(), x.numel(), _stream()), "cgs_vae_out_u8")
        return y
    count("vae_u8", "torch")
    v = torch.clamp((x.float() + 1.0) / 2.0, 0.0, 1.0).movedim(1, -1)
    return (v * 255.0 + 0.5).to(torch.uint8)
