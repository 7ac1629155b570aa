"""Loader for the in-tree native libraries.

Two shared objects are built by ``build_native.py`` (invoked by ``__graft_entry__.build``):

* ``libcgs_kernels.so`` — hand-written HIP kernels for gfx950 (MFMA GEMM / flash attention /
  GroupNorm+SiLU / LayerNorm / fused sampler steps ...). Exposed as ``extern "C"`` launchers that
  take raw device pointers and a ``hipStream_t``; bound here with ctypes so the kernels launch on
  torch's current stream and are captured transparently by hipGraphs.
* ``_cgs_runtime*.so`` — C++ runtime (safetensors mmap reader, CLIP BPE tokenizer, BLAKE3,
  prompt priority queue) as a CPython extension module.

On a GPU box the kernel library MUST load: ops fail loudly instead of silently falling back to
PyTorch (set ``CGS_ALLOW_TORCH_FALLBACK=1`` to opt into the fallback explicitly).
"""
from __future__ import annotations

import ctypes
import glob
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(_HERE, "lib")
_lock = threading.Lock()
_kernels = None
_kernels_err = None


def kernel_lib_path() -> str:
    """The in-tree kernel library (``CGS_KERNELS_SO`` names another build of it: kernel A/B runs)."""
    return os.environ.get("CGS_KERNELS_SO") or os.path.join(LIB_DIR, "libcgs_kernels.so")


def load_kernels():
    """Return the ctypes handle of libcgs_kernels.so or None if it is not built."""
    global _kernels, _kernels_err
    if _kernels is not None or _kernels_err is not None:
        return _kernels
    with _lock:
        if _kernels is not None or _kernels_err is not None:
            return _kernels
        path = kernel_lib_path()
        if not os.path.exists(path):
            _kernels_err = f"{path} not built (run python build_native.py)"
            return None
        try:
            # torch must be imported first so libamdhip64 is already resident with its symbols.
            import torch  # noqa: F401
            lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
            _declare(lib)
            _kernels = lib
        except OSError as e:  # pragma: no cover - depends on the box
            _kernels_err = str(e)
            _kernels = None
    return _kernels


def kernels_error():
    return _kernels_err


_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_longlong
_F = ctypes.c_float

# name -> argtypes. Every launcher returns int (hipError_t) and takes the stream last.
KERNEL_SIGNATURES = {
    # y = GN(x + pre_add) (+SiLU); NHWC layout, x [N, HW, C]; ws = torch-allocated workspace
    "cgs_groupnorm_nhwc_ws": [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _F, _I, _I, _P],
    "cgs_groupnorm_workspace": [_I, _I, _I],
    # GroupNorm over cat([x, x2], C) without materialising the concat (K14): x, x2, C1, y, ...
    "cgs_groupnorm_nhwc_dual": [_P, _P, _I, _P, _P, _P, _P, _P, _I, _I, _I, _I, _F, _I, _I, _P],
    # y = LN(x) over last dim; rows x C
    "cgs_layernorm": [_P, _P, _P, _P, _I, _I, _F, _I, _P],
    # flash attention forward (bf16): q,k,v,o + strides (elements) + shapes
    "cgs_flash_attn_fwd": [_P, _P, _P, _P,
                           _I, _I, _I, _I, _I,          # B, H, Sq, Sk, D
                           _L, _L, _L,                  # q strides (b, s, h)
                           _L, _L, _L,                  # k strides
                           _L, _L, _L,                  # v strides
                           _L, _L, _L,                  # o strides
                           _F, _P, _I, _P],             # scale, key_mask(int8 [B,Sk] or null), causal, stream
    # per-call kernel variant (op-layer autotune): ..., scale, variant, stream
    "cgs_flash_attn_fwd_v": [_P, _P, _P, _P, _I, _I, _I, _I, _I, _L, _L, _L, _L, _L, _L, _L, _L, _L, _L, _L, _L, _F,
                             _I, _P],
    # generic kernel + additive fp32 bias [H,Sq,Sk] and window mask [nW,Sq,Sk] (Swin family): ..., scale, bias,
    # mask, nW, hscale [H] fp32 or null, stream
    "cgs_flash_attn_fwd_bias": [_P, _P, _P, _P, _I, _I, _I, _I, _I, _L, _L, _L, _L, _L, _L, _L, _L, _L, _L, _L, _L,
                                _F, _P, _P, _I, _P, _P],
    # same + fp32 LSE [B, H, Sq] out (ring attention merge): q,k,v,o,lse, B,H,Sq,Sk,D, 12 strides, scale
    "cgs_flash_attn_fwd_lse": [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _L, _L, _L, _L, _L, _L, _L, _L, _L, _L, _L, _L,
                               _F, _P],
    # C[M,N] = A[M,K] @ W[N,K]^T (+bias) (+residual) | GEGLU epilogue; bf16 in/out, fp32 acc
    "cgs_gemm_bf16": [_P, _P, _P, _P, _P, _I, _I, _I, _L, _L, _L, _L, _I, _F, _P],
    "cgs_gemm_set_variant": [_I],   # -1 auto, 1 force 128x128 register-staged, 2 force 256-tile glds, 3 mfma32 4-stage
    "cgs_conv_set_variant": [_I],
    "cgs_attn_set_variant": [_I],     # 0 auto (D=64 fast kernel where legal), 1 generic, 2 fast only
    "cgs_set_tile_group": [_I],       # grouped tile order for GEMM v2/v3 (tile rows per group)
    "cgs_conv_set_tile_group": [_I],   # -1 auto (v3 where legal), 2 force the 8-wave 2-stage kernel
    "cgs_dwconv_set_px": [_I],
    "cgs_affine_layernorm": [_P, _P, _P, _L, _F, _P, _P, _I, _I, _I, _F, _I, _P],         # output pixels per thread of the depthwise 3x3 kernel (1 / 2 / 4)
    # out = a * gelu(g) where [a | g] = x rows of width 2*N
    "cgs_geglu": [_P, _P, _I, _I, _I, _P],   # x [M, 2N] -> out [M, N], dtype
    # fused CFG combine: out = u + (c - u) * scale   (fp32 or bf16 denoised)
    "cgs_cfg_combine": [_P, _P, _P, _L, _F, _I, _P],
    # Euler-ancestral / Euler update: x = x + d * dt (+ noise * s_up), d = (x - den)/sigma
    "cgs_euler_step": [_P, _P, _P, _L, _F, _F, _F, _P],   # in place on x
    # timestep sinusoidal embedding
    "cgs_timestep_embedding": [_P, _P, _I, _I, _F, _I, _P],
    # elementwise y = silu(x) (bf16)
    "cgs_silu": [_P, _P, _L, _I, _P],
    # NHWC nearest upsample x2
    "cgs_upsample_nearest2x_nhwc": [_P, _P, _I, _I, _I, _I, _I, _P],
    # depthwise conv NHWC: x, w[k*k, C], bias, y, N, H, W, C, k, replicate, dtype, stream
    "cgs_dwconv_nhwc": [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P],
    # the same + per-pixel LayerNorm (mean, rstd) over C: x, w, bias, y, rs, N, H, W, C, k, replicate, eps, dtype
    "cgs_dwconv_ln_stats_nhwc": [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _F, _I, _P],
    # conv implicit GEMM NHWC bf16: x[N,H,W,Cin], w[Cout,kh,kw,Cin], bias, residual, out
    "cgs_conv2d_nhwc": [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P],
    # image / utility kernels (csrc/kernels/image.hip)
    "cgs_fused_bias_act": [_P, _P, _P, _L, _I, _L, _F, _F, _I, _P],   # x, bias, y, n, C, inner, slope, scale
    "cgs_upfirdn2d": [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P],
    "cgs_resize": [_P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P],        # x, y, NC, H, W, Ho, Wo, mode, align
    "cgs_vq_nearest": [_P, _P, _P, _P, _I, _I, _I, _I, _P],            # z, codebook, idx(i64), q, M, n, D
    "cgs_grn_nhwc": [_P, _P, _P, _P, _P, _I, _I, _I, _I, _P],          # x, gamma, beta, y, ws, N, HW, C
    # GRN statistics only (gx / block sums in the v2 ws layout): x, ws, N, HW, C, pre_gelu, dtype
    "cgs_grn_stats": [_P, _P, _I, _I, _I, _I, _I, _P],
    "cgs_splitk_ws_bytes": [_I, _I, _I],
    "cgs_gemm_bf16_splitk": [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _L, _L, _L, _L, _I, _F, _I, _I, _P, _L, _P],
    "cgs_grn_stats_gns": [_P, _P, _I, _I, _I, _P],                      # part, ws, N, HW, C
    "cgs_grn_apply_gns": [_P, _P, _P, _P, _P, _P, _I, _I, _I, _P],      # h, part, gamma, beta, y, ws, N, HW, C
    "cgs_gemm_bf16_gelu_gns": [_P, _P, _P, _P, _P, _P, _I, _I, _I, _L, _L, _L, _I, _P, _I, _P],
    # per-image GRN-scaled weights of the next Linear: W, gamma, ws(stats), N, HW, O, K, Wn
    "cgs_grn_scale_weight": [_P, _P, _P, _I, _I, _I, _I, _P, _P],
    # host (mmap) -> device upload through pinned double buffers (csrc/kernels/io.hip)
    "cgs_h2d_upload": [_P, _P, _L, _L, _I, _P],                        # src, dst, nbytes, chunk, threads
    # f32.hip: fp32-I/O GEMM / conv / GroupNorm / LayerNorm (--force-fp32, --fp32-vae)
    "cgs_gemm_f32": [_P, _P, _P, _P, _P, _I, _I, _I, _L, _L, _L, _L, _I, _F, _I, _I, _L, _L, _L, _P],
    "cgs_conv_f32": [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P],
    "cgs_groupnorm_f32_ws": [_I, _I, _I],
    "cgs_groupnorm_f32": [_P, _P, _I, _P, _P, _P, _P, _P, _I, _I, _I, _I, _F, _I, _P],
    "cgs_layernorm_f32": [_P, _P, _P, _P, _L, _I, _F, _P],
    "cgs_softmax_rows": [_P, _P, _L, _I, _F, _I, _P],                  # x, y(f32), rows, cols, scale, dtype
    # bf16 activations x fp8-e4m3fn weights (K21), same epilogues as cgs_gemm_bf16
    "cgs_gemm_bf16_w8": [_P, _P, _P, _P, _P, _I, _I, _I, _L, _L, _L, _L, _I, _F, _P],
    "cgs_gemm_bf16_v": [_P, _P, _P, _P, _P, _I, _I, _I, _L, _L, _L, _L, _I, _F, _I, _P],
    "cgs_conv2d_nhwc_v": [_P, _P, _I, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P],
    # counter-based noise keyed by (seed, global image index, stream) (csrc/kernels/rng.hip, K18)
    "cgs_philox_randn": [_P, _I, _L, ctypes.c_ulonglong, _L, ctypes.c_ulonglong, _P, _F, _I, _P, _P],
    "cgs_euler_ancestral_philox": [_P, _P, _I, _L, _F, _F, _F, ctypes.c_ulonglong, _L, ctypes.c_ulonglong, _P, _P],
    "cgs_brownian_increment": [_P, _I, _L, ctypes.c_ulonglong, _L, ctypes.c_double, ctypes.c_double,
                               ctypes.c_double, ctypes.c_double, ctypes.c_double, _I, _F, _P, _P],
    # device-parameterised sampler step (one captured graph replayed for every step; rng.hip)
    "cgs_sampler_step_dev": [_P, _P, _P, _P, _I, _L, _F, _P, _I, _P, _P],
    "cgs_step_param": [_P, _I, _P, _I, _I, _P, _P],
    "cgs_step_advance": [_P, _P],
    "cgs_vae_out_u8": [_P, _P, _L, _P],                                # bf16 NHWC -> uint8 image (K23)
    "cgs_conv2d_nhwc_ex": [_P, _P, _I, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P],
    # K17/K24 region accumulate: out, div, piece, pdt, mult, mdt, B, C, Ho, Wo, h, w, oy, ox, piece strides x4,
    # Cm, mult strides x4, feather, scale
    "cgs_region_accumulate": [_P, _P, _P, _I, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _L, _L, _L, _L, _I, _L, _L,
                              _L, _L, _I, _F, _P],
    "cgs_region_normalize": [_P, _P, _P, _L, _I, _P],
    # K26 CLIP embeddings: ids, tok, pos, y, B, S, D, vocab, dtype / pooled gather: ids, x, out, B, S, D, dtype
    "cgs_clip_embed": [_P, _P, _P, _P, _I, _I, _I, _I, _I, _P],
    "cgs_pooled_gather": [_P, _P, _P, _I, _I, _I, _I, _P],
    # LayerNorm folded into the GEMM: row stats (x, rs, rows, C, eps, dtype) and the v7 GEMM with the fold
    "cgs_layernorm_stats": [_P, _P, _I, _I, _F, _I, _P],
    "cgs_gemm_bf16_lnfold": [_P, _P, _P, _P, _P, _P, _I, _I, _I, _L, _L, _L, _I, _P, _L, _P],
    "cgs_gemm_bf16_lnfold_v": [_P, _P, _P, _P, _P, _P, _I, _I, _I, _L, _L, _L, _I, _P, _L, _I, _P],
    # v7 split-K tail: workspace bytes for (M, N, K) and the GEMM / conv launchers that take it
    "cgs_v7_ws_bytes": [_I, _I, _I],
    "cgs_v7_set_dbg": [_I],
    "cgs_v6_set_mode": [_I],
    "cgs_attn_set_prio": [_I],
    "cgs_gn_set_blocks": [_I],
    "cgs_conv_smalln_set_lds": [_I],
    "cgs_attn_set_kv2_rows": [_I],
    "cgs_grn_set_rows": [_I],
    "cgs_flash_attn_fwd_ks": [_P, _P, _P, _P, _I, _I, _I, _I, _L, _L, _L, _L, _L, _L, _L, _L, _F, _I, _P, _P, _P],
    "cgs_flash_attn_fwd_kv2": [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _L, _L, _L, _L, _L, _L, _L, _L, _L, _L, _L, _L, _F, _P],
    "cgs_conv2d_nhwc_gns": [_P, _P, _I, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P],
    # row-sharded GroupNorm (parallel/spatial.py): band statistics, then apply with combined (mean, rstd)
    "cgs_groupnorm_band_stats": [_P, _P, _I, _P, _P, _P, _I, _I, _I, _I, _I, _P],
    "cgs_groupnorm_apply_stats": [_P, _P, _I, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P],
    "cgs_groupnorm_nhwc_part": [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _F, _I, _I, _P],
    # the same with a row stride (elements) for pre_add: a column slice of the batched time-embedding GEMM
    "cgs_groupnorm_nhwc_part_pld": [_P, _P, _P, _P, _P, _I, _P, _P, _I, _I, _I, _I, _I, _F, _I, _I, _P],
    "cgs_groupnorm_nhwc_ws_pld": [_P, _P, _P, _P, _P, _I, _P, _I, _I, _I, _I, _F, _I, _I, _P],
    "cgs_groupnorm_nhwc_dual_pld": [_P, _P, _I, _P, _P, _P, _P, _I, _P, _I, _I, _I, _I, _F, _I, _I, _P],
    "cgs_gemm_bf16_v7ws": [_P, _P, _P, _P, _P, _I, _I, _I, _L, _L, _L, _L, _I, _F, _P, _L, _P],
    "cgs_conv2d_nhwc_v7ws": [_P, _P, _I, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _L, _P],
    # K29 FreeU low-frequency filter: x, y, coef ws, B, C, H, W, x strides x4, y strides x4, t, scale, dtype
    "cgs_fourier_filter": [_P, _P, _P, _I, _I, _I, _I, _L, _L, _L, _L, _L, _L, _L, _L, _I, _F, _I, _P],
    # K30 ToMe matching: a, b, ws, vmax, imax(i64), B, Na, Nb, C, a strides (batch, row), b strides, dtype
    "cgs_tome_match": [_P, _P, _P, _P, _P, _I, _I, _I, _I, _L, _L, _L, _L, _I, _P],
    # K28 v2 GRN (vectorised, optional fused pre-GELU): x, gamma, beta, y, ws, N, HW, C, pre_gelu, dtype
    "cgs_grn_nhwc_v2": [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P],
    "cgs_grn_slices": [_I, _I, _I],
    # K05 batched fp32-MFMA GEMM: A, B, C, batch, M, N, K, A strides (b, m, k), B strides (b, k, n), C (b, m), alpha, dta, dtb
    "cgs_bgemm_f32": [_P, _P, _P, _I, _I, _I, _I, _L, _L, _L, _L, _L, _L, _L, _L, _F, _I, _I, _P],
    # K22 materialised wide-head attention: fp32 S -> bf16 P row softmax (log2 units) and a bf16 transpose
    "cgs_softmax2_f32_bf16": [_P, _P, _L, _I, _L, _L, _P],             # x(f32), y(bf16), rows, cols, ldx, ldy
    "cgs_transpose_bf16": [_P, _P, _I, _I, _L, _L, _P],                # x, y, rows, cols, ldx, ldy
    "cgs_abort_stream_capture": [_P],
    "cgs_channel_affine2": [_P, _P, _P, _L, _P, _I, _I, _I, _F, _I, _P],
    # experiment: 4-slot-ring one-wave-per-SIMD GEMM (bias / residual epilogue only)
    "cgs_gemm_bf16_w6": [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _L, _L, _L, _L, _I, _F, _I, _I, _I, _I, _P],
    "cgs_gemm_w6_ok": [_I, _I, _I, _L, _L, _L, _L, _I, _I],
    # skinny GEMM (M <= 128) with its split-K workspace
    "cgs_gemm_skinny_ws": [_P, _P, _P, _P, _P, _I, _I, _I, _L, _L, _L, _L, _I, _F, _P, _L, _P],
    "cgs_gemm_skinny_ws_bytes": [_I, _I, _I],
    # v6 GEMM + per-row LayerNorm statistics partials; partials -> (mean, rstd) rows
    "cgs_gemm_bf16_rowstats": [_P, _P, _P, _P, _P, _I, _I, _I, _L, _L, _L, _L, _I, _F, _P, _P],
    "cgs_gemm_bf16_rowstats_v": [_P, _P, _P, _P, _P, _I, _I, _I, _L, _L, _L, _L, _I, _F, _P, _I, _P],
    "cgs_ln_rs_from_partials": [_P, _P, _I, _I, _F, _P],
    # v6 conv gather override (-1 auto, 1 ConvGatherK, 0 ConvGatherA8): in-process A/B
    "cgs_conv_v6_set_loader": [_I],
}


_RESTYPE = {"cgs_groupnorm_workspace": ctypes.c_longlong, "cgs_splitk_ws_bytes": ctypes.c_longlong, "cgs_groupnorm_f32_ws": ctypes.c_longlong, "cgs_grn_slices": ctypes.c_int, "cgs_v7_ws_bytes": ctypes.c_longlong, "cgs_gemm_skinny_ws_bytes": ctypes.c_longlong, "cgs_gemm_set_variant": None, "cgs_v7_set_dbg": None, "cgs_v6_set_mode": None, "cgs_attn_set_prio": None, "cgs_gn_set_blocks": None, "cgs_conv_smalln_set_lds": None, "cgs_attn_set_kv2_rows": None, "cgs_grn_set_rows": None,
            "cgs_conv_set_variant": None, "cgs_set_tile_group": None, "cgs_conv_set_tile_group": None, "cgs_dwconv_set_px": None,
            "cgs_attn_set_variant": None,
            "cgs_conv_v6_set_loader": None}


def _declare(lib):
    for name, argtypes in KERNEL_SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.argtypes = argtypes
        fn.restype = _RESTYPE.get(name, ctypes.c_int)


def has_kernel(name: str) -> bool:
    lib = load_kernels()
    return lib is not None and getattr(lib, name, None) is not None


_runtime = None
_runtime_err = None


def load_runtime():
    """Import the C++ runtime extension module (_cgs_runtime)."""
    global _runtime, _runtime_err
    if _runtime is not None or _runtime_err is not None:
        return _runtime
    import importlib.util
    import sys
    cands = glob.glob(os.path.join(LIB_DIR, "_cgs_runtime*.so"))
    if not cands:
        _runtime_err = "_cgs_runtime not built"
        return None
    try:
        spec = importlib.util.spec_from_file_location("_cgs_runtime", cands[0])
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        sys.modules["_cgs_runtime"] = mod
        _runtime = mod
    except Exception as e:  # pragma: no cover
        _runtime_err = str(e)
    return _runtime


def runtime_error():
    return _runtime_err
