"""Op layer: the compute backend of every model in ``models/``.

Each op has two implementations:
  * ``hip``   — hand-written gfx950 kernels from ``csrc/kernels`` (bf16 activations, fp32 accumulate,
                NHWC layout for image tensors). Used for every tensor on a ROCm device.
  * ``torch`` — a plain PyTorch fp32 reference used on the CPU (tests, plumbing slice) and as the
                numerics oracle for the kernel tests.

Reference call sites this replaces: ``comfy/ops.py:39-163`` (casting ops),
``comfy/ldm/modules/attention.py:88-383`` (attention backends: basic / sub-quad / split /
xformers / SDPA) — on MI355X all of them collapse to one LDS-tiled MFMA flash-attention kernel.
"""
from . import dispatch  # noqa: F401
from .dispatch import (  # noqa: F401
    backend_for, set_backend_override, native_required, NativeMissingError, stats, reset_stats, torch_reference,
)
from .core import (  # noqa: F401
    linear, linear_geglu, attention, attention_lse, attention_kv2, attention_bias, group_norm, layer_norm, conv2d,
    conv_transpose2d, conv_transpose_phase_weights, silu, gelu,
    upsample_nearest2x, timestep_embedding, cfg_combine, euler_step, depthwise_conv2d_nhwc,
    depthwise_conv2d_nhwc_lnstats,
    interpolate, fused_bias_act, channel_affine_nhwc, channel_affine_layernorm_nhwc, upfirdn2d, upfirdn2d_reference, vq_nearest, grn_nhwc,
    grn_fold_weight, softmax_rows,
    attention_with_probs, philox_randn, euler_ancestral_philox, brownian_increment, step_param, sampler_step_dev,
    step_advance, vae_out_u8, region_accumulate, region_normalize, clip_embed, pooled_gather,
    layernorm_stats, layernorm_stats_for, lnfold_weights, linear_lnfold, lnfold_available, fourier_filter, tome_match,
    rng_key_scope,
)
