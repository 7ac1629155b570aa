"""Command-line flags (parity: ``comfy/cli_args.py:36-117``, ``comfy/options.py``).

Every reference flag is accepted so launch scripts keep working. Flags that select a backend this
framework does not have (xformers, DirectML, IPEX, split/quad attention, cudaMallocAsync) are
accepted and ignored with a log line: on MI355X the attention/GEMM/conv kernels are chosen per
shape by ``ops.autotune``. MI355X-specific additions are grouped at the end.

Like the reference, parsing only happens when the server entry point enables it
(``enable_args_parsing``); library imports get the defaults.
"""
from __future__ import annotations

import argparse
import enum
import logging
import os


class LatentPreviewMethod(enum.Enum):
    NoPreviews = "none"
    Auto = "auto"
    Latent2RGB = "latent2rgb"
    TAESD = "taesd"


class EnumAction(argparse.Action):
    """argparse action for Enum choices (values are the enum's .value strings)."""

    def __init__(self, **kwargs):
        enum_type = kwargs.pop("type", None)
        if enum_type is None or not issubclass(enum_type, enum.Enum):
            raise ValueError("type must be an Enum when using EnumAction")
        kwargs.setdefault("choices", tuple(e.value for e in enum_type))
        super().__init__(**kwargs)
        self._enum = enum_type

    def __call__(self, parser, namespace, values, option_string=None):
        setattr(namespace, self.dest, self._enum(values))


# The reference's module-level mutually-exclusive groups by name (``comfy/cli_args.py``: cm_group,
# fp_group, ...); custom nodes import them to add their own flags to the same group.
GROUPS: dict = {}


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="comfy_gen_server_amd: MI355X-native ComfyUI-compatible generation server")
    # network
    p.add_argument("--listen", type=str, default="127.0.0.1", metavar="IP", nargs="?", const="0.0.0.0")
    p.add_argument("--port", type=int, default=8188)
    p.add_argument("--enable-cors-header", type=str, default=None, metavar="ORIGIN", nargs="?", const="*")
    p.add_argument("--max-upload-size", type=float, default=100)
    p.add_argument("--grpc-port", type=int, default=None,
                   help="also serve comfy_request.v1.Comfy + grpc.health.v1.Health over gRPC on this port")
    # paths
    p.add_argument("--extra-model-paths-config", type=str, default=None, metavar="PATH", nargs="+", action="append")
    p.add_argument("--output-directory", type=str, default=None)
    p.add_argument("--temp-directory", type=str, default=None)
    p.add_argument("--input-directory", type=str, default=None)
    p.add_argument("--base-directory", type=str, default=None, help="root for models/, input/, output/, temp/")
    p.add_argument("--auto-launch", action="store_true")
    p.add_argument("--disable-auto-launch", action="store_true")
    p.add_argument("--cuda-device", type=int, default=None, metavar="DEVICE_ID")
    p.add_argument("--gpus", type=int, default=1, metavar="N",
                   help="serve one API from N GPU ranks (rank 0: server + coordinator; sched/cluster.py)")
    p.add_argument("--latency-mode", action="store_true",
                   help="with --gpus N: prompts whose batch is smaller than N run on all ranks with every UNet "
                        "call split CFG-/token-parallel (one image sooner) instead of on one idle rank")
    cm = GROUPS["cm_group"] = p.add_mutually_exclusive_group()
    cm.add_argument("--cuda-malloc", action="store_true")
    cm.add_argument("--disable-cuda-malloc", action="store_true")
    p.add_argument("--dont-upcast-attention", action="store_true")
    # precision
    fp = GROUPS["fp_group"] = p.add_mutually_exclusive_group()
    fp.add_argument("--force-fp32", action="store_true")
    fp.add_argument("--force-fp16", action="store_true")
    fpu = GROUPS["fpunet_group"] = p.add_mutually_exclusive_group()
    fpu.add_argument("--bf16-unet", action="store_true")
    fpu.add_argument("--fp16-unet", action="store_true")
    fpu.add_argument("--fp8_e4m3fn-unet", action="store_true")
    fpu.add_argument("--fp8_e5m2-unet", action="store_true")
    fpv = GROUPS["fpvae_group"] = p.add_mutually_exclusive_group()
    fpv.add_argument("--fp16-vae", action="store_true")
    fpv.add_argument("--fp32-vae", action="store_true")
    fpv.add_argument("--bf16-vae", action="store_true")
    p.add_argument("--cpu-vae", action="store_true")
    fpt = GROUPS["fpte_group"] = p.add_mutually_exclusive_group()
    fpt.add_argument("--fp8_e4m3fn-text-enc", action="store_true")
    fpt.add_argument("--fp8_e5m2-text-enc", action="store_true")
    fpt.add_argument("--fp16-text-enc", action="store_true")
    fpt.add_argument("--fp32-text-enc", action="store_true")
    # backends (accepted for compatibility)
    p.add_argument("--directml", type=int, nargs="?", metavar="DIRECTML_DEVICE", const=-1)
    p.add_argument("--disable-ipex-optimize", action="store_true")
    p.add_argument("--preview-method", type=LatentPreviewMethod, default=LatentPreviewMethod.NoPreviews,
                   action=EnumAction)
    attn = GROUPS["attn_group"] = p.add_mutually_exclusive_group()
    attn.add_argument("--use-split-cross-attention", action="store_true")
    attn.add_argument("--use-quad-cross-attention", action="store_true")
    attn.add_argument("--use-pytorch-cross-attention", action="store_true")
    p.add_argument("--disable-xformers", action="store_true")
    # VRAM
    vram = GROUPS["vram_group"] = p.add_mutually_exclusive_group()
    vram.add_argument("--gpu-only", action="store_true")
    vram.add_argument("--highvram", action="store_true")
    vram.add_argument("--normalvram", action="store_true")
    vram.add_argument("--lowvram", action="store_true")
    vram.add_argument("--novram", action="store_true")
    vram.add_argument("--cpu", action="store_true")
    p.add_argument("--disable-smart-memory", action="store_true")
    # misc
    p.add_argument("--deterministic", action="store_true")
    p.add_argument("--dont-print-server", action="store_true")
    p.add_argument("--quick-test-for-ci", action="store_true")
    p.add_argument("--windows-standalone-build", action="store_true")
    p.add_argument("--disable-metadata", action="store_true")
    p.add_argument("--multi-user", action="store_true")
    p.add_argument("--verbose", action="store_true")
    # MI355X-native additions
    p.add_argument("--no-autotune", action="store_true", help="always use the default HIP kernel per op")
    p.add_argument("--tune-file", type=str, default=None, help="persist per-shape kernel choices (JSON)")
    p.add_argument("--hbm-budget-gb", type=float, default=None, help="residency budget per GPU (default 90%%)")
    p.add_argument("--hip-graphs", action="store_true", help="capture denoiser steps in hipGraphs")
    p.add_argument("--weight-arena-gb", type=float, default=None,
                   help="place resident model weights in one HBM slab of this size per GPU (runtime/arena.py)")
    p.add_argument("--alloc-expandable", action="store_true",
                   help="caching allocator with expandable segments (runtime/alloc_policy.py)")
    p.add_argument("--queue-journal", type=str, default=None, help="JSONL journal: queued prompts survive restarts")
    p.add_argument("--profile-dir", type=str, default=None,
                   help="write a Perfetto/Chrome trace (torch.profiler, HIP kernels + node/step ranges) per prompt")
    p.add_argument("--log-json", action="store_true", help="structured JSON log lines")
    p.add_argument("--disable-custom-nodes", action="store_true")
    p.add_argument("--custom-nodes-directory", type=str, default=None, nargs="+", action="append")
    return p


parser = build_parser()
_enabled = False
args = parser.parse_args([])


def enable_args_parsing(enable: bool = True):
    global _enabled
    _enabled = enable


def parse(argv=None):
    """Parse ``argv`` (server entry point only) into the module-level ``args``."""
    global args
    args = parser.parse_args(argv)
    if args.windows_standalone_build:
        args.auto_launch = True
    if args.disable_auto_launch:
        args.auto_launch = False
    logging.basicConfig(format="%(message)s", level=logging.DEBUG if args.verbose else logging.INFO)
    if getattr(args, "log_json", False):
        from .utils.telemetry import use_json_logs
        use_json_logs(logging.DEBUG if args.verbose else logging.INFO)
    if getattr(args, "profile_dir", None):
        os.environ["CGS_PROFILE_DIR"] = args.profile_dir
    for flag in ("directml", "use_split_cross_attention", "use_quad_cross_attention", "disable_xformers",
                 "disable_ipex_optimize"):
        if getattr(args, flag, None):
            logging.info("--%s accepted for compatibility; ignored on MI355X (per-shape autotuned kernels)",
                         flag.replace("_", "-"))
    return args
