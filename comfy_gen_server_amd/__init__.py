"""comfy_gen_server_amd — an MI355X-native diffusion node-graph inference engine.

Capability parity target: comfy-creator/Comfy-Gen-Server (a headless ComfyUI fork).
The Python package name uses underscores because Python identifiers cannot contain
hyphens; the project is referred to as ``comfy-gen-server_amd``.

Layer map:
  api/        HTTP + WebSocket prompt server, users/settings, gRPC-style JSON service
  graph/      node protocol, registry, validator, caching executor, prompt queue
  nodes/      core + extra node library
  sampling/   schedulers, k-diffusion samplers, CFG guider, cond batching
  runtime/    device/residency manager, safetensors loader, detection, model patcher, LoRA
  models/     UNet (SD1/2/XL), VAE, CLIP, ControlNet, Stable Cascade, TAESD, upscalers
  ops/        op layer: HIP/CDNA4 kernels on the GPU, fp32 torch reference on the CPU
  parallel/   one-process-per-GPU data parallel over RCCL/xGMI
  csrc/       HIP kernels (gfx950) + C++ runtime (safetensors, BPE, BLAKE3, job queue)
"""

__version__ = "0.1.0"
