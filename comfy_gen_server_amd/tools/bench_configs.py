"""Single-GPU measurements of the other BASELINE.json configs (the headline DP throughput number is
``bench.py``): random-init weights of the exact architectures, synthetic prompts, bf16.

  sdxl_b1        SDXL-base 1024², 20-step Euler-a, batch 1 (latency)
  sdxl_cn_lora   SDXL + ControlNet (SDXL-size cldm, canny-like hint) + LoRA (rank 16 on every attention
                 / FF projection, patched into the weights by ModelPatcher), 1024², 20 steps, batch 1 and 8
  cascade        Stable Cascade Stage C (3.6 B, 20 steps, 24² latent) -> Stage B (1.6 B, 10 steps,
                 256² latent) -> Stage A decode, 1024², batch 1 and 4

    python -m comfy_gen_server_amd.tools.bench_configs [--which all|sdxl_b1|sdxl_cn_lora|cascade] [--reps 2]

Prints one JSON line per measurement: {"config", "batch", "sec_per_job", "sec_per_image", ...}.
"""
from __future__ import annotations

import argparse
import os
import copy
import json
import sys
import time

import torch


def _timed(fn, reps):
    fn()                                   # warmup (kernel tuning, graph capture)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return min(ts), sum(ts) / len(ts)


def _emit(config, batch, best, mean, **extra):
    print(json.dumps({"config": config, "batch": batch, "sec_per_job": round(best, 3),
                      "sec_per_job_mean": round(mean, 3), "sec_per_image": round(best / batch, 4),
                      "images_per_sec": round(batch / best, 3), "dtype": "bf16",
                      "data": "synthetic prompts, random-init weights", **extra}), flush=True)


def bench_sdxl_b1(reps):
    from ..parallel.dp import DataParallelGenerator, Job
    from ..tools.synth import build_pipeline
    dev = torch.device("cuda")
    with torch.inference_mode():
        patcher, clip, vae = build_pipeline("sdxl", device=dev, dtype=torch.bfloat16, seed=1)
    gen = DataParallelGenerator(patcher, clip, vae)
    job = Job(batch=1, steps=20, cfg=8.0, sampler="euler_ancestral")

    def run():
        with torch.inference_mode():
            gen.run(job)
    best, mean = _timed(run, reps)
    _emit("sdxl_b1", 1, best, mean, steps=20, resolution=1024)
    return patcher, clip, vae


def _aten_table(run, top=25):
    """Which ATen (non-native) device ops a run launches, with the Python line that issued them
    (CGS_TORCH_PROFILE=1): the glue the op layer has not absorbed yet."""
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        run()
        torch.cuda.synchronize()
    rows = prof.key_averages(group_by_stack_n=4)
    rows = [r for r in rows if r.key.startswith("aten::") and r.device_time_total > 0]
    rows.sort(key=lambda r: -r.device_time_total)
    for r in rows[:top]:
        stack = " <- ".join(f for f in (r.stack or []) if "comfy_gen_server_amd" in f)[:400]
        print(f"ATEN {r.key:34s} calls={r.count:6d} dev_ms={r.device_time_total / 1e3:8.2f}  {stack}", flush=True)


def bench_sdxl_cn_lora(reps, pipe=None):
    from ..graph import registry
    from ..models.cldm import ControlNet as CNModel
    from ..models.layers import init_random_fast_
    from ..parallel.dp import encode_prompt
    from ..runtime import controlnet as rcn
    from ..runtime.sd import load_lora_for_models
    from ..sampling import sample as S
    from ..tools.synth import SDXL_UNET, build_pipeline, random_lora
    registry.init_nodes(custom_nodes=False)
    NM = registry.NODE_CLASS_MAPPINGS
    dev = torch.device("cuda")
    with torch.inference_mode():
        patcher, clip, vae = pipe or build_pipeline("sdxl", device=dev, dtype=torch.bfloat16, seed=1)
        lora = random_lora(patcher, rank=16, seed=3,
                           prefix_filter=("attn1.to_q", "attn1.to_k", "attn1.to_v", "attn1.to_out.0", "attn2.to_q",
                                          "attn2.to_out.0", "ff.net.2"))
        lpatcher, lclip = load_lora_for_models(patcher, clip, lora, 0.8, 0.0)
        cfg = copy.deepcopy(SDXL_UNET)
        cfg.pop("out_channels", None)
        cfg.update(num_heads=-1, num_head_channels=64)          # the SDXL family's unet_extra_config
        with torch.device("meta"):
            cm = CNModel(hint_channels=3, dtype=torch.bfloat16, device=torch.device("meta"), **cfg)
        cm.to_empty(device=dev)
        init_random_fast_(cm, seed=7)
        cnet = rcn.ControlNet(cm, load_device=dev)
        n_lora = sum(1 for k in lora if k.endswith("lora_up.weight"))
        pos = encode_prompt(lclip, "a modern house, architectural photo", 1024, 1024)
        neg = encode_prompt(lclip, "blurry", 1024, 1024)
        edges = (torch.rand(1, 1024, 1024, 1) > 0.9).float().expand(1, 1024, 1024, 3).contiguous()   # canny-like
        pos_c, neg_c = NM["ControlNetApplyAdvanced"]().apply_controlnet(pos, neg, cnet, edges, 1.0, 0.0, 1.0)

    for batch in (1, 8):
        latent = torch.zeros([batch, 4, 128, 128])
        noise = S.prepare_noise(latent, 11)

        def run():
            with torch.inference_mode():
                s = S.sample(lpatcher, noise, 20, 8.0, "euler_ancestral", "normal", pos_c, neg_c, latent,
                             denoise=1.0, seed=11)
                vae.decode(s)
        best, mean = _timed(run, reps)
        _emit("sdxl_cn_lora", batch, best, mean, steps=20, resolution=1024, lora_layers=n_lora, lora_rank=16,
              controlnet="sdxl-size cldm (random init)")


def bench_cascade(reps, ab=None):
    from ..graph import registry
    from ..models.cascade import StageA
    from ..models.layers import init_random_fast_
    from ..parallel.dp import encode_prompt
    from ..runtime import families
    from ..runtime.patcher import ModelPatcher
    from ..runtime.sd import CLIP, VAE
    registry.init_nodes(custom_nodes=False)
    NM = registry.NODE_CLASS_MAPPINGS
    dev = torch.device("cuda")
    dt = torch.bfloat16

    def stage(fam_cls, seed):
        mc = fam_cls(dict(fam_cls.unet_config))
        mc.set_inference_dtype(dt, None)
        with torch.device("meta"):
            model = mc.get_model({}, "", device=torch.device("meta"))
        model.to_empty(device=dev)
        model.model_sampling = model.model_sampling.__class__(mc)
        model.model_sampling.to(dev)
        init_random_fast_(model.diffusion_model, seed=seed)
        return mc, ModelPatcher(model, load_device=dev, offload_device=dev)

    with torch.inference_mode():
        mc_c, pc = stage(families.Stable_Cascade_C, 21)
        _, pb = stage(families.Stable_Cascade_B, 22)
        clip = CLIP(mc_c.clip_target(), dtype=dt, device=dev)
        clip.cond_stage_model.to(dev)
        init_random_fast_(clip.cond_stage_model, seed=23)
        clip.patcher.offload_device = dev
        sa = StageA()
        sa_sd = {k: v for k, v in sa.state_dict().items()}
        vae = VAE(sd=sa_sd, device=dev, dtype=dt)
        vae.first_stage_model.to(dev)
        init_random_fast_(vae.first_stage_model, seed=24)
        vae.patcher.offload_device = dev
        pos = encode_prompt(clip, "a red fox in the snow, photograph", 1024, 1024)
        neg = encode_prompt(clip, "", 1024, 1024)
    n_c = sum(p.numel() for p in pc.model.diffusion_model.parameters()) / 1e9
    n_b = sum(p.numel() for p in pb.model.diffusion_model.parameters()) / 1e9

    if ab:
        return _cascade_ab(ab, reps, pc, pb, vae, pos, neg, NM, batch=int(os.environ.get("CGS_AB_BATCH", "1")))
    for batch in (1, 4):
        def run():
            with torch.inference_mode():
                lat_c, lat_b = NM["StableCascade_EmptyLatentImage"]().generate(1024, 1024, 42, batch)
                out_c = NM["KSampler"]().sample(pc, 5, 20, 4.0, "euler_ancestral", "simple", pos, neg, lat_c, 1.0)[0]
                cond_b = NM["StableCascade_StageB_Conditioning"]().set_prior(pos, out_c)[0]
                neg_b = NM["StableCascade_StageB_Conditioning"]().set_prior(neg, out_c)[0]
                out_b = NM["KSampler"]().sample(pb, 5, 10, 1.1, "euler_ancestral", "simple", cond_b, neg_b, lat_b,
                                                1.0)[0]
                NM["VAEDecode"]().decode(vae, out_b)
        best, mean = _timed(run, reps)
        if os.environ.get("CGS_TORCH_PROFILE") == "1" and batch == 1:
            _aten_table(run)
        _emit("cascade_c_b_a", batch, best, mean, steps_c=20, steps_b=10, resolution=1024,
              params_c_b=round(n_c, 3), params_b_b=round(n_b, 3))


def _native_knobs():
    """Push the env values of the native A/B knobs (tools/ab_bench.py ``_NATIVE_KNOBS``) into the library."""
    from .ab_bench import _NATIVE_KNOBS
    from .. import _native
    lib = _native.load_kernels()
    for k, (fn, dflt) in _NATIVE_KNOBS.items():
        if lib is not None and _native.has_kernel(fn):
            getattr(lib, fn)(int(os.environ.get(k, dflt)))


def _cascade_ab(cfgs, rounds, pc, pb, vae, pos, neg, NM, batch=1):
    """Cascade jobs (``batch`` images) alternating between env configurations (``name:ENV=V,...``) in one
    process: captured graph plans are dropped on every switch and re-captured in an untimed job."""
    import statistics

    def drop(p):
        m = p.model
        for k in ("_step_graph_plans", "_run_graph_plans"):
            m.__dict__.pop(k, None)
        r = m.__dict__.get("_graph_runner")
        if r is not None:
            r.reset()

    def run():
        with torch.inference_mode():
            lat_c, lat_b = NM["StableCascade_EmptyLatentImage"]().generate(1024, 1024, 42, batch)
            out_c = NM["KSampler"]().sample(pc, 5, 20, 4.0, "euler_ancestral", "simple", pos, neg, lat_c, 1.0)[0]
            cond_b = NM["StableCascade_StageB_Conditioning"]().set_prior(pos, out_c)[0]
            neg_b = NM["StableCascade_StageB_Conditioning"]().set_prior(neg, out_c)[0]
            out_b = NM["KSampler"]().sample(pb, 5, 10, 1.1, "euler_ancestral", "simple", cond_b, neg_b, lat_b, 1.0)[0]
            NM["VAEDecode"]().decode(vae, out_b)
        torch.cuda.synchronize()

    parsed = []
    for c in cfgs:
        name, _, rest = c.partition(":")
        parsed.append((name, dict(kv.split("=", 1) for kv in rest.split(",") if kv)))
    keys = {k for _, e in parsed for k in e}
    times = {n: [] for n, _ in parsed}
    for r in range(rounds + 1):
        for name, env in parsed:
            for k in keys:
                os.environ.pop(k, None)
            os.environ.update(env)
            _native_knobs()
            drop(pc)
            drop(pb)
            run()                                   # untimed: autotune keys, graph capture
            if r:
                t = time.perf_counter()
                run()
                times[name].append(time.perf_counter() - t)
                print(f"[cascade-ab] round {r} {name}: {times[name][-1]:.3f}s", file=sys.stderr, flush=True)
    print(json.dumps({n: {"median_s": round(statistics.median(v), 4), "runs": [round(x, 4) for x in v]}
                      for n, v in times.items()}), flush=True)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--which", default="all")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--ab", action="append", default=None,
                    help="cascade only: name:ENV=V,... configurations alternated per batch-1 job (--reps rounds)")
    a = ap.parse_args(argv)
    if not torch.cuda.is_available():
        print("needs a GPU", file=sys.stderr)
        return 2
    pipe = None
    if a.which in ("all", "sdxl_b1"):
        pipe = bench_sdxl_b1(a.reps)
    if a.which in ("all", "sdxl_cn_lora"):
        bench_sdxl_cn_lora(a.reps, pipe)
    del pipe
    torch.cuda.empty_cache()
    if a.which in ("all", "cascade"):
        bench_cascade(a.reps, a.ab)
    return 0


if __name__ == "__main__":
    sys.exit(main())
