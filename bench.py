#!/usr/bin/env python3
"""Headline benchmark: SDXL 1024x1024, 20-step Euler-ancestral, CFG 8, data-parallel over N GPUs.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W`` (N>1 under torch.distributed.run).
One *step* = one whole-node job of ``batch_per_gpu * N`` images (weak scaling: fixed per-GPU work):
CLIP-L/G prompt encode -> 20 Euler-a steps with cond/uncond batched (UNet batch = 2 x images per GPU)
-> VAE decode -> uint8 -> all-gather to rank 0 (RCCL over xGMI). Weights are random-init SDXL-base
of the exact architecture (no network / checkpoints available); rank 0's weights are broadcast to
every rank (R3). Timed region = exactly K steps bracketed by barrier + device synchronize; the
reported time is the MAX over ranks. Prints one JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


_FAMILY_NAMES = {"sdxl": "SDXL-base", "sd15": "SD1.5", "sd21": "SD2.1", "cascade": "Stable Cascade", "tiny": "tiny test"}


def _labels(args):
    """(metric, data, model) strings for the family actually run: the BASELINE metric string names SDXL
    1024 20-step Euler-a, so it is used only for that config; every other run names what it measured."""
    fam = _FAMILY_NAMES.get(args.family, args.family)
    headline = args.family == "sdxl" and args.res == 1024 and args.sampler_steps == 20 and \
        args.sampler == "euler_ancestral"
    metric = None
    if headline:
        try:
            with open(os.path.join(HERE, "BASELINE.json")) as f:
                metric = json.load(f)["metric"]
        except Exception:
            metric = None
    if metric is None:
        metric = f"images/sec (whole node), {fam} {args.res} {args.sampler_steps}-step {args.sampler}"
    data = f"synthetic prompts, random-init weights (exact {fam} architecture)"
    model = f"{args.family}-base" if args.family == "sdxl" else args.family
    return metric, data, model


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch-per-gpu", type=int, default=8)
    ap.add_argument("--family", default="sdxl")
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--sampler-steps", type=int, default=20)
    ap.add_argument("--sampler", default="euler_ancestral")
    ap.add_argument("--cfg", type=float, default=8.0)
    ap.add_argument("--cpu", action="store_true", help="CPU plumbing run (use with --family tiny)")
    ap.add_argument("--no-graph", action="store_true", help="disable hipGraph capture of the denoiser")
    ap.add_argument("--no-pipeline", dest="pipeline", action="store_false",
                    help="disable the prompt-level multi-stream overlap (job n's VAE decode + gather on a side "
                         "stream while job n+1 samples: dp.run_many); every job still completes inside the "
                         "timed region")
    ap.add_argument("--profile-ops", action="store_true", help="(kept for compatibility; op backends are always reported)")
    ap.add_argument("--latency", action="store_true",
                    help="latency mode: ONE image per step for the whole node; every UNet call split CFG-/token-"
                         "parallel over the N ranks (parallel/latency.py); reports sec/image (strong scaling)")
    ap.add_argument("--via-executor", action="store_true",
                    help="time the product path: a text-to-image workflow JSON through validate_prompt + "
                         "PromptExecutor (CLIPTextEncode x2 -> KSampler -> VAEDecode -> SaveImage PNGs); at N > 1 "
                         "every rank runs it SPMD with the batch split by global image index (sched/spmd.py)")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if args.gpus > 1 and env_world is None:
        # No launcher: become the launcher. This parent never imports torch / touches the GPU; it
        # starts one rank process per GPU (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* like torchrun).
        sys.exit(_spawn_ranks(args.gpus))
    if env_world is not None and int(env_world) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world}; launch {args.gpus} ranks")

    if args.cpu:
        os.environ["CGS_FORCE_CPU"] = "1"
    # MIOpen (only used for convs not yet on the HIP kernel): heuristic solver choice, no
    # exhaustive first-call search on a fresh box.
    os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
    if args.no_graph:
        os.environ["CGS_GRAPHS"] = "0"
    import torch
    from comfy_gen_server_amd.parallel.comm import init_from_env
    comm = init_from_env(backend="gloo" if args.cpu else None)
    assert comm.world == args.gpus, f"communicator has {comm.world} ranks, --gpus {args.gpus}"
    from comfy_gen_server_amd.runtime import device as dm
    if not args.cpu:
        dm.set_device_index(comm.device.index if comm.device.type == "cuda" else comm.local_rank)
    from comfy_gen_server_amd.tools.synth import build_pipeline
    from comfy_gen_server_amd.parallel.dp import DataParallelGenerator, Job
    from comfy_gen_server_amd import ops

    dev = dm.get_torch_device()
    dtype = torch.float32 if args.cpu else torch.bfloat16
    t0 = time.time()
    with torch.inference_mode():
        patcher, clip, vae = build_pipeline(args.family, device=dev, dtype=dtype, seed=1234)
    arena_stats = None
    if not args.cpu:
        # resident weights in the per-GPU HBM slab (runtime/arena.py; on by default on MI355X)
        from comfy_gen_server_amd.runtime import arena
        wa = arena.get(dev)
        if wa is not None:
            for m in (patcher.model, clip.cond_stage_model, vae.first_stage_model):
                wa.place_module(m)
            arena_stats = wa.stats()
    gen = DataParallelGenerator(patcher, clip, vae)
    with torch.inference_mode():
        gen.sync_weights()
    comm.barrier()
    t_build = time.time() - t0

    N = comm.world
    global_batch = args.batch_per_gpu * N
    job = Job(batch=global_batch, steps=args.sampler_steps, cfg=args.cfg, sampler=args.sampler,
              width=args.res, height=args.res)

    def log(msg):
        if comm.rank == 0:
            print(f"[bench {time.time() - t0:7.1f}s] {msg}", file=sys.stderr, flush=True)

    log(f"built pipeline in {t_build:.1f}s")

    if args.via_executor:
        return _bench_executor(args, comm, gen, job, global_batch, t0, t_build, log)
    if args.latency:
        return _bench_latency(args, comm, gen, job, t0, t_build, log)

    def one_step(i):
        j = Job(**{**job.__dict__, "seed": 1000 + i})
        ts = time.perf_counter()
        with torch.inference_mode():
            r = gen.run(j)
        if not args.cpu:
            torch.cuda.synchronize()
        log(f"step {i}: {time.perf_counter() - ts:.2f}s")
        return r

    # pipelined serving at every N: the job broadcast travels on the Gloo control group, so the image
    # gather (side stream) is the only RCCL collective in the loop (dp.run_many docstring)
    if args.pipeline and args.warmup:
        jobs = (Job(**{**job.__dict__, "seed": 1000 + i}) for i in range(args.warmup))
        with torch.inference_mode():
            for i, _ in enumerate(gen.run_many(jobs, pipeline=True)):
                log(f"warmup job {i} done (pipelined)")
    else:
        for i in range(args.warmup):
            one_step(i)
    if not args.cpu:
        torch.cuda.synchronize()
    comm.barrier()
    ops.reset_stats()
    t1 = time.perf_counter()
    if args.pipeline:
        jobs = (Job(**{**job.__dict__, "seed": 1000 + args.warmup + i}) for i in range(args.steps))
        with torch.inference_mode():
            for i, out in enumerate(gen.run_many(jobs, pipeline=True)):
                log(f"job {args.warmup + i} done (pipelined)")
    else:
        for i in range(args.steps):
            out = one_step(args.warmup + i)
    if not args.cpu:
        torch.cuda.synchronize()
    comm.barrier()
    dt = time.perf_counter() - t1
    dt = comm.all_reduce_max(dt)
    ms_per_step = dt * 1000.0 / max(1, args.steps)
    imgs_per_sec = global_batch * args.steps / dt
    if comm.rank == 0:
        metric, data_s, model_s = _labels(args)
        res = {
            "metric": metric,
            "value": round(imgs_per_sec, 4),
            "unit": "images/s",
            "n_gpus": N,
            "ranks": comm.world,
            "backend": comm.backend or "single",
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32" if args.cpu else "bf16",
            "data": data_s,
            "sec_per_image": round(dt / (global_batch * args.steps), 4),
            "sec_per_image_per_gpu": round(dt * N / (global_batch * args.steps), 4),
            "config": {"model": model_s,
                       "global_batch": global_batch, "seq_len": (args.res // 8) ** 2,
                       "resolution": args.res, "sampler_steps": args.sampler_steps, "sampler": args.sampler,
                       "cfg": args.cfg, "unet_batch_per_gpu": 2 * args.batch_per_gpu,
                       "parallelism": f"dp{N}", "pipelined": bool(args.pipeline)},
            "build_s": round(t_build, 1),
            "weight_arena": arena_stats,
        }
        from comfy_gen_server_amd.parallel import dp as _dp
        if _dp.STAGE_TIMES:
            res["stage_seconds"] = {k: [round(x, 3) for x in v] for k, v in _dp.STAGE_TIMES.items()}
        res["op_backends"] = {f"{k[0]}:{k[1]}": v for k, v in sorted(ops.stats().items())}
        from comfy_gen_server_amd.sampling import run_graph as _rg, step_graph as _sg
        res["step_graph"] = dict(_sg.stats)      # capture / replay / capture_failed / ineligible reasons
        res["run_graph"] = dict(_rg.stats)
        print(json.dumps(res), flush=True)
    comm.shutdown()


def _bench_executor(args, comm, gen, job, global_batch, t0, t_build, log):
    """--via-executor: every timed step is one workflow JSON executed by PromptExecutor (rank 0 owns the
    prompt and broadcasts it; SPMD across ranks). The prompt text changes per step, so the CLIP
    encodes run every step (no cross-prompt cache hit), as does the PNG encode + write of SaveImage."""
    import tempfile
    import torch
    from comfy_gen_server_amd import ops
    from comfy_gen_server_amd.graph import registry
    from comfy_gen_server_amd.graph.executor import PromptExecutor
    from comfy_gen_server_amd.graph.validation import validate_prompt
    from comfy_gen_server_amd.sched import spmd
    from comfy_gen_server_amd.tools import synth
    from comfy_gen_server_amd.utils import folder_paths, imageio
    registry.init_nodes(custom_nodes=False)
    synth.register_node()
    synth._PIPELINES[(args.family, 1234)] = (gen.patcher, gen.clip, gen.vae)   # the weights built above
    out_dir = tempfile.mkdtemp(prefix="cgs_bench_out_")
    folder_paths.set_output_directory(out_dir)
    ctx = spmd.SPMD(comm) if comm.world > 1 else None
    ex = PromptExecutor(None, node_hook=ctx)
    imageio.defer_saves(True)

    def step(i):
        wf = synth.text_to_image_workflow(args.family, seed=1000 + i, text=f"{job.prompt}, variation {i}",
                                          negative=job.negative, width=args.res, height=args.res,
                                          batch=global_batch, steps=args.sampler_steps, cfg=args.cfg,
                                          sampler=args.sampler, save_prefix=f"bench{comm.rank}")
        wf = comm.broadcast_object(wf)
        ok, err, outputs, node_errors = validate_prompt(wf)
        assert ok, (err, node_errors)
        if ctx is not None:
            with spmd.activate(ctx):
                ex.execute(wf, f"bench-{i}", {}, outputs)
        else:
            ex.execute(wf, f"bench-{i}", {}, outputs)
        assert ex.success, ex.status_messages[-1:]
        # the PNG encodes of this job run on the CPU pool behind the next job (utils/imageio async
        # saves, as in the server's worker loop); the timed region ends after every file is written
        imageio.take_pending()

    for i in range(args.warmup):
        ts = time.perf_counter()
        step(i)
        log(f"warmup workflow {i}: {time.perf_counter() - ts:.2f}s")
    imageio.flush()
    comm.barrier()
    ops.reset_stats()
    t1 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    imageio.flush()
    if not args.cpu:
        torch.cuda.synchronize()
    comm.barrier()
    dt = comm.all_reduce_max(time.perf_counter() - t1)
    if comm.rank == 0:
        metric, data_s, model_s = _labels(args)
        saved = sum(1 for f in os.listdir(out_dir) if f.endswith(".png"))
        res = {"metric": metric, "value": round(global_batch * args.steps / dt, 4), "unit": "images/s",
               "n_gpus": comm.world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": round(dt * 1000.0 / max(1, args.steps), 2), "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "fp32" if args.cpu else "bf16",
               "data": data_s,
               "path": "workflow JSON -> validate_prompt -> PromptExecutor (SaveImage PNGs included)",
               "pngs_written": saved,
               "config": {"model": model_s,
                          "global_batch": global_batch, "seq_len": (args.res // 8) ** 2, "resolution": args.res,
                          "sampler_steps": args.sampler_steps, "sampler": args.sampler, "cfg": args.cfg,
                          "parallelism": f"dp{comm.world}"},
               "build_s": round(t_build, 1)}
        res["op_backends"] = {f"{k[0]}:{k[1]}": v for k, v in sorted(ops.stats().items())}
        from comfy_gen_server_amd.sampling import run_graph as _rg, step_graph as _sg
        res["step_graph"] = dict(_sg.stats)
        res["run_graph"] = dict(_rg.stats)
        print(json.dumps(res), flush=True)
    comm.shutdown()


def _bench_latency(args, comm, gen, job, t0, t_build, log):
    """--latency: batch 1 per node; rank r evaluates its CFG half / token shard of every UNet call."""
    import torch
    from comfy_gen_server_amd import ops
    from comfy_gen_server_amd.parallel.dp import Job, encode_prompt, generate_local
    from comfy_gen_server_amd.parallel.latency import LatencyParallel
    lat = LatencyParallel(comm)
    patcher = lat.patch(gen.patcher)

    def step(i):
        j = Job(**{**job.__dict__, "seed": 1000 + i, "batch": 1})
        with torch.inference_mode():
            img = generate_local(patcher, gen.clip, gen.vae, j, 0, 1, decode="uint8")
        if not args.cpu:
            torch.cuda.synchronize()
        return img

    for i in range(args.warmup):
        ts = time.perf_counter()
        step(i)
        log(f"warmup image {i}: {time.perf_counter() - ts:.2f}s")
    comm.barrier()
    ops.reset_stats()
    t1 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    comm.barrier()
    dt = comm.all_reduce_max(time.perf_counter() - t1)
    if comm.rank == 0:
        _, data_s, model_s = _labels(args)
        res = {"metric": "sec/image, one image per node (latency mode)", "value": round(dt / max(1, args.steps), 4),
               "unit": "s/image", "n_gpus": comm.world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": round(dt * 1000.0 / max(1, args.steps), 2), "higher_is_better": False,
               "scaling": "strong", "vs_baseline": None, "dtype": "fp32" if args.cpu else "bf16",
               "data": data_s,
               "config": {"model": model_s, "global_batch": 1,
                          "resolution": args.res, "sampler_steps": args.sampler_steps, "sampler": args.sampler,
                          "cfg": args.cfg,
                          "parallelism": f"cfg{lat.G}x{'rows' if lat.spatial_calls else 'token'}{lat.Q}"},
               "unet_calls_on_rank0": lat.calls, "build_s": round(t_build, 1),
               # row-sharded UNet calls (parallel/spatial.py): every layer on 1/Q of the rows per rank
               "spatial_unet_calls": lat.spatial_calls,
               "unet_rows_per_rank": (1.0 / lat.Q) if lat.spatial_calls else 1.0,
               "spatial_stats": None if lat.spatial is None else dict(lat.spatial.stats)}
        res["op_backends"] = {f"{k[0]}:{k[1]}": v for k, v in sorted(ops.stats().items())}
        print(json.dumps(res), flush=True)
    comm.shutdown()


def _spawn_ranks(n: int) -> int:
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    return _watch(procs)


def _watch(procs, poll_s: float = 0.2, grace_s: float = 10.0) -> int:
    """Wait for every rank; on the FIRST non-zero exit terminate the survivors (they would otherwise
    block in a collective until the communicator timeout) and return that exit code."""
    import time as _t
    while True:
        rcs = [p.poll() for p in procs]
        bad = [rc for rc in rcs if rc not in (None, 0)]
        if bad:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            deadline = _t.time() + grace_s
            for p in procs:
                while p.poll() is None and _t.time() < deadline:
                    _t.sleep(0.05)
                if p.poll() is None:
                    p.kill()
                    p.wait()
            print(f"bench.py: rank exited with {bad[0]}; stopped the other ranks", file=sys.stderr, flush=True)
            return abs(bad[0]) or 1
        if all(rc == 0 for rc in rcs):
            return 0
        _t.sleep(poll_s)


if __name__ == "__main__":
    main()
