"""A/B the headline job under two (or more) runtime configurations in ONE process on ONE GPU.

Box-to-box and run-to-run spread (a few %) is larger than most single kernel changes, so
comparisons are made here: the pipeline is built once, then jobs alternate between the
configurations (env flags set before each job; captured graph plans dropped on every switch and
re-captured in an untimed job), and the median wall time per configuration is reported.

python -m comfy_gen_server_amd.tools.ab_bench --cfg "base:" --cfg "noskip:CGS_SKIPCAT=0" [--rounds 3]

``CGS_LIB=<path>`` in a configuration runs it on another build of libcgs_kernels.so (e.g. the previous
commit's, ``tools/build_rev_lib.sh HEAD``): the ops fetch the library handle per call, so the switch is a
handle swap inside the same process.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import time

import torch


# process-wide kernel knobs that live in the native library (set through its setters, not read from the
# environment at launch): name -> (setter, default)
_NATIVE_KNOBS = {"CGS_TILE_GROUP": ("cgs_set_tile_group", 4), "CGS_CONV_TILE_GROUP": ("cgs_conv_set_tile_group", 8),
                 "CGS_DW_PX": ("cgs_dwconv_set_px", 4), "CGS_ATTN_KV2_ROWS": ("cgs_attn_set_kv2_rows", 0),
                 "CGS_GRN_ROWS": ("cgs_grn_set_rows", 1), "CGS_GN_BLOCKS": ("cgs_gn_set_blocks", 2048)}


_LIBS: dict = {}


def _use_lib(path):
    """Make `path` (None: the in-tree build) the kernel library every op launches from."""
    from .. import _native
    if "" not in _LIBS:
        _LIBS[""] = _native.load_kernels()
    key = os.path.abspath(path) if path else ""
    if key not in _LIBS:
        import ctypes
        lib = ctypes.CDLL(key, mode=ctypes.RTLD_LOCAL)
        _native._declare(lib)
        _LIBS[key] = lib
    _native._kernels = _LIBS[key]


def _apply(env: dict, saved: dict):
    for k in saved:
        if saved[k] is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = saved[k]
    for k, v in env.items():
        os.environ[k] = v
    from .. import _native
    _use_lib(os.environ.get("CGS_LIB") or None)
    lib = _native.load_kernels()
    for k, (fn, dflt) in _NATIVE_KNOBS.items():
        if lib is not None and _native.has_kernel(fn):
            getattr(lib, fn)(int(os.environ.get(k, dflt)))


def _drop_plans(patcher):
    m = patcher.model
    m.__dict__.pop("_step_graph_plans", None)
    r = m.__dict__.get("_graph_runner")
    if r is not None:
        r.reset()


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", action="append", required=True, help="name:ENV=VAL,ENV2=VAL")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--jobs", type=int, default=1,
                    help="jobs per timed sample through DataParallelGenerator.run_many (CGS_DP_PIPELINE in a "
                         "--cfg selects the pipelined form); the reported time is per job")
    args = ap.parse_args(argv)
    cfgs = []
    for c in args.cfg:
        name, _, rest = c.partition(":")
        env = dict(kv.split("=", 1) for kv in rest.split(",") if kv)
        cfgs.append((name, env))
    keys = {k for _, env in cfgs for k in env}
    saved = {k: os.environ.get(k) for k in keys}
    from comfy_gen_server_amd.tools.synth import build_pipeline
    from comfy_gen_server_amd.parallel.dp import DataParallelGenerator, Job
    dev = torch.device("cuda", 0)
    with torch.inference_mode():
        patcher, clip, vae = build_pipeline("sdxl", device=dev, dtype=torch.bfloat16, seed=1234)
    gen = DataParallelGenerator(patcher, clip, vae)
    times = {n: [] for n, _ in cfgs}

    def job(seed):
        t = time.perf_counter()
        with torch.inference_mode():
            if args.jobs == 1:
                gen.run(Job(batch=args.batch, steps=args.steps, width=args.res, height=args.res, seed=seed))
            else:
                jobs = (Job(batch=args.batch, steps=args.steps, width=args.res, height=args.res, seed=seed + i)
                        for i in range(args.jobs))
                for _ in gen.run_many(jobs):
                    pass
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / args.jobs
    seed = 0
    for r in range(args.rounds + 1):
        for name, env in cfgs:
            _apply(env, saved)
            _drop_plans(patcher)
            job(seed)                      # untimed: autotune keys, graph capture
            seed += 1
            if r > 0:                      # round 0 is warmup only
                times[name].append(job(seed))
                seed += 1
                print(f"[ab] round {r} {name}: {times[name][-1]:.3f}s", flush=True)
    res = {n: {"median_s": statistics.median(v), "min_s": min(v), "runs": [round(x, 4) for x in v]}
           for n, v in times.items()}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
