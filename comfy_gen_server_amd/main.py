"""Server bootstrap: flags -> paths/devices -> nodes -> HTTP/WS server + prompt worker thread.

Parity: ``main.py:1-258`` (C06, C11): prestartup scripts of custom nodes, extra model paths,
``prompt_worker`` (blocking queue get, execute, history + status, end-of-prompt ``executing``
sentinel, ``/free`` flags, periodic model cleanup + GC at most every 10 s), ``hijack_progress``
(progress events + binary preview frames + interrupt check on every sampler tick), temp cleanup,
and the asyncio loop running the server and its publish loop.

MI355X specifics: ``--gpus N`` serves the whole node from one API (``sched/cluster.py``: rank 0 runs the
server and a coordinator; independent prompts go to idle ranks, a prompt's image batch is split over
all ranks), or one server process per GPU (``--cuda-device`` / LOCAL_RANK) behind a balancer; the
per-shape kernel autotuner (``--no-autotune``, ``--tune-file``) and the HBM residency budget.

Run: ``python -m comfy_gen_server_amd.main --listen 0.0.0.0 --port 8188`` (or ``python main.py``).
"""
from __future__ import annotations

import asyncio
import copy
import functools
import gc
import itertools
import logging
import os
import queue as _queue
import shutil
import threading
import time

from . import cli_args


def apply_args(args):
    """Push parsed flags into the runtime modules (env first: some are read at first use)."""
    if args.cuda_device is not None:
        os.environ["CGS_DEVICE"] = str(args.cuda_device)
    if args.no_autotune:
        os.environ["CGS_AUTOTUNE"] = "0"
    if args.tune_file:
        os.environ["CGS_TUNE_FILE"] = args.tune_file
    if args.hbm_budget_gb:
        os.environ["CGS_HBM_BUDGET_GB"] = str(args.hbm_budget_gb)
    if getattr(args, "weight_arena_gb", None) is not None:
        os.environ["CGS_WEIGHT_ARENA_GB"] = str(args.weight_arena_gb)
    if args.hip_graphs:
        os.environ["CGS_GRAPHS"] = "1"
    if args.deterministic:
        os.environ["CGS_AUTOTUNE"] = "0"   # fixed kernel choice -> reproducible reductions
    from .runtime import device as dm
    from .utils import folder_paths

    if os.environ.get("CGS_REGISTER_TINY") == "1":     # tests: the tiny synthetic family's checkpoints load
        from .tools.synth import register_tiny_family
        register_tiny_family()
    from .nodes import helpers as NH
    pm = getattr(args, "preview_method", None)
    NH.set_flags(preview_method=getattr(pm, "value", pm) or "none",
                 disable_metadata=bool(getattr(args, "disable_metadata", False)))
    if args.cpu:
        dm.set_cpu_mode(True)
    elif args.cuda_device is not None:
        dm.set_device_index(args.cuda_device)
    dm.configure(force_fp32=args.force_fp32, force_fp16=args.force_fp16, bf16_unet=args.bf16_unet,
                 fp16_unet=args.fp16_unet, fp8_e4m3fn_unet=args.fp8_e4m3fn_unet,
                 fp8_e5m2_unet=args.fp8_e5m2_unet, fp32_vae=args.fp32_vae, fp16_vae=args.fp16_vae,
                 bf16_vae=args.bf16_vae, cpu_vae=args.cpu_vae, fp32_text_enc=args.fp32_text_enc,
                 fp16_text_enc=args.fp16_text_enc, disable_smart_memory=args.disable_smart_memory)
    if args.base_directory:
        folder_paths.set_base_path(args.base_directory)
    if args.output_directory:
        folder_paths.set_output_directory(os.path.abspath(args.output_directory))
    if args.temp_directory:
        folder_paths.set_temp_directory(os.path.join(os.path.abspath(args.temp_directory), "temp"))
    if args.input_directory:
        folder_paths.set_input_directory(os.path.abspath(args.input_directory))
    # output/ is also a model search root for checkpoints / clip / vae written by the save nodes
    folder_paths.add_model_folder_path("checkpoints", os.path.join(folder_paths.get_output_directory(), "checkpoints"))
    folder_paths.add_model_folder_path("clip", os.path.join(folder_paths.get_output_directory(), "clip"))
    folder_paths.add_model_folder_path("vae", os.path.join(folder_paths.get_output_directory(), "vae"))
    if args.extra_model_paths_config:
        for group in args.extra_model_paths_config:
            for cfg in group:
                folder_paths.load_extra_path_config(cfg)
    else:
        default = os.path.join(os.getcwd(), "extra_model_paths.yaml")
        if os.path.isfile(default):
            folder_paths.load_extra_path_config(default)


def cleanup_temp():
    from .utils import folder_paths
    temp_dir = folder_paths.get_temp_directory()
    if os.path.exists(temp_dir):
        shutil.rmtree(temp_dir, ignore_errors=True)


def hijack_progress(server):
    """Every ProgressBar update -> WS 'progress' (+ preview frame); interrupt checked per tick."""
    from .api.server import BinaryEventTypes
    from .runtime import device as dm
    from .utils import progress

    def hook(value, total, preview_image):
        dm.throw_exception_if_processing_interrupted()
        progress_ = {"value": value, "max": total, "prompt_id": getattr(server, "last_prompt_id", None),
                     "node": server.last_node_id}
        server.send_sync("progress", progress_, server.client_id)
        if preview_image is not None:
            server.send_sync(BinaryEventTypes.UNENCODED_PREVIEW_IMAGE, preview_image, server.client_id)

    progress.set_progress_bar_global_hook(hook)


def _finish_prompt(q, server, item_id, prompt_id, outputs_ui, success, messages, t0, client_id, save_errors):
    if save_errors:
        success = False
        messages = messages + [("execution_error", {"prompt_id": prompt_id, "node_id": None,
                                                    "exception_message": "; ".join(save_errors),
                                                    "exception_type": "ImageSaveError", "traceback": []})]
    q.task_done(item_id, outputs_ui,
                status=q.ExecutionStatus(status_str="success" if success else "error",
                                         completed=success, messages=messages))
    if client_id is not None:
        server.send_sync("executing", {"node": None, "prompt_id": prompt_id}, client_id)
    dt = time.perf_counter() - t0
    server.metrics["prompts_total"] += 1
    server.metrics["execution_seconds_total"] += dt
    if not success:
        server.metrics["prompts_failed"] += 1
    logging.info("Prompt executed in %.2f seconds", dt)


class _OrderedFinisher:
    """One thread completes prompts in submission order: it waits for a prompt's PNG encodes, then
    reports it (``task_done`` + the end-of-prompt ``executing`` sentinel + metrics). A single consumer
    keeps completions ordered and the metrics single-writer; ``task_done`` runs even when the encode
    wait raises, so no prompt stays in ``currently_running``."""

    def __init__(self):
        self._q: _queue.Queue = _queue.Queue()
        self._t = threading.Thread(target=self._loop, name="prompt-finisher", daemon=True)
        self._t.start()

    def submit(self, done, futs):
        self._q.put((done, futs))

    def drain(self, timeout: float | None = None):
        """Block until every submitted completion has run (tests, shutdown)."""
        t0 = time.perf_counter()
        while self._q.unfinished_tasks:
            if timeout is not None and time.perf_counter() - t0 > timeout:
                return False
            time.sleep(0.005)
        return True

    def _loop(self):
        from .utils import imageio
        while True:
            done, futs = self._q.get()
            errs = []
            try:
                try:
                    errs = imageio.wait_futures(futs) if futs else []
                except Exception as ex:     # noqa: BLE001 - a failed wait is a save error, not a lost prompt
                    errs = [f"{type(ex).__name__}: {ex}"]
                finally:
                    done(errs)
            except Exception:               # noqa: BLE001
                logging.exception("prompt completion failed")
            finally:
                self._q.task_done()


def prompt_worker(q, server, stop_event: threading.Event | None = None, gc_interval: float = 10.0,
                  finisher: _OrderedFinisher | None = None):
    """Blocking worker loop (reference ``main.py:93-146``)."""
    from .graph.executor import PromptExecutor
    from .runtime import device as dm
    from .utils import imageio, telemetry

    e = PromptExecutor(server)
    imageio.defer_saves(True)
    fin = finisher if finisher is not None else _OrderedFinisher()
    last_gc = time.perf_counter()
    need_gc = False
    timeout = 1000.0
    while stop_event is None or not stop_event.is_set():
        item = q.get(timeout=min(timeout, 1.0) if stop_event is not None else timeout)
        if item is not None:
            item, item_id = item
            t0 = time.perf_counter()
            prompt_id = item[1]
            server.last_prompt_id = prompt_id
            with telemetry.maybe_profile(prompt_id):
                e.execute(item[2], prompt_id, item[3], item[4])
            need_gc = True
            # the prompt's PNG encodes (utils/imageio async saves) finish behind the next prompt; the
            # prompt is reported complete once its files are on disk. The next execute() rewrites
            # e.outputs_ui in place, so the finisher gets a snapshot of this prompt's outputs.
            futs = imageio.take_pending()
            done = functools.partial(_finish_prompt, q, server, item_id, prompt_id, copy.deepcopy(e.outputs_ui),
                                     e.success, list(e.status_messages), t0, server.client_id)
            fin.submit(done, futs)

        flags = q.get_flags()
        free_memory = flags.get("free_memory", False)
        if flags.get("unload_models", free_memory):
            dm.unload_all_models()
            need_gc = True
            last_gc = 0.0
        if free_memory:
            e.reset()
            need_gc = True
            last_gc = 0.0
        if need_gc and time.perf_counter() - last_gc > gc_interval:
            dm.cleanup_models()
            gc.collect()
            dm.soft_empty_cache()
            last_gc = time.perf_counter()
            need_gc = False


async def run(server, address="", port=8188, verbose=True, call_on_start=None):
    await asyncio.gather(server.start(address, port, verbose, call_on_start), server.publish_loop())


def build_server(args, loop):
    """Create server + queue, load nodes, register routes (no network I/O yet)."""
    from .api.server import PromptServer
    from .graph import registry
    from .graph.queue import PromptQueue

    server = PromptServer(loop, enable_cors_header=args.enable_cors_header,
                          max_upload_size_mb=args.max_upload_size, multi_user=args.multi_user)
    q = PromptQueue(server, journal_path=args.queue_journal)
    custom_dirs = None
    if args.custom_nodes_directory:
        custom_dirs = list(itertools.chain.from_iterable(args.custom_nodes_directory))
    registry.init_nodes(custom_nodes=not args.disable_custom_nodes, custom_dirs=custom_dirs)
    server.add_routes()
    hijack_progress(server)
    return server, q


def _cluster_start(args, argv):
    """``--gpus N``: rank 0 starts ranks 1..N-1 (same flags) before any device use, then every rank
    joins the process group (RCCL + Gloo control; Gloo only with ``--cpu``)."""
    from .sched import cluster
    role = os.environ.get("CGS_SCHED_ROLE", "coordinator")
    listener = procs = None
    if role != "worker":
        import sys as _sys
        listener, procs = cluster.launch(args.gpus, list(argv) if argv is not None else _sys.argv[1:])
    from .parallel.comm import init_from_env
    # a replacement rank (sched/cluster.py respawn) joins the process group at the next re-rendezvous
    join = os.environ.get("CGS_SCHED_RESPAWN") != "1"
    comm = init_from_env(backend="gloo" if args.cpu else None, join=join)
    return role, comm, listener, procs


def _worker_rank_main(args, comm):
    from .graph import registry
    from .sched import cluster
    apply_args(args)
    registry.init_nodes(custom_nodes=not args.disable_custom_nodes,
                        custom_dirs=list(itertools.chain.from_iterable(args.custom_nodes_directory))
                        if args.custom_nodes_directory else None)
    addr, key = cluster.worker_address()
    cluster.worker_main(comm, addr, key, respawned=os.environ.get("CGS_SCHED_RESPAWN") == "1")
    comm.shutdown()
    return 0


def main(argv=None):
    cli_args.enable_args_parsing()
    args = cli_args.parse(argv)
    cluster_state = None
    if getattr(args, "gpus", 1) > 1:
        cluster_state = _cluster_start(args, argv)
        if cluster_state[0] == "worker":
            return _worker_rank_main(args, cluster_state[1])
    from .runtime import alloc_policy
    logging.info("HBM allocator: %s", alloc_policy.configure(args))   # before any device allocation
    from .graph import registry
    if not args.disable_custom_nodes:
        registry.execute_prestartup_scripts(
            list(itertools.chain.from_iterable(args.custom_nodes_directory)) if args.custom_nodes_directory else None)
    apply_args(args)
    cleanup_temp()
    loop = asyncio.new_event_loop()
    asyncio.set_event_loop(loop)
    server, q = build_server(args, loop)
    coord = None
    if cluster_state is not None:
        from .sched.cluster import Coordinator
        _, comm, listener, procs = cluster_state
        coord = Coordinator(q, server, comm, listener, latency_default=args.latency_mode)
        server.cluster = coord
        threading.Thread(target=coord.run_forever, daemon=True).start()
        logging.info("serving on %d ranks (single prompts on idle ranks, batches split across all)", comm.world)
    else:
        threading.Thread(target=prompt_worker, daemon=True, args=(q, server)).start()
    grpc_srv = None
    if args.grpc_port is not None:
        from .api.grpc_service import start_grpc_server
        grpc_srv, _ = start_grpc_server(server, args.grpc_port, host=args.listen or "0.0.0.0")
    if args.quick_test_for_ci:
        return 0
    call_on_start = None
    if args.auto_launch:
        def call_on_start(address, port):
            import webbrowser
            webbrowser.open(f"http://{'127.0.0.1' if address == '0.0.0.0' else address}:{port}")
    try:
        loop.run_until_complete(run(server, address=args.listen, port=args.port,
                                    verbose=not args.dont_print_server, call_on_start=call_on_start))
    except KeyboardInterrupt:
        logging.info("Stopped server")
    if grpc_srv is not None:
        grpc_srv.stop(grace=1.0)
    if coord is not None:
        coord.shutdown()
        for p in list(cluster_state[3] or []) + list(coord.procs):
            try:
                p.wait(timeout=30)
            except Exception:
                p.kill()
    cleanup_temp()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
