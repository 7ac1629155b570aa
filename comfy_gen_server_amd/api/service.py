"""``comfy_request.v1.Comfy`` + ``grpc.health.v1.Health`` service — actually implemented (the
reference ships only generated stubs, no servicer: ``autogen_python/comfy_request/v1_pb2_grpc.py``;
SURVEY §2.1 C05).

grpcio is present but no protobuf codegen of the contract is (and no network to fetch it), so the
service is exposed over HTTP with the proto field names as JSON (the canonical proto3 JSON
mapping):

  POST /api/v1/comfy/Run               ComfyRequest  -> JobSnapshot      (unary; queues the job)
  POST /api/v1/comfy/RunSync           ComfyRequest  -> JobSnapshot*     (server stream, JSON lines)
  POST /api/v1/comfy/GetJob            JobId         -> JobSnapshot
  POST /api/v1/comfy/GetNodeDefinitions NodeDefRequest -> NodeDefs
  POST /api/v1/comfy/GetModelCatalog   ModelCatalogRequest -> ModelCatalog
  POST /api/v1/comfy/SyncLocalFiles    -> LocalFiles (added/updated/removed since last call, blake3)
  GET  /api/v1/health/Check, /api/v1/health/Watch (stream)

JobSnapshot.status uses the proto enum values (QUEUED=0 EXECUTING=1 COMPLETED=2 ERROR=3 ABORTED=4;
-1 = unknown job in the JSON form, NOT_FOUND over gRPC); outputs carry
WorkflowFile{blake3_hash, mime_type, reference{url, is_temp}}; metrics{queue_seconds,
execution_seconds} are filled (the reference never produces them). ``output_config.webhook_url``
gets a POST of the final snapshot. The same contract over real gRPC (protobuf wire format) is
``grpc_service.py``; both share the job model and the helpers below.
"""
from __future__ import annotations

import asyncio
import json
import logging
import mimetypes
import os
import time
import uuid

from aiohttp import web

from ..graph import registry
from ..graph.validation import validate_prompt
from ..utils import folder_paths
from ..utils.hashing import file_digest

STATUS = {"UNSPECIFIED": -1, "QUEUED": 0, "EXECUTING": 1, "COMPLETED": 2, "ERROR": 3, "ABORTED": 4}


class JobTracker:
    def __init__(self, server):
        self.server = server
        self.jobs = {}   # prompt_id -> dict
        self._local_files = {}

    def snapshot(self, job_id):
        q = self.server.prompt_queue
        j = self.jobs.get(job_id, {"request_id": None, "submitted": time.time()})
        hist = q.get_history(prompt_id=job_id) if q else {}
        cur, pend = q.get_current_queue() if q else ([], [])
        status = "UNSPECIFIED"
        outputs = []
        metrics = {}
        if job_id in hist:
            h = hist[job_id]
            st = (h.get("status") or {}).get("status_str")
            interrupted = any(m[0] == "execution_interrupted" for m in (h.get("status") or {}).get("messages", []))
            status = "ABORTED" if interrupted else ("COMPLETED" if st == "success" else "ERROR")
            prompt = h["prompt"][2]
            for node_id, ui in (h.get("outputs") or {}).items():
                for img in ui.get("images", []):
                    d = folder_paths.get_directory_by_type(img.get("type", "output"))
                    path = os.path.join(d, img.get("subfolder", ""), img["filename"])
                    f = {"mime_type": mimetypes.guess_type(path)[0] or "application/octet-stream",
                         "reference": {"url": f"/view?filename={img['filename']}&subfolder={img.get('subfolder', '')}"
                                              f"&type={img.get('type', 'output')}",
                                       "is_temp": img.get("type") == "temp"}}
                    if os.path.exists(path):
                        f["blake3_hash"] = file_digest(path)
                    outputs.append({"node_id": node_id, "class_type": prompt.get(node_id, {}).get("class_type", ""),
                                    "file": f})
            metrics = {"queue_seconds": int(j.get("started", j["submitted"]) - j["submitted"]),
                       "execution_seconds": int(h.get("metrics", {}).get("total_seconds", 0))}
        elif any(x[1] == job_id for x in cur):
            status = "EXECUTING"
        elif any(x[1] == job_id for x in pend):
            status = "QUEUED"
        snap = {"job_id": job_id, "status": STATUS[status], "status_name": status, "outputs": outputs,
                "metrics": metrics}
        if j.get("request_id"):
            snap["request_id"] = j["request_id"]
        return snap


def _norm_input(v):
    # google.protobuf.Struct carries every number as a double: restore integral link slots
    # ([node_id, 0.0] -> [node_id, 0]); INT widget values are coerced by the validator.
    if isinstance(v, list) and len(v) == 2 and isinstance(v[0], str) and isinstance(v[1], float) and v[1].is_integer():
        return [v[0], int(v[1])]
    return v


def _workflow_to_prompt(req):
    wf = req.get("workflow") or {}
    prompt = {nid: {"class_type": step["class_type"],
                    "inputs": {k: _norm_input(v) for k, v in (step.get("inputs") or {}).items()}}
              for nid, step in wf.items()}
    return prompt


def submit_request(server, tracker, req):
    """Validate + enqueue a ComfyRequest (dict form). Returns (job_id, None) or (None, error dict)."""
    prompt = _workflow_to_prompt(req)
    valid = validate_prompt(prompt)
    if not valid[0]:
        return None, {"error": valid[1], "node_errors": valid[3]}
    job_id = str(uuid.uuid4())
    number = server.number
    server.number += 1
    oc = req.get("output_config") or {}
    tracker.jobs[job_id] = {"request_id": req.get("request_id"), "submitted": time.time(),
                            "webhook_url": oc.get("webhook_url"), "write_to_graph_id": oc.get("write_to_graph_id")}
    server.prompt_queue.put((number, job_id, prompt, {}, valid[2]))
    return job_id, None


def node_definitions(extension_ids=None):
    """NodeDefs.defs: every registered node (or those of the listed extension modules)."""
    defs = {}
    for name in registry.NODE_CLASS_MAPPINGS:
        cls = registry.NODE_CLASS_MAPPINGS[name]
        if extension_ids and getattr(cls, "RELATIVE_PYTHON_MODULE", cls.__module__) not in extension_ids:
            continue
        try:
            info = registry.node_info(name)
        except Exception:
            continue
        inputs = []
        for sect in ("required", "optional"):
            for label, spec in info["input"].get(sect, {}).items():
                et = spec[0] if isinstance(spec[0], str) else "COMBO"
                sp = dict(spec[1]) if len(spec) > 1 and isinstance(spec[1], dict) else {}
                if et == "COMBO":
                    sp["options"] = list(spec[0])
                sp["optional"] = sect == "optional"
                inputs.append({"label": label, "edge_type": et, "spec": json.loads(json.dumps(sp, default=str))})
        outputs = [{"label": n, "edge_type": t} for n, t in zip(info["output_name"], info["output"])]
        defs[name] = {"display_name": info["display_name"], "description": info["description"],
                      "category": info["category"], "inputs": inputs, "outputs": outputs,
                      "output_node": info["output_node"]}
    return defs


def model_catalog(base_family=None):
    models = {}
    for kind in folder_paths.folder_names_and_paths:
        if kind in ("custom_nodes", "configs") or (base_family and kind not in base_family):
            continue
        try:
            files = folder_paths.get_filename_list(kind)
        except Exception:
            files = []
        models[kind] = {"info": [{"display_name": f} for f in files]}
    return models


def local_files_delta(tracker):
    cur = {}
    for kind in ("input", "output", "temp"):
        d = folder_paths.get_directory_by_type(kind)
        if not d or not os.path.isdir(d):
            continue
        for root, _, files in os.walk(d):
            for f in files:
                p = os.path.join(root, f)
                st = os.stat(p)
                cur[p] = (st.st_mtime, st.st_size, kind)
    prev = tracker._local_files

    def entry(p, meta):
        return {"name": os.path.basename(p), "path": p, "size": meta[1],
                "mime_type": mimetypes.guess_type(p)[0] or "application/octet-stream"}
    added = [entry(p, m) for p, m in cur.items() if p not in prev]
    updated = [entry(p, m) for p, m in cur.items() if p in prev and prev[p][:2] != m[:2]]
    removed = [entry(p, m) for p, m in prev.items() if p not in cur]
    tracker._local_files = cur
    return {"added": added, "updated": updated, "removed": removed}


def add_service_routes(routes, server):
    tracker = getattr(server, "job_tracker", None) or JobTracker(server)
    server.job_tracker = tracker

    def submit(req):
        return submit_request(server, tracker, req)

    @routes.post("/api/v1/comfy/Run")
    async def run(request):
        req = await request.json()
        job_id, err = submit(req)
        if err is not None:
            return web.json_response(err, status=400)
        return web.json_response(tracker.snapshot(job_id))

    @routes.post("/api/v1/comfy/RunSync")
    async def run_sync(request):
        req = await request.json()
        job_id, err = submit(req)
        if err is not None:
            return web.json_response(err, status=400)
        resp = web.StreamResponse(headers={"Content-Type": "application/x-ndjson"})
        await resp.prepare(request)
        last = None
        while True:
            snap = tracker.snapshot(job_id)
            key = (snap["status"], len(snap["outputs"]))
            if key != last:
                await resp.write((json.dumps(snap) + "\n").encode())
                last = key
            if snap["status"] in (STATUS["COMPLETED"], STATUS["ERROR"], STATUS["ABORTED"]):
                break
            await asyncio.sleep(0.05)
        await resp.write_eof()
        return resp

    @routes.post("/api/v1/comfy/GetJob")
    async def get_job(request):
        req = await request.json()
        return web.json_response(tracker.snapshot(req["job_id"]))

    @routes.post("/api/v1/comfy/GetNodeDefinitions")
    async def get_node_defs(request):
        try:
            req = await request.json()
        except Exception:
            req = {}
        return web.json_response({"defs": node_definitions(req.get("extension_ids"))})

    @routes.post("/api/v1/comfy/GetModelCatalog")
    async def get_model_catalog(request):
        try:
            req = await request.json()
        except Exception:
            req = {}
        return web.json_response({"models": model_catalog(req.get("base_family"))})

    @routes.post("/api/v1/comfy/SyncLocalFiles")
    async def sync_local_files(request):
        return web.json_response(local_files_delta(tracker))

    @routes.get("/api/v1/health/Check")
    async def health_check(request):
        return web.json_response({"status": "SERVING"})

    @routes.get("/api/v1/health/Watch")
    async def health_watch(request):
        resp = web.StreamResponse(headers={"Content-Type": "application/x-ndjson"})
        await resp.prepare(request)
        for _ in range(int(request.rel_url.query.get("n", 3))):
            await resp.write((json.dumps({"status": "SERVING"}) + "\n").encode())
            await asyncio.sleep(0.2)
        await resp.write_eof()
        return resp


async def post_webhook(url, snapshot):
    import aiohttp
    try:
        async with aiohttp.ClientSession() as s:
            await s.post(url, json=snapshot, timeout=aiohttp.ClientTimeout(total=10))
    except Exception as e:
        logging.warning("webhook %s failed: %s", url, e)
