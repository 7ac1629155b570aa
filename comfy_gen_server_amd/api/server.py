"""HTTP + WebSocket prompt server (parity: ``server.py:115-857``; C01, C02, C03 routes).

Routes: /ws, /, /embeddings, /extensions, /upload/image, /upload/mask, /view,
/view_all, /view_metadata/{folder}, /system_stats, GET/POST /prompt, /object_info[/{class}],
/history[/{id}], GET/POST /queue, /interrupt, /free, POST /history, /users, /userdata/{file},
/settings[/{id}], /extensions/{name}/..., plus (new) /metrics (Prometheus text), /health,
/api/v1/... gRPC-equivalent JSON service (``api/service.py``).
WS events: status, execution_start, execution_cached, executing, progress, executed,
execution_error, execution_interrupted, yjs_update; binary preview frames
``>I event(1=PREVIEW_IMAGE) >I type(1=JPEG,2=PNG) bytes``.

Threading: the asyncio loop owns sockets; the executor thread only calls
``send_sync`` which hands messages over with ``loop.call_soon_threadsafe`` — single-owner message
passing; ``client_id`` / ``last_node_id`` are guarded by a lock.
"""
from __future__ import annotations

import asyncio
import glob
import io
import json
import logging
import mimetypes
import os
import struct
import sys
import threading
import time
import uuid
from urllib.parse import quote

import aiohttp
from aiohttp import web

VIEW_ALL_MAX_PAGE = 500      # /view_all page_size cap

from ..graph import registry
from ..graph.validation import validate_prompt
from ..runtime import device as dm
from ..utils import folder_paths
from .app import UserManager, AppSettings
from .ymap import OutputMap


class BinaryEventTypes:
    PREVIEW_IMAGE = 1
    UNENCODED_PREVIEW_IMAGE = 2


def encode_bytes(event: int, data: bytes) -> bytes:
    return struct.pack(">I", event) + data


@web.middleware
async def cache_control(request, handler):
    response = await handler(request)
    if request.path.endswith(".js") or request.path.endswith(".css"):
        response.headers.setdefault("Cache-Control", "no-cache")
    return response


def create_cors_middleware(allowed_origin: str):
    @web.middleware
    async def cors_middleware(request, handler):
        if request.method == "OPTIONS":
            response = web.Response()
        else:
            response = await handler(request)
        response.headers["Access-Control-Allow-Origin"] = allowed_origin
        response.headers["Access-Control-Allow-Methods"] = "POST, GET, DELETE, PUT, OPTIONS"
        response.headers["Access-Control-Allow-Headers"] = "Content-Type, Authorization"
        response.headers["Access-Control-Allow-Credentials"] = "true"
        return response
    return cors_middleware


def _telemetry_snapshot():
    from ..utils import telemetry
    return telemetry.snapshot()


class PromptServer:
    instance = None

    def __init__(self, loop, enable_cors_header=None, max_upload_size_mb=100.0, multi_user=False, web_root=None):
        PromptServer.instance = self
        mimetypes.init()
        mimetypes.types_map[".js"] = "application/javascript; charset=utf-8"
        self.user_manager = UserManager(multi_user=multi_user)
        self.settings = AppSettings(self.user_manager)
        self.supports = ["custom_nodes_from_web"]
        self.prompt_queue = None
        self.loop = loop
        self.messages = asyncio.Queue()
        self.number = 0
        self._state_lock = threading.Lock()
        self._client_id = None
        self._last_node_id = None
        self.output_map = OutputMap(self)
        self.metrics = {"prompts_total": 0, "prompts_failed": 0, "images_total": 0, "execution_seconds_total": 0.0}
        self.interrupt_hooks = []
        self.cluster = None
        middlewares = [cache_control]
        if enable_cors_header:
            middlewares.append(create_cors_middleware(enable_cors_header))
        self.app = web.Application(client_max_size=round(max_upload_size_mb * 1024 * 1024), middlewares=middlewares)
        self.sockets = {}
        self.web_root = web_root or os.path.join(os.path.dirname(os.path.dirname(os.path.realpath(__file__))), "web")
        self.on_prompt_handlers = []
        self.routes = web.RouteTableDef()
        self._register_routes()

    # ------------------------------------------------------------------ shared state
    @property
    def client_id(self):
        with self._state_lock:
            return self._client_id

    @client_id.setter
    def client_id(self, v):
        with self._state_lock:
            self._client_id = v

    @property
    def last_node_id(self):
        with self._state_lock:
            return self._last_node_id

    @last_node_id.setter
    def last_node_id(self, v):
        with self._state_lock:
            self._last_node_id = v

    # ------------------------------------------------------------------ routes
    def _register_routes(self):
        routes = self.routes

        @routes.get("/ws")
        async def websocket_handler(request):
            ws = web.WebSocketResponse()
            await ws.prepare(request)
            sid = request.rel_url.query.get("clientId", "")
            if sid:
                self.sockets.pop(sid, None)
            else:
                sid = uuid.uuid4().hex
            self.sockets[sid] = ws
            try:
                await self.send("status", {"status": self.get_queue_info(), "sid": sid}, sid)
                if self.client_id == sid and self.last_node_id is not None:
                    await self.send("executing", {"node": self.last_node_id}, sid)
                async for msg in ws:
                    if msg.type == aiohttp.WSMsgType.ERROR:
                        logging.warning("ws connection closed with exception %s", ws.exception())
            finally:
                self.sockets.pop(sid, None)
            return ws

        @routes.get("/")
        async def get_root(request):
            index = os.path.join(self.web_root, "index.html")
            if os.path.exists(index):
                return web.FileResponse(index)
            return web.Response(text="comfy_gen_server_amd: headless MI355X gen-server", content_type="text/plain")

        @routes.get("/embeddings")
        async def get_embeddings(request):
            emb = folder_paths.get_filename_list("embeddings")
            return web.json_response([os.path.splitext(e)[0] for e in emb])

        @routes.get("/extensions")
        async def get_extensions(request):
            files = glob.glob(os.path.join(glob.escape(self.web_root), "extensions/**/*.js"), recursive=True)
            exts = ["/" + os.path.relpath(f, self.web_root).replace(os.sep, "/") for f in files]
            for name, d in registry.EXTENSION_WEB_DIRS.items():
                fs = glob.glob(os.path.join(glob.escape(d), "**/*.js"), recursive=True)
                exts.extend("/extensions/" + quote(name) + "/" + os.path.relpath(f, d).replace(os.sep, "/") for f in fs)
            return web.json_response(exts)

        def get_dir_by_type(dir_type):
            if dir_type is None:
                dir_type = "input"
            if dir_type == "input":
                return folder_paths.get_input_directory(), dir_type
            if dir_type == "temp":
                return folder_paths.get_temp_directory(), dir_type
            if dir_type == "output":
                return folder_paths.get_output_directory(), dir_type
            return folder_paths.get_input_directory(), "input"

        def _within(root, path):
            root = os.path.abspath(root)
            return os.path.commonpath((root, os.path.abspath(path))) == root

        def image_upload(post, image_save_function=None):
            """Contract of ``/upload/image`` (reference ``server.py:254-309``): the file lands in
            ``{type dir}/{subfolder}/{name}`` -- renamed ``name (i).ext`` unless ``overwrite`` is true --
            and the response names it. A path outside the type directory is 400. ``image_save_function``
            (the mask upload) writes the file itself and returns None, or an error response -- then
            nothing is written and that error is the answer (never a 200 for a file that does not exist)."""
            image = post.get("image")
            overwrite = post.get("overwrite")
            upload_dir, image_upload_type = get_dir_by_type(post.get("type"))
            if not (image and getattr(image, "file", None)):
                return web.Response(status=400)
            filename = image.filename
            if not filename or filename != os.path.basename(filename) or filename in (".", ".."):
                return web.Response(status=400)
            subfolder = post.get("subfolder", "") or ""
            full_output_folder = os.path.abspath(os.path.join(upload_dir, os.path.normpath(subfolder)))
            if not _within(upload_dir, full_output_folder):
                return web.Response(status=400)
            filepath = os.path.join(full_output_folder, filename)
            if not (overwrite is not None and overwrite in ("true", "1")):
                stem, ext = os.path.splitext(filename)
                i = 1
                while os.path.exists(filepath):
                    filename = f"{stem} ({i}){ext}"
                    filepath = os.path.join(full_output_folder, filename)
                    i += 1
            if image_save_function is not None:     # validates its reference first; creates the folder itself
                err = image_save_function(image, post, filepath)
                if err is not None:
                    return err
            else:
                os.makedirs(full_output_folder, exist_ok=True)
                with open(filepath, "wb") as f:
                    f.write(image.file.read())
            return web.json_response({"name": filename, "subfolder": subfolder, "type": image_upload_type})

        @routes.post("/upload/image")
        async def upload_image(request):
            post = await request.post()
            return image_upload(post)

        @routes.post("/upload/mask")
        async def upload_mask(request):
            """The uploaded image's alpha channel applied to ``original_ref`` (an existing image; its PNG
            text chunks kept), saved as a new file. A malformed reference is 400, an escaping subfolder
            403, a missing original 404 -- and in each case nothing is written."""
            post = await request.post()

            def image_save_function(image, post, filepath):
                from PIL import Image
                from PIL.PngImagePlugin import PngInfo
                try:
                    original_ref = json.loads(post.get("original_ref") or "")
                    ref_name = original_ref["filename"]
                except (ValueError, KeyError, TypeError):
                    return web.Response(status=400)
                if not isinstance(ref_name, str) or not ref_name:
                    return web.Response(status=400)
                filename, output_dir = folder_paths.annotated_filepath(ref_name)
                if filename.startswith("/") or ".." in filename or filename != os.path.basename(filename):
                    return web.Response(status=400)
                if output_dir is None:
                    output_dir = get_dir_by_type(original_ref.get("type", "output"))[0]
                output_dir = os.path.abspath(output_dir)
                if original_ref.get("subfolder"):
                    full = os.path.abspath(os.path.join(output_dir, original_ref["subfolder"]))
                    if not _within(output_dir, full):
                        return web.Response(status=403)
                    output_dir = full
                file = os.path.join(output_dir, filename)
                if not os.path.isfile(file):
                    return web.Response(status=404)
                with Image.open(file) as original_pil:
                    metadata = PngInfo()
                    for key, val in getattr(original_pil, "text", {}).items():
                        metadata.add_text(key, val)
                    original_pil = original_pil.convert("RGBA")
                    mask_pil = Image.open(image.file).convert("RGBA")
                    original_pil.putalpha(mask_pil.getchannel("A"))
                    os.makedirs(os.path.dirname(filepath), exist_ok=True)   # only once the reference checked out
                    original_pil.save(filepath, compress_level=4, pnginfo=metadata)
                return None
            return image_upload(post, image_save_function)

        @routes.get("/view")
        async def view_image(request):
            if "filename" not in request.rel_url.query:
                return web.Response(status=404)
            filename = request.rel_url.query["filename"]
            filename, output_dir = folder_paths.annotated_filepath(filename)
            if filename[0] == "/" or ".." in filename:
                return web.Response(status=400)
            if output_dir is None:
                output_dir = folder_paths.get_directory_by_type(request.rel_url.query.get("type", "output"))
            if output_dir is None:
                return web.Response(status=400)
            if "subfolder" in request.rel_url.query:
                full = os.path.join(output_dir, request.rel_url.query["subfolder"])
                if os.path.commonpath((os.path.abspath(full), output_dir)) != output_dir:
                    return web.Response(status=403)
                output_dir = full
            filename = os.path.basename(filename)
            file = os.path.join(output_dir, filename)
            from ..utils import imageio
            fut = imageio.pending(file)
            if fut is not None:          # still being encoded behind the worker (async saves)
                try:
                    await asyncio.wait_for(asyncio.wrap_future(fut), timeout=120)
                except Exception:
                    pass
            if not os.path.isfile(file):
                return web.Response(status=404)
            from PIL import Image
            if "preview" in request.rel_url.query:
                with Image.open(file) as img:
                    pp = request.rel_url.query["preview"].split(";")
                    image_format = pp[0]
                    if image_format not in ["webp", "jpeg"] or "a" in request.rel_url.query.get("channel", ""):
                        image_format = "webp"
                    quality = int(pp[-1]) if pp[-1].isdigit() else 90
                    buf = io.BytesIO()
                    if image_format == "jpeg" or image_format == "jpg":
                        img = img.convert("RGB")
                    img.save(buf, format=image_format, quality=quality)
                    return web.Response(body=buf.getvalue(), content_type=f"image/{image_format}",
                                        headers={"Content-Disposition": f'filename="{filename}"'})
            channel = request.rel_url.query.get("channel", "rgba")
            if channel == "rgb":
                with Image.open(file) as img:
                    buf = io.BytesIO()
                    (img.convert("RGB") if img.mode == "RGBA" else img).save(buf, format="PNG")
                    return web.Response(body=buf.getvalue(), content_type="image/png",
                                        headers={"Content-Disposition": f'filename="{filename}"'})
            if channel == "a":
                with Image.open(file) as img:
                    if img.mode == "RGBA":
                        alpha = img.getchannel("A")
                    else:
                        alpha = Image.new("L", img.size, 255)
                    ai = Image.new("RGBA", img.size)
                    ai.putalpha(alpha)
                    buf = io.BytesIO()
                    ai.save(buf, format="PNG")
                    return web.Response(body=buf.getvalue(), content_type="image/png",
                                        headers={"Content-Disposition": f'filename="{filename}"'})
            return web.FileResponse(file, headers={"Content-Disposition": f'filename="{filename}"'})

        @routes.get("/view_all")
        async def view_all(request):
            try:
                page = int(request.rel_url.query.get("page", 1))
                page_size = int(request.rel_url.query.get("page_size", 50))
            except ValueError:
                return web.json_response({"error": "page and page_size must be integers"}, status=400)
            if page < 1 or not 1 <= page_size <= VIEW_ALL_MAX_PAGE:
                return web.json_response({"error": f"page >= 1, 1 <= page_size <= {VIEW_ALL_MAX_PAGE}"}, status=400)
            out_dir = folder_paths.get_output_directory()
            files = []
            if os.path.isdir(out_dir):
                for root, _, fs in os.walk(out_dir):
                    for f in fs:
                        if f.lower().endswith((".png", ".jpg", ".jpeg", ".webp")):
                            p = os.path.join(root, f)
                            files.append((os.path.getmtime(p), os.path.relpath(p, out_dir)))
            files.sort(reverse=True)
            total = len(files)
            sel = files[(page - 1) * page_size: page * page_size]
            items = []
            for _, rel in sel:
                sub, name = os.path.split(rel)
                items.append({"filename": name, "subfolder": sub, "type": "output",
                              "url": f"/view?filename={quote(name)}&subfolder={quote(sub)}&type=output"})
            return web.json_response({"images": items, "page": page, "page_size": page_size, "total": total})

        @routes.get("/view_metadata/{folder_name}")
        async def view_metadata(request):
            folder_name = request.match_info.get("folder_name", None)
            if folder_name is None:
                return web.Response(status=404)
            if "filename" not in request.rel_url.query:
                return web.Response(status=404)
            filename = request.rel_url.query["filename"]
            if not filename.endswith(".safetensors"):
                return web.Response(status=404)
            path = folder_paths.get_full_path(folder_name, filename)
            if path is None:
                return web.Response(status=404)
            from ..runtime.checkpoint import safetensors_header
            out = safetensors_header(path, max_size=1024 * 1024 * 1024)
            if out is None:
                return web.Response(status=404)
            dt = json.loads(out)
            if "__metadata__" not in dt:
                return web.Response(status=404)
            return web.json_response(dt["__metadata__"])

        @routes.get("/system_stats")
        async def system_stats(request):
            import torch
            device = dm.get_torch_device()
            vram_total, torch_vram_total = dm.get_total_memory(device, torch_total_too=True)
            vram_free, torch_vram_free = dm.get_free_memory(device, torch_free_too=True)
            stats = {
                "system": {"os": os.name, "python_version": sys.version, "embedded_python": False,
                           "torch_version": torch.__version__},
                "devices": [{"name": dm.get_torch_device_name(device), "type": device.type, "index": device.index,
                             "vram_total": vram_total, "vram_free": vram_free, "torch_vram_total": torch_vram_total,
                             "torch_vram_free": torch_vram_free}],
                "runtime": {"resident_models": len(dm.current_loaded_models), "metrics": dict(self.metrics),
                            "telemetry": _telemetry_snapshot()},
            }
            if self.cluster is not None:     # node-wide serving (sched/cluster.py)
                c = self.cluster
                stats["cluster"] = {"world": c.world, "generation": c.gen, "regroups": c.regroups,
                                    "dead": sorted(c.dead), "busy": {str(r): p for r, p in dict(c.busy).items()},
                                    "spmd_sizes": sorted(c.ctxs), "regroup_failures": getattr(c, "regroup_failures", 0),
                                    "replaced": dict(getattr(c, "_respawns", {})), "groups_ok": getattr(c, "groups_ok", True)}
            return web.json_response(stats)

        @routes.get("/prompt")
        async def get_prompt(request):
            return web.json_response(self.get_queue_info())

        def node_info(node_class):
            return registry.node_info(node_class)

        @routes.get("/object_info")
        async def get_object_info(request):
            out = {}
            for x in registry.NODE_CLASS_MAPPINGS:
                try:
                    out[x] = node_info(x)
                except Exception:
                    logging.error("[ERROR] An error occurred while retrieving information for the '%s' node.", x)
            return web.json_response(out)

        @routes.get("/object_info/{node_class}")
        async def get_object_info_node(request):
            node_class = request.match_info.get("node_class", None)
            out = {}
            if node_class is not None and node_class in registry.NODE_CLASS_MAPPINGS:
                out[node_class] = node_info(node_class)
            return web.json_response(out)

        @routes.get("/history")
        async def get_history(request):
            max_items = request.rel_url.query.get("max_items", None)
            if max_items is not None:
                max_items = int(max_items)
            return web.json_response(self.prompt_queue.get_history(max_items=max_items))

        @routes.get("/history/{prompt_id}")
        async def get_history_id(request):
            return web.json_response(self.prompt_queue.get_history(prompt_id=request.match_info.get("prompt_id", None)))

        @routes.get("/queue")
        async def get_queue(request):
            cur, pend = self.prompt_queue.get_current_queue()
            return web.json_response({"queue_running": _strip(cur), "queue_pending": _strip(pend)})

        @routes.post("/prompt")
        async def post_prompt(request):
            try:
                json_data = await request.json()
            except Exception:
                return web.json_response({"error": "invalid json", "node_errors": []}, status=400)
            json_data = self.trigger_on_prompt(json_data)
            if "number" in json_data:
                number = float(json_data["number"])
            else:
                number = self.number
                if "front" in json_data and json_data["front"]:
                    number = -number
                self.number += 1
            if "prompt" in json_data:
                prompt = json_data["prompt"]
                valid = validate_prompt(prompt)
                extra_data = json_data.get("extra_data", {})
                if "client_id" in json_data:
                    extra_data["client_id"] = json_data["client_id"]
                if valid[0]:
                    prompt_id = str(uuid.uuid4())
                    outputs_to_execute = valid[2]
                    self.prompt_queue.put((number, prompt_id, prompt, extra_data, outputs_to_execute))
                    return web.json_response({"prompt_id": prompt_id, "number": number, "node_errors": valid[3]})
                logging.warning("invalid prompt: %s", valid[1])
                return web.json_response({"error": valid[1], "node_errors": valid[3]}, status=400)
            return web.json_response({"error": "no prompt", "node_errors": []}, status=400)

        @routes.post("/queue")
        async def post_queue(request):
            json_data = await request.json()
            if "clear" in json_data and json_data["clear"]:
                self.prompt_queue.wipe_queue()
            if "delete" in json_data:
                for id_to_delete in json_data["delete"]:
                    self.prompt_queue.delete_queue_item(lambda a: a[1] == id_to_delete)
            return web.Response(status=200)

        @routes.post("/interrupt")
        async def post_interrupt(request):
            dm.interrupt_current_processing()
            for h in self.interrupt_hooks:         # multi-rank serving: forward to busy ranks
                h()
            return web.Response(status=200)

        @routes.post("/free")
        async def post_free(request):
            json_data = await request.json()
            unload_models = json_data.get("unload_models", False)
            free_memory = json_data.get("free_memory", False)
            if unload_models:
                self.prompt_queue.set_flag("unload_models", unload_models)
            if free_memory:
                self.prompt_queue.set_flag("free_memory", free_memory)
            return web.Response(status=200)

        @routes.post("/history")
        async def post_history(request):
            json_data = await request.json()
            if "clear" in json_data and json_data["clear"]:
                self.prompt_queue.wipe_history()
            if "delete" in json_data:
                for id_to_delete in json_data["delete"]:
                    self.prompt_queue.delete_history_item(id_to_delete)
            return web.Response(status=200)

        @routes.get("/metrics")
        async def get_metrics(request):
            lines = []
            for k, v in self.metrics.items():
                lines.append(f"# TYPE cgs_{k} counter")
                lines.append(f"cgs_{k} {v}")
            lines.append("# TYPE cgs_queue_remaining gauge")
            lines.append(f"cgs_queue_remaining {self.get_queue_info()['exec_info']['queue_remaining']}")
            lines.append("# TYPE cgs_resident_models gauge")
            lines.append(f"cgs_resident_models {len(dm.current_loaded_models)}")
            from ..utils import telemetry
            lines += telemetry.prometheus_lines()
            # sampler-loop graph coverage: why a run was not replayed from hipGraphs
            from ..sampling import run_graph, step_graph
            for name, st in (("step_graph", step_graph.stats), ("run_graph", run_graph.stats)):
                for k, v in st.items():
                    if isinstance(v, (int, float)):
                        lines.append(f"# TYPE cgs_{name}_{k} counter")
                        lines.append(f"cgs_{name}_{k} {v}")
                lines.append(f"# TYPE cgs_{name}_ineligible counter")
                for reason, n in sorted(st.get("ineligible", {}).items()):
                    r = reason.replace("\\", "\\\\").replace('"', "'")
                    lines.append(f'cgs_{name}_ineligible{{reason="{r}"}} {n}')
            return web.Response(text="\n".join(lines) + "\n", content_type="text/plain")

        @routes.get("/health")
        async def get_health(request):
            return web.json_response({"status": "SERVING", "queue_remaining": self.get_queue_info()["exec_info"]["queue_remaining"]})

    def add_routes(self):
        self.user_manager.add_routes(self.routes)
        self.settings.add_routes(self.routes)
        from .service import add_service_routes
        add_service_routes(self.routes, self)
        api_routes = web.RouteTableDef()
        for route in self.routes:
            if isinstance(route, web.RouteDef):
                api_routes.route(route.method, "/api" + route.path)(route.handler, **route.kwargs)
        self.app.add_routes(api_routes)
        self.app.add_routes(self.routes)
        for name, d in registry.EXTENSION_WEB_DIRS.items():
            self.app.add_routes([web.static("/extensions/" + quote(name), d)])
        if os.path.isdir(self.web_root):
            self.app.add_routes([web.static("/", self.web_root)])

    def get_queue_info(self):
        return {"exec_info": {"queue_remaining": self.prompt_queue.get_tasks_remaining() if self.prompt_queue else 0}}

    # ------------------------------------------------------------------ messaging
    async def send(self, event, data, sid=None):
        if event == BinaryEventTypes.UNENCODED_PREVIEW_IMAGE:
            await self.send_image(data, sid=sid)
        elif isinstance(data, (bytes, bytearray)):
            await self.send_bytes(event, data, sid)
        else:
            await self.send_json(event, data, sid)

    async def send_image(self, image_data, sid=None):
        image_type, image, max_size = image_data
        from PIL import Image
        if max_size is not None:
            image.thumbnail((max_size, max_size), Image.LANCZOS if hasattr(Image, "LANCZOS") else Image.Resampling.LANCZOS)
        type_num = 2 if image_type == "PNG" else 1
        bio = io.BytesIO()
        header = struct.pack(">I", type_num)
        bio.write(header)
        image.save(bio, format=image_type, quality=95, compress_level=1)
        await self.send_bytes(BinaryEventTypes.PREVIEW_IMAGE, bio.getvalue(), sid=sid)

    async def send_bytes(self, event, data, sid=None):
        message = encode_bytes(event, data)
        if sid is None:
            for ws in list(self.sockets.values()):
                await _send_socket_catch_exception(ws.send_bytes, message)
        elif sid in self.sockets:
            await _send_socket_catch_exception(self.sockets[sid].send_bytes, message)

    async def send_json(self, event, data, sid=None):
        message = {"type": event, "data": data}
        if sid is None:
            for ws in list(self.sockets.values()):
                await _send_socket_catch_exception(ws.send_json, message)
        elif sid in self.sockets:
            await _send_socket_catch_exception(self.sockets[sid].send_json, message)

    def send_sync(self, event, data, sid=None):
        """Thread-safe hand-off to the event loop (reference server.py:813-815). After shutdown the
        loop is closed: late progress ticks from a still-running node are dropped, not raised."""
        if self.loop.is_closed():
            return
        try:
            self.loop.call_soon_threadsafe(self.messages.put_nowait, (event, data, sid))
        except RuntimeError:      # closed between the check and the call
            pass

    def queue_updated(self):
        self.send_sync("status", {"status": self.get_queue_info()})

    def broadcast_yjs_updates(self):
        self.send_sync("yjs_update", self.output_map.encode_update())

    async def publish_loop(self):
        while True:
            msg = await self.messages.get()
            await self.send(*msg)

    async def start(self, address, port, verbose=True, call_on_start=None):
        runner = web.AppRunner(self.app, access_log=None)
        await runner.setup()
        site = web.TCPSite(runner, address, port)
        await site.start()
        self._runner = runner
        if verbose:
            logging.info("Starting server\nTo see the GUI go to: http://%s:%s", address, port)
        if call_on_start is not None:
            call_on_start(address, port)

    def add_on_prompt_handler(self, handler):
        self.on_prompt_handlers.append(handler)

    def trigger_on_prompt(self, json_data):
        for handler in self.on_prompt_handlers:
            try:
                json_data = handler(json_data)
            except Exception:
                logging.warning("[ERROR] An error occurred during the on_prompt_handler processing", exc_info=True)
        return json_data


def _strip(items):
    """Queue entries are (number, id, prompt, extra, outputs) — JSON-friendly copy."""
    return [list(x) for x in items]


async def _send_socket_catch_exception(function, message):
    try:
        await function(message)
    except (aiohttp.ClientError, aiohttp.ClientPayloadError, ConnectionResetError, ConnectionError) as err:
        logging.warning("send error: %s", err)
