#!/usr/bin/env python3
"""Client usage of the prompt API (the three patterns of the reference's ``script_examples/``):

  python examples/api_client.py queue  --server 127.0.0.1:8188 [--ckpt NAME] [--seed N]
      POST /prompt and return (fire and forget).
  python examples/api_client.py run    --server 127.0.0.1:8188 --out DIR
      queue over HTTP, follow progress on /ws, then fetch the images via /history + /view.
  python examples/api_client.py grpc   --server 127.0.0.1:50051 --out DIR
      the same through gRPC RunSync (comfy_request.v1.Comfy), images streamed back as references.

Only the standard library and aiohttp (already a server dependency) are used.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import urllib.parse
import urllib.request
import uuid


def txt2img_workflow(ckpt="sd_xl_base_1.0.safetensors", prompt="a lighthouse on a cliff at dawn, oil painting",
                     negative="blurry, low quality", seed=0, steps=20, cfg=8.0, width=1024, height=1024, batch=1,
                     sampler="euler_ancestral", scheduler="normal", prefix="api"):
    """ComfyUI workflow JSON (API format): checkpoint -> two text encodes -> KSampler -> decode -> save."""
    return {
        "4": {"class_type": "CheckpointLoaderSimple", "inputs": {"ckpt_name": ckpt}},
        "5": {"class_type": "EmptyLatentImage", "inputs": {"width": width, "height": height, "batch_size": batch}},
        "6": {"class_type": "CLIPTextEncode", "inputs": {"text": prompt, "clip": ["4", 1]}},
        "7": {"class_type": "CLIPTextEncode", "inputs": {"text": negative, "clip": ["4", 1]}},
        "3": {"class_type": "KSampler", "inputs": {"seed": seed, "steps": steps, "cfg": cfg, "sampler_name": sampler,
                                                  "scheduler": scheduler, "denoise": 1.0, "model": ["4", 0],
                                                  "positive": ["6", 0], "negative": ["7", 0],
                                                  "latent_image": ["5", 0]}},
        "8": {"class_type": "VAEDecode", "inputs": {"samples": ["3", 0], "vae": ["4", 2]}},
        "9": {"class_type": "SaveImage", "inputs": {"filename_prefix": prefix, "images": ["8", 0]}},
    }


def queue_prompt(server, workflow, client_id=None):
    body = json.dumps({"prompt": workflow, "client_id": client_id or str(uuid.uuid4())}).encode()
    req = urllib.request.Request(f"http://{server}/prompt", data=body, headers={"Content-Type": "application/json"})
    with urllib.request.urlopen(req) as r:
        return json.loads(r.read())


async def run_and_fetch(server, workflow, out_dir, session=None, timeout=600):
    """Queue over HTTP, wait on the WebSocket for the end-of-prompt sentinel, download the images.
    ``session`` may be any aiohttp-compatible client whose paths are relative (tests pass a TestClient)."""
    import aiohttp
    own = session is None
    base = "" if session is not None else f"http://{server}"
    session = session or aiohttp.ClientSession()
    client_id = str(uuid.uuid4())
    try:
        ws = await session.ws_connect(f"{base}/ws?clientId={client_id}")
        r = await session.post(f"{base}/prompt", json={"prompt": workflow, "client_id": client_id})
        prompt_id = (await r.json())["prompt_id"]
        progress = []
        while True:
            msg = await ws.receive(timeout=timeout)
            if msg.type != aiohttp.WSMsgType.TEXT:
                continue                                   # binary frames = latent previews
            m = json.loads(msg.data)
            if m["type"] == "progress":
                progress.append((m["data"]["value"], m["data"]["max"]))
            if m["type"] == "execution_error":
                raise RuntimeError(m["data"].get("exception_message"))
            if m["type"] == "executing" and m["data"].get("node") is None and m["data"].get("prompt_id") == prompt_id:
                break
        await ws.close()
        hist = await (await session.get(f"{base}/history/{prompt_id}")).json()
        saved = []
        os.makedirs(out_dir, exist_ok=True)
        for node_out in hist[prompt_id]["outputs"].values():
            for im in node_out.get("images", []):
                q = urllib.parse.urlencode({"filename": im["filename"], "subfolder": im["subfolder"], "type": im["type"]})
                data = await (await session.get(f"{base}/view?{q}")).read()
                path = os.path.join(out_dir, im["filename"])
                with open(path, "wb") as f:
                    f.write(data)
                saved.append(path)
        return prompt_id, saved, progress
    finally:
        if own:
            await session.close()


def run_grpc(server, workflow, timeout=600):
    import grpc
    from google.protobuf import json_format
    from comfy_gen_server_amd.api import grpc_service as G
    req = G.M["ComfyRequest"]()
    json_format.ParseDict({"request_id": str(uuid.uuid4()), "workflow": workflow}, req)
    with grpc.insecure_channel(server) as ch:
        return [json_format.MessageToDict(o) for o in G.stubs(ch)["RunSync"](req, timeout=timeout)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["queue", "run", "grpc"])
    ap.add_argument("--server", default="127.0.0.1:8188")
    ap.add_argument("--ckpt", default="sd_xl_base_1.0.safetensors")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default="api_out")
    a = ap.parse_args()
    wf = txt2img_workflow(ckpt=a.ckpt, seed=a.seed)
    if a.mode == "queue":
        print(queue_prompt(a.server, wf))
    elif a.mode == "run":
        pid, files, _ = asyncio.run(run_and_fetch(a.server, wf, a.out))
        print(pid, files)
    else:
        for o in run_grpc(a.server, wf):
            print(o)


if __name__ == "__main__":
    main()
