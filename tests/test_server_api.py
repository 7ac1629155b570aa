"""HTTP/WS API round trip on the CPU (the reference's tests/inference drive a real server
through /prompt + /ws + /history + /view; here the same contract in-process with aiohttp's test
server and the real prompt_worker thread)."""
import asyncio
import json
import threading

import pytest
from aiohttp.test_utils import TestClient, TestServer

from test_e2e_cpu import env, graph  # noqa: F401  (module fixture + workflow builder)


async def _wait_done(ws, prompt_id, timeout=300):
    """Collect WS events until the end-of-prompt sentinel (executing node=None)."""
    events = []
    while True:
        msg = await ws.receive(timeout=timeout)
        if msg.type.name != "TEXT":
            continue
        m = json.loads(msg.data)
        events.append(m)
        if m["type"] == "executing" and m["data"].get("node") is None and m["data"].get("prompt_id") == prompt_id:
            return events


def test_http_ws_roundtrip(env):  # noqa: F811
    from comfy_gen_server_amd import cli_args
    from comfy_gen_server_amd.main import build_server, prompt_worker

    async def main():
        loop = asyncio.get_running_loop()
        args = cli_args.parser.parse_args(["--disable-custom-nodes"])
        server, q = build_server(args, loop)
        stop = threading.Event()
        worker = threading.Thread(target=prompt_worker, args=(q, server, stop), daemon=True)
        worker.start()
        pub = asyncio.ensure_future(server.publish_loop())
        client = TestClient(TestServer(server.app))
        await client.start_server()
        try:
            ws = await client.ws_connect("/ws?clientId=test-client")
            first = json.loads((await ws.receive(timeout=30)).data)
            assert first["type"] == "status" and first["data"]["sid"] == "test-client"

            # object_info covers the node catalog
            oi = await (await client.get("/object_info")).json()
            for name in ("KSampler", "CheckpointLoaderSimple", "SaveImage", "CLIPTextEncode"):
                assert name in oi and "input" in oi[name]
            one = await (await client.get("/object_info/KSampler")).json()
            assert list(one) == ["KSampler"]

            # invalid prompt -> 400 with node_errors
            bad = graph()
            bad["3"]["inputs"]["sampler_name"] = "not_a_sampler"
            r = await client.post("/prompt", json={"prompt": bad, "client_id": "test-client"})
            assert r.status == 400 and "node_errors" in await r.json()

            r = await client.post("/prompt", json={"prompt": graph(seed=11), "client_id": "test-client"})
            assert r.status == 200
            pid = (await r.json())["prompt_id"]
            events = await _wait_done(ws, pid)
            kinds = [e["type"] for e in events]
            assert "execution_start" in kinds and "executed" in kinds and "progress" in kinds

            hist = await (await client.get(f"/history/{pid}")).json()
            assert hist[pid]["status"]["completed"] is True
            img = hist[pid]["outputs"]["9"]["images"][0]
            v = await client.get("/view", params={"filename": img["filename"], "type": "output",
                                                  "subfolder": img["subfolder"]})
            assert v.status == 200 and (await v.read())[:8] == b"\x89PNG\r\n\x1a\n"
            # /api prefix alias, queue, stats, metrics, health
            assert (await client.get("/api/queue")).status == 200
            qd = await (await client.get("/queue")).json()
            assert qd["queue_pending"] == [] and qd["queue_running"] == []
            st = await (await client.get("/system_stats")).json()
            assert "devices" in st and "system" in st
            assert (await client.get("/prompt")).status == 200
            assert (await client.get("/embeddings")).status == 200
            assert (await client.get("/extensions")).status == 200
            met = await (await client.get("/metrics")).text()
            assert "prompts_total" in met
            assert (await client.get("/health")).status == 200
            assert (await client.post("/interrupt")).status == 200
            assert (await client.post("/free", json={"unload_models": True})).status == 200
            assert (await client.post("/history", json={"clear": True})).status == 200
            assert await (await client.get("/history")).json() == {}
            await ws.close()
        finally:
            stop.set()
            await client.close()
            pub.cancel()
        worker.join(timeout=30)

    asyncio.run(main())


def test_example_client_against_server(env, tmp_path):  # noqa: F811
    """examples/api_client.py (HTTP queue + WS progress + /history + /view download) against the
    real server; the example's workflow builder produces a valid prompt for the tiny checkpoint."""
    import importlib.util
    import os
    from comfy_gen_server_amd import cli_args
    from comfy_gen_server_amd.main import build_server, prompt_worker
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("api_client", os.path.join(root, "examples", "api_client.py"))
    ac = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ac)
    wf = ac.txt2img_workflow(ckpt="tiny.safetensors", steps=2, width=64, height=64, batch=2, seed=5, prefix="ex")

    async def main():
        loop = asyncio.get_running_loop()
        args = cli_args.parser.parse_args(["--disable-custom-nodes"])
        server, q = build_server(args, loop)
        stop = threading.Event()
        threading.Thread(target=prompt_worker, args=(q, server, stop), daemon=True).start()
        pub = asyncio.ensure_future(server.publish_loop())
        client = TestClient(TestServer(server.app))
        await client.start_server()
        try:
            pid, files, progress = await ac.run_and_fetch(None, wf, str(tmp_path), session=client)
        finally:
            stop.set()
            pub.cancel()
            await client.close()
        return pid, files, progress

    pid, files, progress = asyncio.new_event_loop().run_until_complete(main())
    assert len(files) == 2 and all(os.path.getsize(f) > 100 for f in files)
    assert progress and progress[-1][0] == progress[-1][1]
