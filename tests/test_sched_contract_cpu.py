"""Node-mode serving (``main --gpus N``, sched/cluster.py) keeps the single-process API contract, and its
scheduler keeps idle ranks busy -- on the CPU over Gloo:

* a prompt served by a WORKER rank still reaches the submitting client over the websocket: the binary
  frames (latent previews, ``SaveImageWebsocket`` PNGs -- reference ``custom_nodes/websocket_image_save.py``,
  ``server.py:754-791``) and the Yjs ``outputs`` map update (``execution.py:334-345``, ``server.py:825-832``);
* in an SPMD prompt the Yjs value of a batch split over the ranks describes the whole batch;
* an SPMD prompt on a rank prefix does not block the dispatch loop: single prompts submitted after it run
  concurrently on the ranks outside the prefix;
* a re-rendezvous whose process-group teardown hangs on one rank replaces that rank (bounded) and the node
  becomes whole again.
"""
import asyncio
import base64
import json
import struct
import time
import uuid

import pytest

from test_sched_cpu import _get, _graph, _post, _start, _stop, _wait


def _ws_graph(seed, batch):
    g = _graph(seed, batch, "ws")
    g["9"] = {"class_type": "SaveImageWebsocket", "inputs": {"images": ["8", 0]}}
    return g


async def _run_ws(url, prompts, timeout=180):
    """Submit ``prompts`` (list of (graph, extra)) under one websocket client; collect everything sent to it
    until every prompt reported ``executing`` with node None."""
    import aiohttp
    cid = uuid.uuid4().hex
    frames, events = [], []
    async with aiohttp.ClientSession() as s:
        async with s.ws_connect(url.replace("http", "ws") + f"/ws?clientId={cid}") as ws:
            pids = []
            for graph, extra in prompts:
                async with s.post(url + "/prompt", json={"prompt": graph, "client_id": cid,
                                                         "extra_data": dict(extra or {})}) as r:
                    pids.append((await r.json())["prompt_id"])
            done = set()
            deadline = time.time() + timeout
            while len(done) < len(pids) and time.time() < deadline:
                try:
                    msg = await ws.receive(timeout=5)
                except asyncio.TimeoutError:
                    continue
                if msg.type == aiohttp.WSMsgType.BINARY:
                    frames.append(msg.data)
                elif msg.type == aiohttp.WSMsgType.TEXT:
                    m = json.loads(msg.data)
                    events.append(m)
                    d = m.get("data") or {}
                    if m["type"] == "executing" and d.get("node") is None and d.get("prompt_id") in pids:
                        done.add(d["prompt_id"])
                else:
                    break
    return pids, frames, events


def _yjs_state(events):
    from comfy_gen_server_amd.api import ymap
    ups = [e["data"] for e in events if e["type"] == "yjs_update"]
    assert ups, [e["type"] for e in events]
    return ymap.decode_update(base64.b64decode(ups[-1]["update"]))["maps"]["workflows"]


@pytest.fixture(scope="module")
def node3(tmp_path_factory):
    proc, url, base = _start(tmp_path_factory, 3, ["--preview-method", "latent2rgb"])
    yield url, base
    _stop(proc)


def test_worker_rank_sends_binary_frames_and_yjs_updates(node3):
    url, base = node3
    g = _ws_graph(41, 2)
    g["outputs"] = {"final_latent": ["3", 0]}
    pids, frames, events = asyncio.run(_run_ws(url, [(g, {"dp": "single"})]))
    h = _wait(url, pids)[pids[0]]
    assert h["status"]["status_str"] == "success", h["status"]
    assert h["metrics"]["ranks"] == 2, h["metrics"]           # an idle node serves it on its last worker
    kinds = [struct.unpack(">II", f[:8]) for f in frames]
    assert all(ev == 1 for ev, _ in kinds), kinds             # PREVIEW_IMAGE frames
    pngs = [f[8:] for f, (_, t) in zip(frames, kinds) if t == 2]
    jpgs = [f for f, (_, t) in zip(frames, kinds) if t == 1]
    assert len(pngs) == 2, len(pngs)                          # SaveImageWebsocket: one PNG per image
    assert all(p[:8] == b"\x89PNG\r\n\x1a\n" for p in pngs)
    assert len(jpgs) >= 1                                     # latent2rgb previews of the sampler steps
    state = _yjs_state(events)
    val = json.loads(state["final_latent"])
    assert val[0]["samples"]["tensor"] == [2, 4, 8, 8], val    # one value per list-mapped run of the node
    assert any(e["type"] == "progress" for e in events)


def test_spmd_yjs_value_is_the_whole_batch(node3):
    url, base = node3
    g = _graph(42, 6, "yspmd")
    g["outputs"] = {"lat": ["3", 0], "img": ["8", 0]}
    pids, frames, events = asyncio.run(_run_ws(url, [(g, {})]))
    h = _wait(url, pids)[pids[0]]
    assert h["status"]["status_str"] == "success" and h["metrics"]["ranks"] == "all", h
    state = _yjs_state(events)
    assert json.loads(state["lat"])[0]["samples"]["tensor"] == [6, 4, 8, 8], state["lat"]
    assert json.loads(state["img"])[0]["tensor"] == [6, 64, 64, 3], state["img"]


def test_spmd_prefix_prompt_does_not_block_single_prompts(tmp_path_factory):
    """4 ranks: a batch-2 prompt runs SPMD on [0, 2); two single prompts submitted right after it run on
    ranks 3 and 2 while it is still running."""
    proc, url, base = _start(tmp_path_factory, 4)
    try:
        warm = [_post(url + "/prompt", {"prompt": _graph(1 + i, 1, f"w{i}")})["prompt_id"] for i in range(4)]
        _wait(url, warm)
        big = _graph(50, 2, "big")
        big["3"]["inputs"]["steps"] = 40
        a = _post(url + "/prompt", {"prompt": big})["prompt_id"]
        singles = [_post(url + "/prompt", {"prompt": _graph(60 + i, 1, f"s{i}")})["prompt_id"] for i in range(2)]
        h = _wait(url, [a] + singles, timeout=300)
        c = _post(url + "/prompt", {"prompt": _graph(65, 3, "three")})["prompt_id"]
        h.update(_wait(url, [c], timeout=300))
    finally:
        _stop(proc)
    assert all(e["status"]["status_str"] == "success" for e in h.values()), {k: v["status"] for k, v in h.items()}
    assert h[a]["metrics"]["ranks"] == [0, 1], h[a]["metrics"]
    assert sorted(h[s]["metrics"]["ranks"] for s in singles) == [2, 3]
    for s in singles:     # overlap in time with the SPMD prompt
        assert h[s]["metrics"]["started_at"] < h[a]["metrics"]["finished_at"], (h[s]["metrics"], h[a]["metrics"])
        assert h[s]["metrics"]["finished_at"] < h[a]["metrics"]["finished_at"], (h[s]["metrics"], h[a]["metrics"])
    # a batch of 3 on 4 ranks runs on the 3-rank prefix (every prefix size has its groups)
    assert h[c]["status"]["status_str"] == "success", h[c]["status"]
    assert h[c]["metrics"]["ranks"] == [0, 1, 2] and h[c]["metrics"]["images_per_rank"] == {"0": 1, "1": 1, "2": 1}


def test_hung_teardown_rank_is_replaced_and_node_regroups(tmp_path_factory, monkeypatch):
    """Rank 1 dies inside its sampler; at the re-rendezvous rank 2's process-group teardown hangs: it exits
    after the bound and is replaced, the next re-rendezvous succeeds and a batch-4 prompt uses all 4 ranks."""
    monkeypatch.setenv("CGS_FAULT", "node_exit:KSampler@1,teardown_hang:2")
    monkeypatch.setenv("CGS_TEARDOWN_TIMEOUT_S", "5")
    proc, url, base = _start(tmp_path_factory, 4)
    try:
        a = _post(url + "/prompt", {"prompt": _graph(70, 4, "died")})["prompt_id"]
        ha = _wait(url, [a], timeout=180)[a]
        t0 = time.time()
        deadline = t0 + 240
        cl = None
        while time.time() < deadline:
            cl = _get(url + "/system_stats")["cluster"]
            if cl["generation"] >= 1 and not cl["dead"]:
                break
            time.sleep(0.5)
        whole_after = time.time() - t0
        b = _post(url + "/prompt", {"prompt": _graph(71, 4, "whole")})["prompt_id"]
        hb = _wait(url, [b], timeout=180)[b]
    finally:
        _stop(proc)
    assert ha["status"]["status_str"] == "success", ha["status"]
    assert cl["generation"] >= 1 and cl["dead"] == [], cl
    assert cl["regroup_failures"] >= 1 and cl["replaced"].get("2", 0) >= 1, cl   # the hung teardown's rank
    assert whole_after < 200, whole_after
    assert hb["status"]["status_str"] == "success", hb["status"]
    assert hb["metrics"]["ranks"] == "all" and hb["metrics"]["images_per_rank"] == {"0": 1, "1": 1, "2": 1, "3": 1}
