"""comfy_request.v1.Comfy over real gRPC (protobuf wire format) against the tiny CPU model: health,
node definitions, model catalog, Run + GetJob polling, RunSync output stream, SyncLocalFiles."""
import asyncio
import threading
import time

import grpc
import pytest

from test_e2e_cpu import env, graph  # noqa: F401


def _workflow(g):
    from google.protobuf import json_format
    from comfy_gen_server_amd.api import grpc_service as G
    req = G.M["ComfyRequest"]()
    json_format.ParseDict({"request_id": "req-1",
                           "workflow": {k: {"class_type": v["class_type"], "inputs": v["inputs"]} for k, v in g.items()}},
                          req)
    return req


def test_grpc_roundtrip(env):  # noqa: F811
    from comfy_gen_server_amd import cli_args
    from comfy_gen_server_amd.api import grpc_service as G
    from comfy_gen_server_amd.main import build_server, prompt_worker

    loop = asyncio.new_event_loop()
    args = cli_args.parser.parse_args(["--disable-custom-nodes"])
    server, q = build_server(args, loop)
    stop = threading.Event()
    threading.Thread(target=prompt_worker, args=(q, server, stop), daemon=True).start()
    srv, port = G.start_grpc_server(server, 0, host="127.0.0.1", workers=4)
    try:
        ch = grpc.insecure_channel(f"127.0.0.1:{port}")
        st = G.stubs(ch)
        assert st["Check"](G.HealthCheckRequest(), timeout=10).status == 1
        defs = st["GetNodeDefinitions"](G.M["NodeDefRequest"](), timeout=30).defs
        assert "KSampler" in defs and any(i.label == "seed" for i in defs["KSampler"].inputs)
        assert defs["SaveImage"].output_node
        cat = st["GetModelCatalog"](G.M["ModelCatalogRequest"](base_family=["checkpoints"]), timeout=10).models
        assert [i.display_name for i in cat["checkpoints"].info] == ["tiny.safetensors"]
        st["SyncLocalFiles"](G.Empty(), timeout=10).__next__()     # prime the file-state baseline

        # invalid workflow -> INVALID_ARGUMENT
        bad = graph()
        bad["3"]["inputs"]["sampler_name"] = "nope"
        with pytest.raises(grpc.RpcError) as ei:
            st["Run"](_workflow(bad), timeout=30)
        assert ei.value.code() == grpc.StatusCode.INVALID_ARGUMENT

        snap = st["Run"](_workflow(graph(seed=21)), timeout=30)
        assert snap.request_id == "req-1" and snap.status in (0, 1)
        t0 = time.time()
        while snap.status not in G.TERMINAL and time.time() - t0 < 300:
            time.sleep(0.2)
            snap = st["GetJob"](G.M["JobId"](job_id=snap.job_id), timeout=10)
        assert snap.status == 2, snap                     # COMPLETED
        assert len(snap.outputs) == 2 and snap.outputs[0].class_type == "SaveImage"
        f = snap.outputs[0].file
        assert f.mime_type == "image/png" and len(f.blake3_hash) == 64 and f.reference.url.startswith("/view?")
        assert snap.HasField("metrics")

        outs = list(st["RunSync"](_workflow(graph(seed=22)), timeout=300))
        assert len(outs) == 2 and all(o.node_id == "9" for o in outs)

        delta = next(st["SyncLocalFiles"](G.Empty(), timeout=10))
        assert len(delta.added) >= 4 and all(a.mime_type == "image/png" for a in delta.added)

        with pytest.raises(grpc.RpcError) as ei:
            st["GetJob"](G.M["JobId"](job_id="no-such-job"), timeout=10)
        assert ei.value.code() == grpc.StatusCode.NOT_FOUND
    finally:
        srv.stop(0)
        stop.set()
        loop.close()
