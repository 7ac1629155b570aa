"""Latency mode (parallel/latency.py, spatial.py, sp.py) with several ranks on real hardware: the
shared-GPU rehearsal (``CGS_SHARED_GPU=1``: every rank on the one card of the development box, Gloo with
the device payloads staged through host memory, parallel/coll.py). The model-parallel call sequence --
halo exchanges, group-summed GroupNorm statistics, Ulysses / K-V all-gather attention, the CFG all-gather
-- is the one an 8-GPU node runs over RCCL; here it runs on the HIP kernels and must sample the same
latents as one process."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_WORKER = r'''
import json, os, sys, torch
sys.path.insert(0, os.environ["PYTHONPATH"])
from comfy_gen_server_amd.parallel.comm import init_from_env
c = init_from_env()
assert c.backend == "gloo" and c.device.type == "cuda", (c.backend, c.device)
from comfy_gen_server_amd import ops
from comfy_gen_server_amd.runtime import device as dm
dm.set_device_index(c.device.index)
from comfy_gen_server_amd.tools.synth import build_pipeline
from comfy_gen_server_amd.parallel.dp import generate_local, Job
from comfy_gen_server_amd.parallel.latency import LatencyParallel
lay = int(os.environ["CGS_TEST_LAYOUT_BATCH"])
res = int(os.environ["CGS_TEST_RES"])
with torch.inference_mode():
    patcher, clip, vae = build_pipeline(os.environ["CGS_TEST_FAMILY"], device=c.device, dtype=torch.bfloat16, seed=5)
    lp = LatencyParallel(c, batch=lay)
    job = Job(batch=1, steps=4, width=res, height=res, seed=21)
    ref = generate_local(patcher, clip, vae, job, 0, 1, decode=False).float()
    ops.reset_stats()
    got = generate_local(lp.patch(patcher), clip, vae, job, 0, 1, decode=False).float()
    torch.cuda.synchronize()
st = ops.stats()
rel = ((got - ref).norm() / ref.norm()).item()
out = {"rank": c.rank, "G": lp.G, "Q": lp.Q, "calls": lp.calls, "spatial_calls": lp.spatial_calls,
       "spatial": None if lp.spatial is None else dict(lp.spatial.stats),
       "sp": None if lp.sp is None else dict(lp.sp.stats), "rel": rel,
       "lib": {f"{k[0]}:{k[1]}": v for k, v in st.items() if k[1] == "lib"},
       "hip_gn": st.get(("groupnorm", "hip"), 0), "hip_conv": st.get(("conv", "hip"), 0)}
print("RESULT " + json.dumps(out), flush=True)
c.shutdown()
'''


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,layout_batch,attn,res", [(2, 1, "auto", 256), (2, 2, "auto", 256),
                                                         (2, 1, "kvgather", 256)])
def test_latency_mode_two_ranks_on_one_gpu(tmp_path, world, layout_batch, attn, res):
    """SD1.5 architecture (random init, bf16; every head dim on the flash kernels) in latency mode on two
    ranks sharing the GPU vs one process."""
    import json
    script = tmp_path / "lat_gpu_worker.py"
    script.write_text(_WORKER)
    env = dict(os.environ, PYTHONPATH=ROOT, CGS_SHARED_GPU="1", MASTER_ADDR="127.0.0.1",
               CGS_TEST_LAYOUT_BATCH=str(layout_batch), CGS_SP_ATTN=attn, CGS_TEST_RES=str(res), CGS_TEST_FAMILY="sd15",
               OMP_NUM_THREADS="4", HSA_ENABLE_IPC_MODE_LEGACY="0")
    port = str(_free_port())
    procs = [subprocess.Popen([sys.executable, "-u", str(script)], cwd=ROOT,
                              env=dict(env, WORLD_SIZE=str(world), RANK=str(r), LOCAL_RANK=str(r), MASTER_PORT=port),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(world)]
    try:
        outs = [p.communicate(timeout=200) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    res_ = []
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, (o[-2000:], e[-3000:])
        line = [l for l in o.splitlines() if l.startswith("RESULT ")]
        assert line, o[-2000:]
        res_.append(json.loads(line[0][7:]))
    for r in res_:
        assert not r["lib"], r                                 # every op on the HIP kernels
        assert r["calls"] >= 4 and r["rel"] < 3e-2, r          # bf16: same latents as one process
        if layout_batch == 1:                                  # whole UNet row-sharded (Q = world)
            assert r["spatial_calls"] == r["calls"], r
            assert r["spatial"]["halo"] > 0 and r["spatial"]["gn"] > 0 and r["spatial"]["gather_fallback"] == 0, r
            assert r["hip_gn"] > 0 and r["hip_conv"] > 0, r
