"""Multi-process data-parallel path on the CPU (gloo, world_size 2) — the same code the driver runs
on 8 MI355X over RCCL (§7.4 'distributed tests without a cluster')."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env():
    env = dict(os.environ)
    env.update(CGS_FORCE_CPU="1", OMP_NUM_THREADS="2", PYTHONPATH=ROOT)
    return env


def test_bench_dp2_gloo():
    """bench.py under torch.distributed.run with 2 ranks: job broadcast, weight broadcast, per-rank
    generation with global noise indices, uint8 all-gather, max-over-ranks timing, one JSON line."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "1", "--warmup", "0", "--cpu", "--family", "tiny", "--res", "64",
           "--sampler-steps", "2", "--batch-per-gpu", "1"]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["global_batch"] == 2 and res["config"]["parallelism"] == "dp2"
    assert res["value"] > 0 and res["scaling"] == "weak" and res["higher_is_better"] is True


_WORKER = r'''
import os, sys, torch
sys.path.insert(0, os.environ["PYTHONPATH"])
from comfy_gen_server_amd.parallel.comm import init_from_env
c = init_from_env(backend="gloo")
assert c.world == 2
# R1: object broadcast
job = c.broadcast_object({"seed": 7, "prompt": "x"} if c.rank == 0 else None)
assert job == {"seed": 7, "prompt": "x"}
# R3: bucketed module broadcast (tiny buckets force several rounds)
m = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.Linear(16, 4))
torch.manual_seed(100 + c.rank)
for p in m.parameters():
    p.data.normal_()
c.broadcast_module(m, bucket_bytes=256)
flat = torch.cat([p.data.reshape(-1) for p in m.parameters()])
ref = c.all_gather(flat[None])
assert torch.equal(ref[0], ref[1])
# R2: all-gather of per-rank uint8 images
img = torch.full((2, 4, 4, 3), c.rank, dtype=torch.uint8)
g = c.all_gather(img)
assert g.shape == (4, 4, 4, 3) and int(g[0, 0, 0, 0]) == 0 and int(g[3, 0, 0, 0]) == 1
# R6: heartbeat + max
assert c.heartbeat() == 2
assert c.all_reduce_max(float(c.rank)) == 1.0
c.barrier()
c.shutdown()
open(os.path.join(os.environ["CGS_TEST_OUT"], f"ok{c.rank}"), "w").write("ok")
'''


def test_comm_collectives_gloo(tmp_path):
    script = tmp_path / "w.py"
    script.write_text(_WORKER)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(script)]
    env = _env()
    env["CGS_TEST_OUT"] = str(tmp_path)
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert (tmp_path / "ok0").exists() and (tmp_path / "ok1").exists()


def test_dp_split_matches_single_process():
    """Per-image noise replay: the DP split of a batch reproduces the single-rank noise exactly."""
    from comfy_gen_server_amd.sampling import sample as S
    latent = torch.zeros(5, 4, 8, 8)
    full = S.prepare_noise(latent, 123, noise_inds=list(range(5)))
    a = S.prepare_noise(latent[:3], 123, noise_inds=[0, 1, 2])
    b = S.prepare_noise(latent[3:], 123, noise_inds=[3, 4])
    assert torch.equal(torch.cat([a, b]), full)


_SP_WORKER = r'''
import os, sys, torch
sys.path.insert(0, os.environ["PYTHONPATH"])
from comfy_gen_server_amd.parallel.comm import init_from_env
from comfy_gen_server_amd.parallel import sp
from comfy_gen_server_amd import ops
c = init_from_env(backend="gloo")
P = c.world
g = torch.Generator().manual_seed(0)
for heads, S, D in [(8, 64, 16), (4, 48, 32), (1, 32, 64)]:
    q, k, v = (torch.randn(2, S, heads * D, generator=g) for _ in range(3))
    from comfy_gen_server_amd.ops.core import attention_reference
    ref = attention_reference(q, k, v, heads)
    qs, ks, vs = (sp.shard_sequence(t) for t in (q, k, v))
    out_r = sp.ring_attention(qs, ks, vs, heads)
    assert torch.allclose(sp.gather_sequence(out_r), ref, atol=2e-5), ("ring", heads)
    if heads % P == 0:
        out_u = sp.ulysses_attention(qs, ks, vs, heads)
        assert torch.allclose(sp.gather_sequence(out_u), ref, atol=2e-5), ("ulysses", heads)
open(os.path.join(os.environ["CGS_TEST_OUT"], f"sp_ok_{c.rank}"), "w").write("ok")
c.shutdown()
'''


@pytest.mark.parametrize("world", [2, 4])
def test_sequence_parallel_attention_gloo(tmp_path, world):
    """Ulysses (all-to-all heads<->sequence) and ring attention (K/V ring with log-sum-exp merge)
    over gloo ranks reproduce single-process attention on the gathered sequence."""
    env = _env()
    env["CGS_TEST_OUT"] = str(tmp_path)
    script = tmp_path / "sp_worker.py"
    script.write_text(_SP_WORKER)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(script)]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert all((tmp_path / f"sp_ok_{i}").exists() for i in range(world))
