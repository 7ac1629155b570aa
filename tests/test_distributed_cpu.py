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


_FT_WORKER = r'''
import os, sys, torch
sys.path.insert(0, os.environ["PYTHONPATH"])
from comfy_gen_server_amd.parallel.comm import init_from_env
from comfy_gen_server_amd.runtime import device as dm
dm.set_cpu_mode(True)
c = init_from_env(backend="gloo")
from comfy_gen_server_amd.tools.synth import build_pipeline
from comfy_gen_server_amd.parallel.dp import DataParallelGenerator, Job
with torch.inference_mode():
    patcher, clip, vae = build_pipeline("tiny", device=torch.device("cpu"), dtype=torch.float32, seed=5)
gen = DataParallelGenerator(patcher, clip, vae)
job = Job(batch=5, steps=2, width=64, height=64, seed=9)
with torch.inference_mode():
    out = gen.run(job, fault_tolerant=True)
out_dir = os.environ["CGS_TEST_OUT"]
if c.world == 1 or c.rank == 0:
    torch.save(out, os.path.join(out_dir, f"imgs_ws{c.world}.pt"))
open(os.path.join(out_dir, f"done_{c.world}_{c.rank}"), "w").write("ok")
'''


def test_dp_rank_failure_recovery(tmp_path):
    """3 ranks (own launcher, not torchrun's fail-fast agent); rank 2 dies after generating. Rank 0
    sees it missing in the store liveness round, collects rank 1's shard through the store,
    recomputes rank 2's shard and returns the whole batch — the same images as a 1-rank run (same
    per-image noise; only the fp32 reduction order of different batch sizes differs)."""
    script = tmp_path / "ft_worker.py"
    script.write_text(_FT_WORKER)
    env = _env()
    env.update(CGS_TEST_OUT=str(tmp_path), CGS_DP_LIVENESS_TIMEOUT="10", MASTER_ADDR="127.0.0.1")
    r1 = subprocess.run([sys.executable, str(script)], cwd=ROOT, env=dict(env, WORLD_SIZE="1", RANK="0"),
                        capture_output=True, text=True, timeout=300)
    assert r1.returncode == 0, r1.stderr[-3000:]
    port = str(_free_port())
    procs = [subprocess.Popen([sys.executable, str(script)], cwd=ROOT,
                              env=dict(env, WORLD_SIZE="3", RANK=str(r), LOCAL_RANK=str(r), MASTER_PORT=port,
                                       CGS_FAULT="rank_exit:2"),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(3)]
    rcs = [p.wait(timeout=300) for p in procs]
    assert rcs[2] == 17, rcs                          # the injected death
    assert rcs[0] == 0 and rcs[1] == 0, (rcs, procs[0].stderr.read()[-3000:])
    full = torch.load(tmp_path / "imgs_ws1.pt", weights_only=True)
    rec = torch.load(tmp_path / "imgs_ws3.pt", weights_only=True)
    assert rec.shape == full.shape == (5, 64, 64, 3)
    d = (rec.int() - full.int()).abs()       # batch-size-dependent fp32 reduction order only
    assert d.max() <= 2 and d.float().mean() < 0.25, (d.max(), d.float().mean())


def test_bench_spawns_ranks_without_launcher():
    """``bench.py --gpus 2`` with no torchrun: the parent (which never imports torch) starts the two
    rank processes itself; the JSON line reports the communicator's world size and backend."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0", "--cpu",
           "--family", "tiny", "--res", "64", "--sampler-steps", "2", "--batch-per-gpu", "1"]
    env = _env()
    env.pop("WORLD_SIZE", None)
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["ranks"] == 2 and res["backend"] == "gloo"
    assert res["config"]["global_batch"] == 2 and "op_backends" in res


def test_bench_rejects_world_mismatch():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--cpu", "--family", "tiny"]
    env = dict(_env(), WORLD_SIZE="1", RANK="0")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def test_step_noise_is_keyed_by_global_index():
    """Ancestral/SDE noise of image i depends on (seed, i, step) only: any rank split reproduces the
    one-rank draw, and rank r's local image j does NOT reuse rank 0's image-j noise (the round-1 bug:
    a per-rank generator seeded with the job seed)."""
    from comfy_gen_server_amd import ops
    shape = (6, 4, 8, 8)
    for stream in (0, 5):
        full = ops.philox_randn(shape, 77, list(range(6)), stream)
        parts = [ops.philox_randn((2,) + shape[1:], 77, [2 * r, 2 * r + 1], stream) for r in range(3)]
        assert torch.equal(torch.cat(parts), full)
        assert (parts[1][0] - parts[0][0]).abs().mean() > 0.5
    assert (ops.philox_randn(shape, 77, range(6), 0) - ops.philox_randn(shape, 77, range(6), 1)).abs().mean() > 0.5
    # Brownian increments split the same way
    bt = [ops.brownian_increment((2, 4, 4, 4), 3, [2 * r, 2 * r + 1], 0.0, 4.0, 1.0, 1.5, 1e-3, 24, 1.0)
          for r in range(2)]
    bf = ops.brownian_increment((4, 4, 4, 4), 3, [0, 1, 2, 3], 0.0, 4.0, 1.0, 1.5, 1e-3, 24, 1.0)
    assert torch.equal(torch.cat(bt), bf)


_EQ_WORKER = r'''
import os, sys, torch
sys.path.insert(0, os.environ["PYTHONPATH"])
from comfy_gen_server_amd.parallel.comm import init_from_env
from comfy_gen_server_amd.runtime import device as dm
dm.set_cpu_mode(True)
torch.set_num_threads(1)
c = init_from_env(backend="gloo")
from comfy_gen_server_amd.tools.synth import build_pipeline
from comfy_gen_server_amd.parallel.dp import DataParallelGenerator, Job, generate_local
with torch.inference_mode():
    patcher, clip, vae = build_pipeline("tiny", device=torch.device("cpu"), dtype=torch.float32, seed=5)
gen = DataParallelGenerator(patcher, clip, vae)
gen.sync_weights()
job = Job(batch=6, steps=int(os.environ["EQ_STEPS"]), width=64, height=64, seed=11,
          sampler=os.environ["EQ_SAMPLER"])
off, n = gen._shard(job, c.rank)
with torch.inference_mode():
    lat = generate_local(patcher, clip, vae, job, off, n, decode=False).contiguous()
allv = c.all_gather(lat)
if c.rank == 0:
    torch.save(allv, os.path.join(os.environ["CGS_TEST_OUT"], f"lat_ws{c.world}.pt"))
c.shutdown()
'''


@pytest.mark.parametrize("sampler", ["euler_ancestral", "dpmpp_2m_sde"])
def test_dp_ws3_equals_ws1(tmp_path, sampler):
    """A 3-rank data-parallel run of a 6-image batch with a stochastic sampler (8 steps) gives the
    same latents as the 1-rank run of the whole batch (reference semantics: independent per-image
    noise, comfy/k_diffusion/sampling.py:60-61, made split-invariant by keying on the global index)."""
    script = tmp_path / "eq_worker.py"
    script.write_text(_EQ_WORKER)
    env = dict(_env(), CGS_TEST_OUT=str(tmp_path), EQ_STEPS="8", EQ_SAMPLER=sampler, OMP_NUM_THREADS="1")
    for ws in (1, 3):
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ws}",
               "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(script)]
        r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-3000:]
    a = torch.load(tmp_path / "lat_ws1.pt", weights_only=True)
    b = torch.load(tmp_path / "lat_ws3.pt", weights_only=True)
    assert a.shape == b.shape == (6, 4, 8, 8)
    assert torch.allclose(a, b, atol=1e-4, rtol=1e-4), (a - b).abs().max()
    # distinct images really got distinct noise (no rank-correlated images)
    assert (b[2] - b[0]).abs().mean() > 0.05 and (b[4] - b[0]).abs().mean() > 0.05


def test_run_many_matches_run_cpu(monkeypatch):
    """``run_many`` (the serving loop; its pipelined form needs a GPU) gives each job's images in
    order, identical to ``run`` per job."""
    monkeypatch.setenv("CGS_FORCE_CPU", "1")
    from comfy_gen_server_amd.parallel.dp import DataParallelGenerator, Job
    from comfy_gen_server_amd.tools.synth import build_pipeline
    with torch.inference_mode():
        patcher, clip, vae = build_pipeline("tiny", device=torch.device("cpu"), dtype=torch.float32, seed=5)
        gen = DataParallelGenerator(patcher, clip, vae)
        jobs = [Job(batch=2, steps=3, seed=s, width=64, height=64) for s in (3, 4)]
        many = list(gen.run_many(iter(jobs), pipeline=True))     # no GPU: falls back to in-order
        one = [gen.run(j) for j in jobs]
    assert len(many) == 2
    for a, b in zip(many, one):
        assert a.dtype == torch.uint8 and torch.equal(a, b)


_LAT_WORKER = r'''
import os, sys, torch
sys.path.insert(0, os.environ["PYTHONPATH"])
from comfy_gen_server_amd.parallel.comm import init_from_env
from comfy_gen_server_amd.runtime import device as dm
dm.set_cpu_mode(True)
c = init_from_env(backend="gloo")
from comfy_gen_server_amd.tools.synth import build_pipeline
from comfy_gen_server_amd.parallel.dp import generate_local, Job
from comfy_gen_server_amd.parallel.latency import LatencyParallel
lay = int(os.environ["CGS_TEST_LAYOUT_BATCH"])
with torch.inference_mode():
    patcher, clip, vae = build_pipeline("tiny", device=torch.device("cpu"), dtype=torch.float32, seed=5)
    lp = LatencyParallel(c, batch=lay)
    res = int(os.environ.get("CGS_TEST_RES", "64"))
    job = Job(batch=1, steps=4, width=res, height=res, seed=21)
    ref = generate_local(patcher, clip, vae, job, 0, 1, decode=False)
    got = generate_local(lp.patch(patcher), clip, vae, job, 0, 1, decode=False)
assert lp.calls >= 4, lp.calls
if lp.Q > 1:
    st = lp.sp.stats
    assert sum(st.values()) > 0, st
    mode = os.environ.get("CGS_SP_ATTN", "auto")
    if mode in ("ring", "kvgather"):
        assert st[mode] > 0, st
if os.environ.get("CGS_TEST_EXPECT_SPATIAL") == "1":
    # every UNet call row-sharded: halo exchanges, group-summed GroupNorms, no whole-image fallback conv
    assert lp.spatial_calls == lp.calls, (lp.spatial_calls, lp.calls)
    st = lp.spatial.stats
    assert st["halo"] > 0 and st["gn"] > 0 and st["gather_fallback"] == 0, st
d = (got - ref).abs().max().item()
print("layout", lay, "G", lp.G, "Q", lp.Q, "maxdiff", d, "sp", None if lp.sp is None else lp.sp.stats, flush=True)
# the batch split changes CPU BLAS blocking (reduction order): fp32 round-off, scaled to the latent
assert d < 2e-5 * max(1.0, ref.abs().max().item()) + 2e-4, d
c.shutdown()
'''


@pytest.mark.parametrize("world,layout_batch,attn,res", [(2, 2, "auto", 64), (2, 1, "auto", 64),
                                                         (2, 1, "kvgather", 64), (4, 2, "auto", 64),
                                                         (2, 1, "ring", 64), (2, 1, "auto", 128),
                                                         (4, 1, "auto", 256), (4, 2, "kvgather", 128)])
def test_latency_mode_matches_single_gpu(tmp_path, world, layout_batch, attn, res):
    """Latency mode (parallel/latency.py) on gloo: CFG/batch split (G groups) x token-parallel
    SpatialTransformers (Q ranks: Ulysses / K-V all-gather / ring attention) sample the same
    latents as the plain single-process sampler. At 128^2 / 256^2 the latent divides into Q row bands
    at every level, so the whole UNet runs row-sharded (parallel/spatial.py: halo exchange per 3x3
    conv, group-summed GroupNorm statistics) -- still equal to the single process."""
    script = tmp_path / "lat_worker.py"
    script.write_text(_LAT_WORKER)
    env = _env()
    env.update(MASTER_ADDR="127.0.0.1", CGS_TEST_LAYOUT_BATCH=str(layout_batch), CGS_SP_ATTN=attn,
               CGS_TEST_RES=str(res))
    if res >= 128:
        env["CGS_TEST_EXPECT_SPATIAL"] = "1"
    port = str(_free_port())
    procs = [subprocess.Popen([sys.executable, str(script)], cwd=ROOT,
                              env=dict(env, WORLD_SIZE=str(world), RANK=str(r), LOCAL_RANK=str(r), MASTER_PORT=port),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(world)]
    outs = [p.communicate(timeout=300) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, (o[-2000:], e[-3000:])
    assert all("maxdiff" in o for o, _ in outs)


def test_bench_watchdog_stops_survivors():
    """``bench.py --gpus 3`` (own launcher): rank 2 dies at its first job; the survivors are blocked in a
    collective, the parent notices the non-zero exit, stops them and exits non-zero within a minute
    (instead of hanging until the 600 s communicator timeout)."""
    import time
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--steps", "1", "--warmup", "1", "--cpu",
           "--family", "tiny", "--res", "64", "--sampler-steps", "2", "--batch-per-gpu", "1"]
    env = _env()
    env.pop("WORLD_SIZE", None)
    env["CGS_FAULT"] = "rank_exit:2"
    t0 = time.time()
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0, r.stdout[-2000:]
    assert "stopped the other ranks" in r.stderr, r.stderr[-3000:]
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert time.time() - t0 < 120


def test_bench_via_executor_two_ranks():
    """``bench.py --via-executor --gpus 2``: the workflow-JSON path (validate_prompt + PromptExecutor),
    SPMD over two ranks; rank 0 writes every image of the batch."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "1", "--cpu",
           "--family", "tiny", "--res", "64", "--sampler-steps", "2", "--batch-per-gpu", "2", "--via-executor"]
    env = _env()
    env.pop("WORLD_SIZE", None)
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["global_batch"] == 4 and "PromptExecutor" in res["path"]
    assert res["pngs_written"] == 8        # warmup + timed step, 4 images each, all on rank 0
