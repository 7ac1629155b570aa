"""R3 checkpoint broadcast inside an SPMD prompt (``SPMD.load_state_dict`` -> ``Comm.broadcast_state_dict``),
two Gloo ranks on the CPU:

* a flat {name: tensor} checkpoint is read by rank 0 only and received by rank 1 over the data plane;
* a nested checkpoint (an upscaler ``.pth`` saved as ``{"params_ema": {...}}``, a hypernetwork with
  non-tensor values) cannot be described by a key / shape / dtype table: every rank reads it itself,
  instead of rank 0 raising while rank 1 waits in the broadcast until the group timeout;
* a failed read on rank 0 fails rank 1 too.
"""
import os
import types

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _plain(o):
    if isinstance(o, torch.Tensor):
        return ("tensor", str(o.dtype), o.float().tolist())
    if isinstance(o, dict):
        return {k: _plain(v) for k, v in o.items()}
    if isinstance(o, (list, tuple)):
        return type(o)(_plain(v) for v in o)
    return o


def _same(plain, t):
    return plain == ("tensor", str(t.dtype), t.float().tolist())


def _worker(rank, world, port, tmp, q):
    import datetime
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from comfy_gen_server_amd.parallel import comm as C
    from comfy_gen_server_amd.sched.spmd import SPMD
    # a file rendezvous: no TCP port to race for when the suite runs in parallel workers
    dist.init_process_group("gloo", init_method=f"file://{tmp}/rdzv", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=120))
    c = C.init_from_env(backend="gloo", timeout_s=120)
    ctx = types.SimpleNamespace(comm=c, rank=c.rank, loads_received=0)
    reads = []

    def loader(path, meta=False):
        def f():
            reads.append(os.path.basename(path))
            sd = torch.load(path, weights_only=True)
            return (sd, {"k": "v"}) if meta else sd
        return f

    out = {}
    flat = os.path.join(tmp, "flat.pt")
    sd = SPMD.load_state_dict(ctx, flat, torch.device("cpu"), False, loader(flat))
    out["flat"] = {k: v.clone() for k, v in sd.items()}
    sd, meta = SPMD.load_state_dict(ctx, flat, torch.device("cpu"), True, loader(flat, True))
    out["flat_meta"] = meta
    nested = os.path.join(tmp, "nested.pth")
    sd = SPMD.load_state_dict(ctx, nested, torch.device("cpu"), False, loader(nested))
    out["nested"] = sd
    sd, meta = SPMD.load_state_dict(ctx, nested, torch.device("cpu"), True, loader(nested, True))
    out["nested_meta"] = meta
    missing = os.path.join(tmp, "missing.pt")
    try:
        SPMD.load_state_dict(ctx, missing, torch.device("cpu"), False, loader(missing))
        out["missing"] = "no error"
    except Exception as ex:   # noqa: BLE001
        out["missing"] = type(ex).__name__
    out["reads"] = reads
    out["received"] = ctx.loads_received
    # plain Python values only: a tensor in the queue travels as a shared-memory fd that the parent may try to
    # receive after this process has exited (connection reset)
    q.put((rank, _plain(out)))
    dist.barrier()
    dist.destroy_process_group()


def test_spmd_checkpoint_broadcast_flat_nested_and_failure(tmp_path):
    g = torch.Generator().manual_seed(0)
    flat = {"w": torch.randn(4, 3, generator=g), "b": torch.randn(3, generator=g).to(torch.bfloat16)}
    torch.save(flat, tmp_path / "flat.pt")
    nested = {"params_ema": {"conv.weight": torch.randn(2, 2, generator=g)}, "activation_func": "relu",
              "is_layer_norm": False, 320: [torch.ones(1)]}
    torch.save(nested, tmp_path / "nested.pth")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, 0, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in (0, 1):
        o = res[r]
        assert set(o["flat"]) == {"w", "b"}
        assert _same(o["flat"]["w"], flat["w"]) and _same(o["flat"]["b"], flat["b"])
        assert o["flat_meta"] == {"k": "v"}
        assert _same(o["nested"]["params_ema"]["conv.weight"], nested["params_ema"]["conv.weight"])
        assert o["nested"]["activation_func"] == "relu" and o["nested_meta"] == {"k": "v"}
        assert o["missing"] in ("FileNotFoundError", "RuntimeError"), o["missing"]
    # the flat checkpoint: rank 0 read it twice, rank 1 never (received twice); the nested one: both ranks
    assert res[0]["reads"] == ["flat.pt", "flat.pt", "nested.pth", "nested.pth", "missing.pt"], res[0]["reads"]
    assert res[1]["reads"] == ["nested.pth", "nested.pth"], res[1]["reads"]
    assert res[1]["received"] == 2 and res[0]["received"] == 0


if __name__ == "__main__":
    pytest.main([__file__, "-q"])
