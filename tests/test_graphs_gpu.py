"""hipGraph capture/replay of the denoiser (runtime/graphs.py): replayed forwards must equal the
eager forward, plans are retired when weights change, hooks keep the forward eager."""
import pytest
import torch

from comfy_gen_server_amd.models.layers import init_random_fast_, invalidate_all
from comfy_gen_server_amd.models.unet import UNetModel
from comfy_gen_server_amd.runtime.graphs import GraphedForward

CFG = dict(in_channels=4, model_channels=128, out_channels=4, num_res_blocks=[1, 1], channel_mult=[1, 2],
           transformer_depth=[1, 1], transformer_depth_output=[1, 1, 1, 1], transformer_depth_middle=1,
           num_heads=2, num_head_channels=-1, use_linear_in_transformer=True, context_dim=128,
           num_classes="sequential", adm_in_channels=64)


def _inputs(dev, B=4, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(B, 4, 32, 32, generator=g).to(dev, torch.bfloat16)
    t = torch.tensor([999.0, 500.0, 10.0, 1.0][:B]).to(dev)
    ctx = torch.randn(B, 77, 128, generator=g).to(dev, torch.bfloat16)
    y = torch.randn(B, 64, generator=g).to(dev, torch.bfloat16)
    return x, t, ctx, y


@pytest.mark.gpu
def test_graph_replay_matches_eager(cuda, monkeypatch):
    monkeypatch.setenv("CGS_GRAPHS", "1")
    with torch.inference_mode():
        m = UNetModel(**CFG, dtype=torch.bfloat16, device=cuda)
        init_random_fast_(m, seed=3)
        runner = GraphedForward(m)
        x, t, ctx, y = _inputs(cuda)
        ref = m(x, t, context=ctx, y=y, transformer_options={}).float()
        outs = [runner(x, t, context=ctx, y=y, transformer_options={}).float() for _ in range(3)]
        torch.cuda.synchronize()
        assert runner.stats == {"eager": 1, "capture": 1, "replay": 2}, runner.stats
        for o in outs:
            assert (o - ref).abs().max().item() < 2e-2 * (ref.abs().max().item() + 1)
        # new inputs through the same plan
        x2, t2, ctx2, y2 = _inputs(cuda, seed=7)
        ref2 = m(x2, t2, context=ctx2, y=y2, transformer_options={}).float()
        o2 = runner(x2, t2, context=ctx2, y=y2, transformer_options={}).float()
        assert runner.stats["replay"] == 3
        assert (o2 - ref2).abs().max().item() < 2e-2 * (ref2.abs().max().item() + 1)
        # a weight change (LoRA merge / unpatch path) retires the plan
        for p in m.parameters():
            p.data = p.data * 0.5
        invalidate_all(m)
        ref3 = m(x2, t2, context=ctx2, y=y2, transformer_options={}).float()
        o3 = [runner(x2, t2, context=ctx2, y=y2, transformer_options={}).float() for _ in range(3)][-1]
        assert runner.stats["capture"] == 2
        assert (o3 - ref3).abs().max().item() < 2e-2 * (ref3.abs().max().item() + 1)
        # hooks make the forward dynamic: always eager
        e0 = runner.stats["eager"]
        runner(x2, t2, context=ctx2, y=y2, transformer_options={"patches": {"middle_patch": [lambda h, o: h]}})
        assert runner.stats["eager"] == e0 + 1


def test_graphs_cpu_is_eager():
    m = UNetModel(**dict(CFG, model_channels=32, num_heads=2, context_dim=32), dtype=torch.float32)
    from comfy_gen_server_amd.models.layers import init_random_
    init_random_(m, seed=0)
    runner = GraphedForward(m)
    x = torch.randn(2, 4, 16, 16)
    t = torch.tensor([10.0, 20.0])
    ctx = torch.randn(2, 7, 32)
    y = torch.randn(2, 64)
    with torch.inference_mode():
        a = runner(x, t, context=ctx, y=y, transformer_options={})
        b = runner(x, t, context=ctx, y=y, transformer_options={})
    assert runner.stats == {"eager": 2, "capture": 0, "replay": 0}
    assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("sampler", ["euler_ancestral", "euler", "dpmpp_2m", "lcm"])
def test_step_graph_matches_eager_loop(cuda, monkeypatch, sampler):
    """One captured graph per sampler step (UNet(cond||uncond) + CFG + Euler(-a) + in-register noise,
    every scalar from a device table) reproduces the eager Python loop, for two jobs through the
    same plan (second job = pure replay with a new seed, prompt latents and global image offset)."""
    from comfy_gen_server_amd.tools.synth import build_pipeline
    from comfy_gen_server_amd.parallel.dp import Job, generate_local
    from comfy_gen_server_amd.sampling import step_graph
    with torch.inference_mode():
        patcher, clip, vae = build_pipeline("tiny", device=cuda, dtype=torch.bfloat16, seed=2)
        res = {}
        before = dict(step_graph.stats)
        for mode in ("0", "1"):
            monkeypatch.setenv("CGS_GRAPHS", mode)
            outs = []
            for seed, off in ((5, 0), (9, 3)):
                job = Job(batch=3, steps=6, cfg=6.0, sampler=sampler, width=64, height=64, seed=seed)
                outs.append(generate_local(patcher, clip, vae, job, off, 3, decode=False).float())
            res[mode] = outs
        torch.cuda.synchronize()
    assert step_graph.stats["capture"] - before["capture"] >= 1
    assert step_graph.stats["replay"] - before["replay"] >= 12 and step_graph.stats["jobs"] - before["jobs"] == 2
    for a, b in zip(res["0"], res["1"]):
        err = (a - b).abs().max().item()
        assert err < 2e-2 * (a.abs().max().item() + 1), err


@pytest.mark.gpu
@pytest.mark.parametrize("sampler", ["dpm_2_ancestral", "dpmpp_2s_ancestral", "heun"])
def test_step_graph_only_serves_euler_family(cuda, monkeypatch, sampler):
    """The whole-step graph implements Euler / Euler-a only; other samplers must run their own loop."""
    from comfy_gen_server_amd.tools.synth import build_pipeline
    from comfy_gen_server_amd.parallel.dp import Job, generate_local
    from comfy_gen_server_amd.sampling import step_graph
    monkeypatch.setenv("CGS_GRAPHS", "1")
    with torch.inference_mode():
        patcher, clip, vae = build_pipeline("tiny", device=cuda, dtype=torch.bfloat16, seed=2)
        jobs = step_graph.stats["jobs"]
        generate_local(patcher, clip, vae, Job(batch=2, steps=3, sampler=sampler, width=64, height=64, seed=1), 0, 2,
                       decode=False)
    assert step_graph.stats["jobs"] == jobs


@pytest.mark.gpu
@pytest.mark.parametrize("window", [(0.0, 1.0), (0.0, 0.5)])
def test_step_graph_with_controlnet_matches_eager(cuda, monkeypatch, window):
    """ControlNet inside the captured step (K15 path of the step graph): residual injection, strength
    and a host-evaluated timestep window (two on/off patterns -> two graphs) reproduce the eager loop,
    for two jobs with different hints through one plan."""
    import copy
    from comfy_gen_server_amd.graph import registry
    from comfy_gen_server_amd.models.cldm import ControlNet as CN
    from comfy_gen_server_amd.models.layers import init_random_fast_
    from comfy_gen_server_amd.parallel.dp import encode_prompt
    from comfy_gen_server_amd.runtime import controlnet as rcn
    from comfy_gen_server_amd.sampling import sample as S, step_graph
    from comfy_gen_server_amd.tools.synth import TINY_UNET, build_pipeline
    registry.init_nodes(custom_nodes=False)
    NM = registry.NODE_CLASS_MAPPINGS
    with torch.inference_mode():
        patcher, clip, vae = build_pipeline("tiny", device=cuda, dtype=torch.bfloat16, seed=2)
        cfg = copy.deepcopy(TINY_UNET)
        cfg.update(num_heads=2, num_head_channels=-1)
        cm = CN(hint_channels=3, dtype=torch.bfloat16, device=cuda, **cfg)
        init_random_fast_(cm, seed=7)
        pos = encode_prompt(clip, "a house", 64, 64)
        neg = encode_prompt(clip, "blurry", 64, 64)
        res = {}
        for mode in ("0", "1"):
            monkeypatch.setenv("CGS_GRAPHS", mode)
            outs = []
            for j in range(2):
                g = torch.Generator().manual_seed(j)
                hint = torch.rand(1, 64, 64, 3, generator=g)
                cnet = rcn.ControlNet(cm, load_device=cuda)
                pc, nc = NM["ControlNetApplyAdvanced"]().apply_controlnet(pos, neg, cnet, hint, 0.8, window[0],
                                                                          window[1])
                latent = torch.zeros([2, 4, 8, 8])
                noise = S.prepare_noise(latent, 5 + j)
                outs.append(S.sample(patcher, noise, 6, 5.0, "euler_ancestral", "normal", pc, nc, latent,
                                     seed=5 + j).float())
            res[mode] = outs
        torch.cuda.synchronize()
    assert step_graph.stats["replay"] >= 12
    for a, b in zip(res["0"], res["1"]):
        err = (a - b).abs().max().item()
        assert err < 2e-2 * (a.abs().max().item() + 1), err
    assert (res["1"][0] - res["1"][1]).abs().max() > 1e-3     # different hints -> different images


@pytest.mark.gpu
def test_split_k_tail_inside_captured_graph(cuda):
    """The v7 split-K tail (arrival counters zeroed by a kernel node ahead of the GEMM) replays
    correctly from a hipGraph with NEW inputs -- a memset on the capturing stream did not."""
    from comfy_gen_server_amd import _native
    from comfy_gen_server_amd.ops import core
    lib = _native.load_kernels()
    M, N, K = 16384, 1280, 5120
    assert lib.cgs_v7_ws_bytes(M, N, K) > 0
    lib.cgs_gemm_set_variant(7)
    try:
        with torch.inference_mode():
            a = torch.randn(M, K, device=cuda).to(torch.bfloat16)
            w = (torch.randn(N, K, device=cuda) / K ** 0.5).to(torch.bfloat16)
            b = torch.randn(N, device=cuda).to(torch.bfloat16)
            ws = torch.empty(lib.cgs_v7_ws_bytes(M, N, K), dtype=torch.uint8, device=cuda)
            out = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)

            def call():
                assert lib.cgs_gemm_bf16_v7ws(a.data_ptr(), w.data_ptr(), out.data_ptr(), b.data_ptr(), None, M, N, K,
                                              K, K, N, 0, 1, 1.0, ws.data_ptr(), ws.numel(), core._stream()) == 0
            call()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                with torch.cuda.graph(g, stream=s):
                    call()
            torch.cuda.current_stream().wait_stream(s)
            for seed in (1, 2):
                torch.manual_seed(seed)
                a.copy_(torch.randn(M, K, device=cuda).to(torch.bfloat16))
                ws.fill_(0x7F)                     # poison partials and counters between replays
                g.replay()
                torch.cuda.synchronize()
                ref = a.float() @ w.float().t() + b.float()
                err = ((out.float() - ref).norm() / ref.norm()).item()
                assert err < 1e-2, (seed, err)
    finally:
        lib.cgs_gemm_set_variant(-1)


@pytest.mark.gpu
def test_step_graph_static_kv_new_prompt_per_job(cuda, monkeypatch):
    """Cross-attention K/V of the constant context are computed once per job (prologue) and read by
    the replayed steps: a second job with a DIFFERENT prompt through the same plan must see its own
    K/V (equal to the eager loop), not the first job's."""
    from comfy_gen_server_amd.tools.synth import build_pipeline
    from comfy_gen_server_amd.parallel.dp import Job, generate_local
    from comfy_gen_server_amd.sampling import step_graph
    with torch.inference_mode():
        patcher, clip, vae = build_pipeline("tiny", device=cuda, dtype=torch.bfloat16, seed=2)
        res = {}
        for mode in ("0", "1"):
            monkeypatch.setenv("CGS_GRAPHS", mode)
            outs = []
            for seed, prompt in ((5, "a red cube on a table"), (9, "a forest lake at dawn, mist")):
                job = Job(prompt=prompt, batch=2, steps=5, cfg=6.0, sampler="euler_ancestral", width=64, height=64,
                          seed=seed)
                outs.append(generate_local(patcher, clip, vae, job, 0, 2, decode=False).float())
            res[mode] = outs
        torch.cuda.synchronize()
    assert step_graph.stats.get("kv_refresh", 0) > 0
    for a, b in zip(res["0"], res["1"]):
        err = (a - b).abs().max().item()
        assert err < 2e-2 * (a.abs().max().item() + 1), err


@pytest.mark.gpu
@pytest.mark.parametrize("strength", [1.0, 0.7])
def test_controlnet_fused_merge_matches_unfused(cuda, monkeypatch, strength):
    """K15: strength and the chained net's residuals applied in the zero convs' epilogues (scaled 1x1
    weights + residual epilogue) give the same control dict as the unfused merge (x * strength, cast,
    then + previous)."""
    import copy
    from comfy_gen_server_amd.models.cldm import ControlNet as CN
    from comfy_gen_server_amd.models.layers import init_random_fast_
    from comfy_gen_server_amd.runtime import controlnet as rcn
    from comfy_gen_server_amd.tools.synth import TINY_UNET, build_pipeline
    from comfy_gen_server_amd import ops
    with torch.inference_mode():
        patcher, _, _ = build_pipeline("tiny", device=cuda, dtype=torch.bfloat16, seed=2)
        cfg = copy.deepcopy(TINY_UNET)
        cfg.update(num_heads=2, num_head_channels=-1)
        nets = []
        for seed in (7, 8):
            cm = CN(hint_channels=3, dtype=torch.bfloat16, device=cuda, **cfg)
            init_random_fast_(cm, seed=seed)
            c = rcn.ControlNet(cm, load_device=cuda)
            c.cond_hint_original = torch.rand(1, 3, 64, 64)
            c.strength = strength if seed == 7 else 0.5
            c.model_sampling_current = patcher.model.model_sampling
            nets.append(c)
        nets[0].previous_controlnet = nets[1]
        x = torch.randn(2, 4, 8, 8, device=cuda)
        t = torch.tensor([5.0, 5.0], device=cuda)
        cond = {"c_crossattn": torch.randn(2, 7, cfg["context_dim"], device=cuda, dtype=torch.bfloat16)}
        if cfg.get("adm_in_channels"):
            cond["y"] = torch.randn(2, cfg["adm_in_channels"], device=cuda)
        res = {}
        for mode in ("0", "1"):
            monkeypatch.setenv("CGS_CN_FUSE", mode)
            for n in nets:
                n.cond_hint = None
            res[mode] = nets[0].get_control(x, t, cond, 1)
        torch.cuda.synchronize()
    assert ops.stats().get(("conv", "hip"), 0) > 0
    for key in ("middle", "output"):
        assert len(res["0"][key]) == len(res["1"][key]) > 0
        for a, b in zip(res["0"][key], res["1"][key]):
            assert b.dtype == torch.bfloat16
            err = (a.float() - b.float()).abs().max().item()
            assert err < 2e-2 * (a.float().abs().max().item() + 1e-3), (key, err)


@pytest.mark.gpu
def test_cascade_stage_c_step_graph_captures(cuda, monkeypatch):
    """Stable Cascade Stage C sampling captures its Euler-a steps into hipGraphs (a host->device copy in
    the Cascade timestep used to abort every capture silently) and replays the eager result."""
    from comfy_gen_server_amd.graph import registry
    from comfy_gen_server_amd.models.layers import init_random_fast_
    from comfy_gen_server_amd.runtime import families
    from comfy_gen_server_amd.runtime.patcher import ModelPatcher
    from comfy_gen_server_amd.sampling import step_graph
    registry.init_nodes(custom_nodes=False)
    NM = registry.NODE_CLASS_MAPPINGS
    cfg = dict(c_in=16, c_out=16, c_r=64, c_cond=64, c_hidden=[64, 64], nhead=[2, 2], blocks=[[1, 1], [1, 1]],
               block_repeat=[[1, 1], [2, 1]], level_config=["CTA", "CTA"], c_clip_text=64, c_clip_text_pooled=64,
               c_clip_img=768, c_clip_seq=2, switch_level=[False], stable_cascade_stage="c")
    model = families.Stable_Cascade_C(cfg).get_model({})
    model.diffusion_model.to(device=cuda, dtype=torch.bfloat16)
    init_random_fast_(model.diffusion_model, seed=10)
    patcher = ModelPatcher(model, load_device=cuda, offload_device=cuda)
    g = torch.Generator().manual_seed(0)
    pos = [[torch.randn(1, 7, 64, generator=g), {"pooled_output": torch.randn(1, 64, generator=g)}]]
    neg = [[torch.zeros(1, 7, 64), {"pooled_output": torch.zeros(1, 64)}]]
    lat_c, _ = NM["StableCascade_EmptyLatentImage"]().generate(512, 512, 42, 2)
    res = {}
    with torch.inference_mode():
        for mode in ("0", "1"):
            monkeypatch.setenv("CGS_GRAPHS", mode)
            before = dict(step_graph.stats)
            res[mode] = NM["KSampler"]().sample(patcher, 3, 5, 4.0, "euler_ancestral", "simple", pos, neg, lat_c,
                                                1.0)[0]["samples"].float()
        torch.cuda.synchronize()
    assert step_graph.stats.get("capture_failed", 0) == before.get("capture_failed", 0)
    assert step_graph.stats["capture"] > before.get("capture", 0) and step_graph.stats["replay"] > before["replay"]
    err = (res["0"] - res["1"]).abs().max().item()
    assert err < 2e-2 * (res["0"].abs().max().item() + 1), err


@pytest.mark.parametrize("dev", [pytest.param("cuda", marks=pytest.mark.gpu), "cpu"])
@pytest.mark.parametrize("stage", ["c", "b"])
def test_cascade_static_cond_protocol(dev, stage):
    """Stable Cascade's conditioning-only work (every attention block's clip K/V, Stage B's effnet /
    pixel maps) under the step graph's static protocol: "fill" equals the inline forward, "use" reads
    the stored buffers (stale after the cond tensors change in place) and refresh_static_kv brings them
    to the new job's conditioning."""
    from comfy_gen_server_amd.models import cascade as SC
    from comfy_gen_server_amd.models.attention import refresh_static_kv
    from comfy_gen_server_amd.models.layers import init_random_fast_
    if dev == "cuda" and not torch.cuda.is_available():
        pytest.skip("no GPU")
    cuda = torch.device(dev)
    g = torch.Generator().manual_seed(3)
    bf = dict(device=cuda, dtype=torch.bfloat16 if dev == "cuda" else torch.float32)
    if stage == "c":
        m = SC.StageC(c_in=16, c_out=16, c_r=64, c_cond=128, c_hidden=[128, 128], nhead=[2, 2],
                      blocks=[[1, 1], [1, 1]], block_repeat=[[1, 1], [2, 1]], level_config=["CTA", "CTA"],
                      c_clip_text=64, c_clip_text_pooled=64, c_clip_img=768, c_clip_seq=2, switch_level=[False],
                      **bf)
        x = torch.randn(2, 16, 12, 12, generator=g).to(**bf)
        conds = [torch.randn(2, 7, 64, generator=g).to(**bf), torch.randn(2, 1, 64, generator=g).to(**bf),
                 torch.randn(2, 1, 768, generator=g).to(**bf)]

        def run(**kw):
            return m(x, torch.tensor([0.5, 0.25], device=cuda), *conds, **kw).float()
    else:
        m = SC.StageB(c_in=4, c_out=4, c_r=64, patch_size=2, c_cond=128, c_hidden=[64, 128], nhead=[-1, 2],
                      blocks=[[1, 1], [1, 1]], block_repeat=[[1, 1], [1, 1]], level_config=["CT", "CTA"],
                      c_clip=64, c_clip_seq=2, **bf)
        x = torch.randn(2, 4, 32, 32, generator=g).to(**bf)
        conds = [torch.randn(2, 16, 6, 6, generator=g).to(**bf), torch.randn(2, 1, 64, generator=g).to(**bf)]

        def run(**kw):
            return m(x, torch.tensor([0.5, 0.25], device=cuda), conds[0], conds[1], **kw).float()
    init_random_fast_(m, seed=4)
    ids = frozenset(id(t) for t in conds)
    with torch.inference_mode():
        ref = run()
        fill = run(transformer_options={"kv_static": ("fill", ids)})
        assert m.__dict__.get("_kv_static"), "static conditioning store not filled"
        use = run(transformer_options={"kv_static": ("use", ids)})
        for t in conds:                           # the next job's conditioning lands in the same tensors
            t.copy_(torch.randn(t.shape, generator=g).to(**bf))
        ref2 = run()
        stale = run(transformer_options={"kv_static": ("use", ids)})
        assert refresh_static_kv(m, ids) == 1
        use2 = run(transformer_options={"kv_static": ("use", ids)})
    tol = 2e-2 * (ref.abs().max().item() + 1)
    assert (fill - ref).abs().max().item() < tol
    assert (use - ref).abs().max().item() < tol
    assert (use2 - ref2).abs().max().item() < tol
    assert (stale - ref2).abs().max().item() > 10 * (use2 - ref2).abs().max().item()


def _run_jobs(patcher, clip, vae, sampler, seeds, steps=4, scheduler="normal"):
    from comfy_gen_server_amd.parallel.dp import Job, generate_local
    out = []
    for sd in seeds:
        j = Job(batch=2, steps=steps, sampler=sampler, scheduler=scheduler, width=64, height=64, seed=sd, cfg=5.0)
        out.append(generate_local(patcher, clip, vae, j, 0, 2, decode=False).float())
    torch.cuda.synchronize()
    return out


RUN_GRAPH_SAMPLERS = ["heun", "dpm_2", "dpm_2_ancestral", "lms", "dpmpp_2s_ancestral", "dpmpp_sde", "dpmpp_2m_sde",
                      "dpmpp_3m_sde", "ddpm", "heunpp2", "uni_pc", "uni_pc_bh2", "dpmpp_sde_gpu",
                      "dpmpp_2m_sde_gpu", "dpmpp_3m_sde_gpu"]


@pytest.mark.gpu
@pytest.mark.parametrize("sampler", RUN_GRAPH_SAMPLERS)
def test_run_graph_replay_matches_eager(cuda, monkeypatch, sampler):
    """Samplers outside the fused Euler-family step graph replay whole runs from one hipGraph per step
    (run_graph.py): the first run of a plan is eager, the second captures, later ones replay. Replays for
    two seeds (device-resident noise key) equal the eager loop of the same seeds."""
    from comfy_gen_server_amd.sampling import run_graph, samplers
    from comfy_gen_server_amd.tools.synth import build_pipeline
    if sampler not in samplers.KSampler.SAMPLERS:
        pytest.skip(f"{sampler} not in this sampler list")
    monkeypatch.setenv("CGS_GRAPHS", "1")
    with torch.inference_mode():
        patcher, clip, vae = build_pipeline("tiny", device=cuda, dtype=torch.bfloat16, seed=2)
        monkeypatch.setenv("CGS_RUN_GRAPHS", "0")
        ref5, ref6 = _run_jobs(patcher, clip, vae, sampler, [5, 6])
        monkeypatch.setenv("CGS_RUN_GRAPHS", "1")
        before = dict(run_graph.stats)
        _, g6, g5 = _run_jobs(patcher, clip, vae, sampler, [5, 6, 5])
    assert run_graph.stats["capture"] - before["capture"] == 1, run_graph.stats
    assert run_graph.stats["replay_runs"] - before["replay_runs"] == 2, run_graph.stats
    for got, want in ((g6, ref6), (g5, ref5)):
        err = ((got - want).norm() / want.norm()).item()
        assert err < 1e-2, err
    assert ((g5 - g6).norm() / g5.norm()).item() > 1e-2      # the seed reached the replayed noise


@pytest.mark.gpu
@pytest.mark.parametrize("patch", ["FreeU_V2", "PerturbedAttentionGuidance", "SelfAttentionGuidance", "HyperTile",
                                   "TomePatchModel", "PatchModelAddDownscale"])
def test_run_graph_with_model_patches(cuda, monkeypatch, patch):
    """Model patches (transformer / block hooks, post-CFG guidance) run inside the per-step graphs and
    match the eager loop (euler_ancestral: the fused step graph declines patched models)."""
    from comfy_gen_server_amd.graph import registry
    from comfy_gen_server_amd.sampling import run_graph
    from comfy_gen_server_amd.tools.synth import build_pipeline
    registry.init_nodes(custom_nodes=False)
    NM = registry.NODE_CLASS_MAPPINGS
    monkeypatch.setenv("CGS_GRAPHS", "1")
    with torch.inference_mode():
        patcher, clip, vae = build_pipeline("tiny", device=cuda, dtype=torch.bfloat16, seed=2)
        node = NM[patch]()
        kw = {"FreeU_V2": dict(b1=1.3, b2=1.4, s1=0.9, s2=0.2), "PerturbedAttentionGuidance": dict(scale=2.0),
              "SelfAttentionGuidance": dict(scale=0.5, blur_sigma=2.0), "HyperTile": dict(
                  tile_size=32, swap_size=1, max_depth=0, scale_depth=False),
              "TomePatchModel": dict(ratio=0.3), "PatchModelAddDownscale": dict(
                  block_number=1, downscale_factor=2.0, start_percent=0.0, end_percent=0.5,
                  downscale_after_skip=True, downscale_method="bicubic", upscale_method="bicubic")}[patch]
        (patched,) = getattr(node, node.FUNCTION)(patcher, **kw)
        monkeypatch.setenv("CGS_RUN_GRAPHS", "0")
        ref5, ref6 = _run_jobs(patched, clip, vae, "euler_ancestral", [5, 6])
        monkeypatch.setenv("CGS_RUN_GRAPHS", "1")
        before = dict(run_graph.stats)
        _, g6, g5 = _run_jobs(patched, clip, vae, "euler_ancestral", [5, 6, 5])
    assert run_graph.stats["replay_runs"] - before["replay_runs"] == 2, run_graph.stats
    if patch == "TomePatchModel":      # random dst tokens per call: replay draws its own, only check sanity
        assert torch.isfinite(g5).all() and torch.isfinite(g6).all()
        return
    for got, want in ((g6, ref6), (g5, ref5)):
        err = ((got - want).norm() / want.norm()).item()
        assert err < 1e-2, (patch, err)


def _tiny_controlnet(cuda, seed=7):
    import copy
    from comfy_gen_server_amd.models.cldm import ControlNet as CN
    from comfy_gen_server_amd.models.layers import init_random_fast_
    from comfy_gen_server_amd.tools.synth import TINY_UNET
    cfg = copy.deepcopy(TINY_UNET)
    cfg.update(num_heads=2, num_head_channels=-1)
    cm = CN(hint_channels=3, dtype=torch.bfloat16, device=cuda, **cfg)
    init_random_fast_(cm, seed=seed)
    return cm


@pytest.mark.gpu
@pytest.mark.parametrize("sampler", ["dpmpp_2m_sde", "heun"])
def test_run_graph_with_controlnet_matches_eager(cuda, monkeypatch, sampler):
    """ControlNet under a sampler outside the fused Euler family replays from the per-step run graphs:
    the original hint is a static input, so three jobs with three different hints (eager, capture,
    replay) equal the eager loop of the same hints, with a timestep window gating the net."""
    from comfy_gen_server_amd.graph import registry
    from comfy_gen_server_amd.parallel.dp import encode_prompt
    from comfy_gen_server_amd.runtime import controlnet as rcn
    from comfy_gen_server_amd.sampling import run_graph, sample as S
    from comfy_gen_server_amd.tools.synth import build_pipeline
    registry.init_nodes(custom_nodes=False)
    NM = registry.NODE_CLASS_MAPPINGS
    monkeypatch.setenv("CGS_GRAPHS", "1")
    with torch.inference_mode():
        patcher, clip, vae = build_pipeline("tiny", device=cuda, dtype=torch.bfloat16, seed=2)
        cm = _tiny_controlnet(cuda)
        pos = encode_prompt(clip, "a house", 64, 64)
        neg = encode_prompt(clip, "blurry", 64, 64)
        res = {}
        cnet = rcn.ControlNet(cm, load_device=cuda)      # one loaded net, as the cached loader node's output
        for mode in ("0", "1"):
            monkeypatch.setenv("CGS_RUN_GRAPHS", mode)
            before = dict(run_graph.stats)
            outs = []
            for j in range(3):
                g = torch.Generator().manual_seed(j)
                hint = torch.rand(1, 64, 64, 3, generator=g).to(cuda)
                pc, nc = NM["ControlNetApplyAdvanced"]().apply_controlnet(pos, neg, cnet, hint, 0.8, 0.0, 0.6)
                latent = torch.zeros([2, 4, 8, 8])
                noise = S.prepare_noise(latent, 5)
                outs.append(S.sample(patcher, noise, 5, 5.0, sampler, "normal", pc, nc, latent, seed=5).float())
            res[mode] = outs
        torch.cuda.synchronize()
    assert run_graph.stats["capture"] - before["capture"] == 1, run_graph.stats
    assert run_graph.stats["replay_runs"] - before["replay_runs"] == 2, run_graph.stats
    # the replay of job 2 tracks ITS hint: eager vs replay of the same job agree far more closely than two
    # jobs with different hints differ (the random tiny net moves the output only ~1e-3 per hint change)
    hint_effect = (res["0"][1] - res["0"][2]).norm().item()
    assert hint_effect > 0
    for a, b in zip(res["0"], res["1"]):
        diff = (a - b).norm().item()
        assert diff / a.norm().item() < 1e-2, diff
        assert diff < 0.25 * hint_effect, (diff, hint_effect)


@pytest.mark.gpu
def test_run_graph_with_gligen_matches_eager(cuda, monkeypatch):
    """GLIGEN position conditioning (gated self-attention in every transformer block) replays from the
    per-step run graphs: the boxes and phrase embedding are part of the plan key, the device tensors are
    memoised on the eager run, and replay equals the eager loop."""
    from comfy_gen_server_amd.graph import registry
    from comfy_gen_server_amd.models.gligen import GatedSelfAttentionDense, PositionNet, gligen_from_state_dict
    from comfy_gen_server_amd.models.layers import init_random_
    from comfy_gen_server_amd.parallel.dp import encode_prompt
    from comfy_gen_server_amd.runtime.patcher import ModelPatcher
    from comfy_gen_server_amd.sampling import run_graph, sample as S
    from comfy_gen_server_amd.tools.synth import build_pipeline
    registry.init_nodes(custom_nodes=False)
    NM = registry.NODE_CLASS_MAPPINGS
    monkeypatch.setenv("CGS_GRAPHS", "1")
    sd = {}
    for part, b, dim in [("input_blocks", 1, 32), ("input_blocks", 3, 64), ("middle_block", 1, 64),
                         ("output_blocks", 0, 64), ("output_blocks", 1, 64), ("output_blocks", 2, 32),
                         ("output_blocks", 3, 32)]:
        g = GatedSelfAttentionDense(dim, 64, 2, dim // 2)
        init_random_(g, seed=b)
        for k, v in g.state_dict().items():
            sd[f"model.diffusion_model.{part}.{b}.1.transformer_blocks.0.fuser.{k}"] = v
    pn = PositionNet(64, 64)
    init_random_(pn, seed=9)
    for k, v in pn.state_dict().items():
        sd[f"position_net.{k}"] = v
    with torch.inference_mode():
        gl = gligen_from_state_dict(sd)
        for m in gl.modules():           # gates open so the boxes change the image
            for nm in ("alpha_attn", "alpha_dense"):
                if hasattr(m, nm):
                    getattr(m, nm).fill_(0.5)
        gl.to(device=cuda, dtype=torch.bfloat16)
        gp = ModelPatcher(gl, load_device=cuda, offload_device=cuda)
        patcher, clip, vae = build_pipeline("tiny", device=cuda, dtype=torch.bfloat16, seed=2)
        pos = encode_prompt(clip, "a park", 64, 64)
        neg = encode_prompt(clip, "blurry", 64, 64)
        cond = NM["GLIGENTextBoxApply"]().append(pos, clip, gp, "a dog", 32, 32, 0, 0)[0]
        res = {}
        for mode in ("0", "1"):
            monkeypatch.setenv("CGS_RUN_GRAPHS", mode)
            before = dict(run_graph.stats)
            outs = []
            for seed in (5, 6, 5):
                latent = torch.zeros([2, 4, 8, 8])
                noise = S.prepare_noise(latent, seed)
                outs.append(S.sample(patcher, noise, 4, 5.0, "euler_ancestral", "normal", cond, neg, latent,
                                     seed=seed).float())
            res[mode] = outs
        torch.cuda.synchronize()
    assert run_graph.stats["capture"] - before["capture"] == 1, run_graph.stats
    assert run_graph.stats["replay_runs"] - before["replay_runs"] == 2, run_graph.stats
    for a, b in zip(res["0"], res["1"]):
        err = ((a - b).norm() / a.norm()).item()
        assert err < 1e-2, err


@pytest.mark.gpu
def test_run_graph_skips_empty_segments(cuda, monkeypatch):
    """A sampler whose last update runs before its last progress callback leaves an empty final segment:
    it is dropped at capture (no "CUDA Graph is empty" replay) and the run still equals the eager loop."""
    import warnings
    from comfy_gen_server_amd.sampling import run_graph
    from comfy_gen_server_amd.tools.synth import build_pipeline
    monkeypatch.setenv("CGS_GRAPHS", "1")
    with torch.inference_mode():
        patcher, clip, vae = build_pipeline("tiny", device=cuda, dtype=torch.bfloat16, seed=2)
        monkeypatch.setenv("CGS_RUN_GRAPHS", "0")
        (ref,) = _run_jobs(patcher, clip, vae, "dpmpp_2m_sde", [5])
        monkeypatch.setenv("CGS_RUN_GRAPHS", "1")
        e0 = run_graph.stats.get("empty_segments", 0)
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            _, got = _run_jobs(patcher, clip, vae, "dpmpp_2m_sde", [5, 5])
    assert not [x for x in w if "empty" in str(x.message).lower()], [str(x.message) for x in w]
    assert run_graph.stats.get("empty_segments", 0) > e0, run_graph.stats
    err = ((got - ref).norm() / ref.norm()).item()
    assert err < 1e-2, err
