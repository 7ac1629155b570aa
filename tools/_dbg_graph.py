import os, sys, torch
sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
from comfy_gen_server_amd.models.layers import init_random_fast_
from comfy_gen_server_amd.models.unet import UNetModel
from comfy_gen_server_amd.runtime.graphs import GraphedForward
from test_graphs_gpu import CFG, _inputs
from comfy_gen_server_amd import ops
cuda = torch.device("cuda", 0)
os.environ["CGS_GRAPHS"] = "1"
with torch.inference_mode():
    m = UNetModel(**CFG, dtype=torch.bfloat16, device=cuda)
    init_random_fast_(m, seed=3)
    runner = GraphedForward(m)
    x, t, ctx, y = _inputs(cuda)
    ref = m(x, t, context=ctx, y=y, transformer_options={}).float()
    outs = [runner(x, t, context=ctx, y=y, transformer_options={}).float() for _ in range(3)]
    torch.cuda.synchronize()
    print("ref nan", ref.isnan().any().item(), [o.isnan().any().item() for o in outs], [(o - ref).abs().max().item() for o in outs])
    x2, t2, ctx2, y2 = _inputs(cuda, seed=7)
    ref2 = m(x2, t2, context=ctx2, y=y2, transformer_options={}).float()
    ref2b = m(x2, t2, context=ctx2, y=y2, transformer_options={}).float()
    o2 = runner(x2, t2, context=ctx2, y=y2, transformer_options={}).float()
    o2b = runner(x2, t2, context=ctx2, y=y2, transformer_options={}).float()
    torch.cuda.synchronize()
    print("ref2 nan", ref2.isnan().any().item(), "ref2b nan", ref2b.isnan().any().item(), "o2 nan", o2.isnan().any().item(), "o2b nan", o2b.isnan().any().item())
    print("ref2 vs ref2b", (ref2 - ref2b).abs().max().item(), "o2 vs ref2", (o2 - ref2).abs().max().item(), "o2b vs ref2b", (o2b-ref2b).abs().max().item())
    print({k: v for k, v in ops.stats().items()})
