import sys, os, torch
sys.path[:0] = ["/root/repo", "/root/repo/pfs-neural-net_amd", "/root/repo/tests"]
import pfsgnn
from harness import make_problem
from test_gpu_parity import oracle_step, ours_step
G, NF, NC, B, sharp = 3, 10, 7, 3, 0.0
model, graph = make_problem(G, NF, NC, B=B, seed=G + NF + NC)
m64, o64, l64 = oracle_step(model, graph, G, NF, NC, 777 + NC, sharp, torch.float64)
p64 = dict(m64.named_parameters())
for path in ("mfma32", "mfma32", "mfma", "valu", "mfma32"):
    pfsgnn.set_edge_path(path)
    gnn, out, loss = ours_step(model, graph, G, NF, NC, B, 777 + NC, sharp)
    g = dict(gnn.named_parameters())
    errs = {n: ((g[n].grad.double().cpu() - p64[n].grad).abs().max().item() / p64[n].grad.abs().max().item()) for n in ("encoder_t.0.bias", "encoder_t.0.weight", "encoder_s.0.weight")}
    print(path, f"loss {loss.item():.8f}", {k: f"{v:.2e}" for k, v in errs.items()}, flush=True)
