"""Diagnostic: normed=False training step of one 2394x16 graph (B=8) on the
GPU vs the fp64 oracle; prints which outputs / gradients are non-finite."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "pfs-neural-net_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import torch  # noqa: E402
from harness import make_problem  # noqa: E402
from test_gpu_parity import oracle_step, ours_step  # noqa: E402

for (G, NF, NC, B) in [(1, 70, 16, 3), (1, 2394, 16, 8), (2, 2394, 16, 8)]:
    model, graph = make_problem(G, NF, NC, B=B, seed=3, normed=False)
    m64, o64, l64 = oracle_step(model, graph, G, NF, NC, 9, 10.0, torch.float64)
    gnn, out, loss = ours_step(model, graph, G, NF, NC, B, 9, 10.0, normed=False)
    print(f"G={G} NF={NF} NC={NC} B={B}: loss ours {loss.item():.6g} oracle {l64.item():.6g}")
    for nm in ("x_e", "x_s", "x_t", "x_u"):
        a, b = getattr(out, nm).detach().double().cpu(), getattr(o64, nm).detach()
        print(f"  {nm}: finite {torch.isfinite(a).all().item()} / oracle {torch.isfinite(b).all().item()}"
              f" maxabs {b.abs().max().item():.3e} err {(a - b).abs().max().item():.3e}")
    p64 = dict(m64.named_parameters())
    for n, p in gnn.named_parameters():
        r = p64[n].grad if p64[n].grad is not None else torch.zeros_like(p64[n])
        g = p.grad.double().cpu()
        bad = (~torch.isfinite(g)).sum().item()
        rbad = (~torch.isfinite(r)).sum().item()
        err = (g - r).abs().max().item()
        sc = r.abs().max().item()
        if bad or rbad or err > 1e-3 * max(sc, 1e-6):
            print(f"  grad {n}: nonfinite ours {bad} oracle {rbad} err {err:.3e} scale {sc:.3e}")
