"""Bitwise reproducibility of the training step's gradients at a given batch
geometry: the same fwd + train.py loss + bwd run R times from one state; prints
which gradients differ between runs (first in parameter order) per edge path.
    python tools/det_probe.py [G] [NF] [NC] [B] [paths] [R]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pfs-neural-net_amd")]
import torch  # noqa: E402

import pfsgnn  # noqa: E402
from pfsgnn.train import loss_function  # noqa: E402

G, NF, NC, B = (int(a) for a in (sys.argv[1:5] + ["16", "2394", "128", "8"][len(sys.argv[1:5]):]))
paths = (sys.argv[5] if len(sys.argv) > 5 else "mfma,bf16x6").split(",")
R = int(sys.argv[6]) if len(sys.argv) > 6 else 3
F = 10
gen = torch.Generator().manual_seed(5)
ci = torch.cat([torch.randint(2, 13, (G * NC, 1), generator=gen).float(),
                torch.randint(1000, 100000, (G * NC, 1), generator=gen).float()], 1)
e = torch.arange(G * NF * NC)
data = pfsgnn.BipartiteData(torch.stack([e // NC, (e // (NF * NC)) * NC + e % NC]),
                            torch.arange(NF, dtype=torch.float).repeat(G).reshape(-1, 1), ci,
                            2.0 + 8.0 * torch.rand(G * NF * NC, F, generator=gen), torch.zeros(G, F))
ci = ci.cuda()
torch.manual_seed(0)
gnn = pfsgnn.GNN(B=B, Fdim=F, T=NC, F_s=1, F_t=2).cuda()
gnn.train()
state = {k: v.clone() for k, v in gnn.state_dict().items()}
for path in paths:
    pfsgnn.set_edge_path(path)
    runs = []
    for r in range(R):
        gnn.load_state_dict(state)
        gnn.zero_grad()
        out = gnn(data)
        loss, _ = loss_function(out, ci, pclass=0.1, pfiber=0.1, sharpness=10.0, seed=7)
        loss.backward()
        torch.cuda.synchronize()
        runs.append((loss.item(), {n: p.grad.detach().clone() for n, p in gnn.named_parameters()
                                   if p.grad is not None}, out.x_e.detach().clone()))
    for r in range(1, R):
        diff = [n for n in runs[0][1] if not torch.equal(runs[0][1][n], runs[r][1][n])]
        xe = torch.equal(runs[0][2], runs[r][2])
        print(f"{path} run {r} vs 0: loss {runs[0][0]!r} {runs[r][0]!r} x_e equal {xe}; "
              f"{len(diff)} grads differ; first {diff[:6]}", flush=True)
print("sync_faults", pfsgnn.native.sync_faults())
