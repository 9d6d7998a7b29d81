"""Bitwise reproducibility of the general-graph (sliced) path at the bench
geometry: one GNN forward + backward (tools/sparse_bench.py's model, batch
and linear objective) repeated R times on the same parameters and inputs;
prints, per run, how many elements of the outputs and parameter gradients
differ from run 0.
    python tools/sparse_det.py [density] [R]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "pfs-neural-net_amd")):
    sys.path.insert(0, p)
import torch  # noqa: E402

import pfsgnn  # noqa: E402
from pfsgnn import config  # noqa: E402

DENS = float(sys.argv[1]) if len(sys.argv) > 1 else 0.3
R = int(sys.argv[2]) if len(sys.argv) > 2 else 3
G, NF, NC, B, F = 16, 2394, 128, 8, 10
config.device = torch.device("cuda")
gen = torch.Generator().manual_seed(0)
keep = torch.rand(G, NF, NC, generator=gen) < DENS
g, f, c = torch.nonzero(keep, as_tuple=True)
perm = torch.randperm(g.numel(), generator=gen)
ei = torch.stack([(g * NF + f)[perm], (g * NC + c)[perm]])
E = ei.shape[1]
xs = torch.arange(NF, dtype=torch.float).repeat(G).reshape(-1, 1)
xt = torch.cat([torch.randint(2, 13, (G * NC, 1), generator=gen).float(),
                torch.randint(1000, 100000, (G * NC, 1), generator=gen).float()], 1)
xe = 2.0 + 8.0 * torch.rand(E, F, generator=gen)
data = pfsgnn.BipartiteData(ei, xs, xt, xe, torch.zeros(G, F))
torch.manual_seed(0)
gnn = pfsgnn.GNN(B=B, Fdim=F, T=NC, F_s=1, F_t=2).cuda()
gnn.train()
w = [torch.randn(n, F, device="cuda") * 1e-3 for n in (G * NF, G * NC, E, G)]
state = {k: v.clone() for k, v in gnn.state_dict().items()}
runs = []
for r in range(R):
    gnn.load_state_dict(state)   # (BatchNorm running statistics back to the start)
    gnn.zero_grad()
    out = gnn(data)
    loss = ((out.x_s * w[0]).sum() + (out.x_t * w[1]).sum() + (out.x_e * w[2]).sum()
            + (out.x_u * w[3]).sum())
    loss.backward()
    runs.append([t.detach().clone() for t in (out.x_s, out.x_t, out.x_e, out.x_u)]
                + [p.grad.clone() for p in gnn.parameters()])
torch.cuda.synchronize()
names = ["x_s", "x_t", "x_e", "x_u"] + [n for n, _ in gnn.named_parameters()]
for r in range(1, R):
    bad = {n: int((a != b).sum()) for n, a, b in zip(names, runs[0], runs[r])}
    bad = {n: v for n, v in bad.items() if v}
    print(f"density {DENS} E={E} run {r}: {sum(bad.values())} elements differ from run 0"
          + (f" {bad}" if bad else ""), flush=True)
