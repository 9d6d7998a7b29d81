"""Throughput of the general-graph path (pfsgnn.sparse) next to the fused
complete-graph path, on the bench geometry (GPU box).

The objective is a fixed random linear functional of the GNN outputs (x_s,
x_t, x_e, u) -- train.py's loss needs complete fiber-major graphs -- and the
step is zero_grad + GNN forward + objective + backward + FusedAdam, captured
as a HIP graph and replayed (as bench.py times the headline; SPARSE_GRAPH=0:
eager launches), synchronised around the timed steps; the median of
SPARSE_RUNS (default 5) timed runs is reported, with the spread.  The edge
kernels' eager per-step times (pfsgnn timing) follow each line.

    python tools/sparse_bench.py [G] [NF] [NC] [B] [steps]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "pfs-neural-net_amd")):
    sys.path.insert(0, p)
import torch  # noqa: E402

import pfsgnn  # noqa: E402
from pfsgnn import config  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 16
NF = int(sys.argv[2]) if len(sys.argv) > 2 else 2394
NC = int(sys.argv[3]) if len(sys.argv) > 3 else 128
B = int(sys.argv[4]) if len(sys.argv) > 4 else 8
STEPS = int(sys.argv[5]) if len(sys.argv) > 5 else 20
F = 10
config.device = torch.device("cuda")
gen = torch.Generator().manual_seed(0)


def edges(density):
    if density >= 1.0:
        e = torch.arange(G * NF * NC)
        return torch.stack([e // NC, (e // (NF * NC)) * NC + e % NC])
    keep = torch.rand(G, NF, NC, generator=gen) < density
    g, f, c = torch.nonzero(keep, as_tuple=True)
    p = torch.randperm(g.numel(), generator=gen)
    return torch.stack([(g * NF + f)[p], (g * NC + c)[p]])


def run(density, label):
    torch.manual_seed(0)
    ei = edges(density)
    E = ei.shape[1]
    xs = torch.arange(NF, dtype=torch.float).repeat(G).reshape(-1, 1)
    xt = torch.cat([torch.randint(2, 13, (G * NC, 1), generator=gen).float(),
                    torch.randint(1000, 100000, (G * NC, 1), generator=gen).float()], 1)
    xe = 2.0 + 8.0 * torch.rand(E, F, generator=gen)
    data = pfsgnn.BipartiteData(ei, xs, xt, xe, torch.zeros(G, F))
    gnn = pfsgnn.GNN(B=B, Fdim=F, T=NC, F_s=1, F_t=2).cuda()
    gnn.train()
    use_graph = os.environ.get("SPARSE_GRAPH", "1") != "0"
    opt = pfsgnn.FusedAdam(gnn.parameters(), lr=1e-4, capturable=use_graph)
    w = [torch.randn(n, F, device="cuda") * 1e-3 for n in (G * NF, G * NC, E, G)]

    def step():
        gnn.zero_grad()
        out = gnn(data)
        loss = ((out.x_s * w[0]).sum() + (out.x_t * w[1]).sum() + (out.x_e * w[2]).sum()
                + (out.x_u * w[3]).sum())
        loss.backward()
        opt.step()

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    from pfsgnn import native
    native.timing_enable("spin")
    native.timing_reset()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    native.timing_enable(False)
    kt = {k: round(native.timing_query(k)[0] / 3, 3) for k in native.KERNELS}
    kt = {k: v for k, v in kt.items() if v}
    run_step = step
    if use_graph:
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            step()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            step()
        run_step = g.replay
    # median of SPARSE_RUNS timed runs of STEPS steps (one short run swings on a
    # shared box)
    runs = []
    for _ in range(int(os.environ.get("SPARSE_RUNS", "5"))):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(STEPS):
            run_step()
        torch.cuda.synchronize()
        runs.append((time.perf_counter() - t) / STEPS * 1e3)
    runs.sort()
    ms = runs[len(runs) // 2]
    from pfsgnn import gnn as gmod
    pad = ""
    for e in gmod._LAYOUT_CACHE.d.values():
        if e[0]() is data.edge_index and e[3].sp is not None and e[3].sp.sl is not None:
            pad = f"  EP/E {e[3].sp.sl.EP / E:.3f}"
    print(f"{label:34s} E={E:9d}  {ms:8.2f} ms/step  {E / ms / 1e3:8.1f} M edges/s{pad}"
          f"  (runs {runs[0]:.2f}..{runs[-1]:.2f} ms; {'graph' if use_graph else 'eager'})",
          flush=True)
    print(f"{'':34s} edge kernels, ms per eager step: {kt}", flush=True)


dens = [float(x) for x in os.environ.get("SPARSE_DENSITIES", "1.0,0.999,0.3,0.05").split(",")]
for dd in dens:
    run(dd, "complete (fused edge kernels)" if dd >= 1.0 else
        f"{100 * dd:g}% dense (general, " +
        ("composed)" if os.environ.get("PFSGNN_SLICED") == "0" else "sliced)"))
