"""Time every node-level HipBackend op of one training step by shape (GPU box).

    python tools/node_shapes.py [--graphs 16] [--blocks 8]
"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pfs-neural-net_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--graphs", type=int, default=16)
ap.add_argument("--blocks", type=int, default=8)
args = ap.parse_args()

import bench  # noqa: E402
import pfsgnn  # noqa: E402
from pfsgnn import native  # noqa: E402
from pfsgnn.train import loss_function  # noqa: E402

stats = collections.defaultdict(lambda: [0, 0.0])
OPS = ["lin", "lin_t", "wgrad", "bn_fwd", "bn_bwd", "graph_reduce", "graph_bcast_add", "rms2_fwd",
       "rms2_bwd", "bn2_finalize", "bn2_bwd_coef", "moment_coef", "zeros", "empty"]


def wrap(name, fn):
    def w(*a, **k):
        shape = tuple(tuple(x.shape) for x in a if isinstance(x, torch.Tensor))
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        r = fn(*a, **k)
        e.record()
        e.synchronize()
        st = stats[(name, shape)]
        st[0] += 1
        st[1] += s.elapsed_time(e)
        return r
    return w


be = native.HipBackend.__new__  # noqa
hb = pfsgnn.gnn.backend()
for op in OPS:
    if hasattr(hb, op):
        setattr(hb, op, wrap(op, getattr(hb, op)))
device = torch.device("cuda", 0)
pfsgnn.config.device = device
gnn = pfsgnn.GNN(B=args.blocks, Fdim=10, T=128, F_s=1, F_t=2).to(device)
gnn.train()
data, ci = bench.make_batch(args.graphs, 0, device)
for it in range(2):
    if it == 1:
        stats.clear()
    gnn.zero_grad()
    out = gnn(data)
    loss, _ = loss_function(out, ci, pclass=0.1, pfiber=0.1, sharpness=10.0, seed=it)
    loss.backward()
torch.cuda.synchronize()
tot = sum(v[1] for v in stats.values())
print(f"node ops total {tot:.3f} ms (event-bracketed, incl. launch)")
for (name, shape), (n, ms) in sorted(stats.items(), key=lambda kv: -kv[1][1])[:40]:
    print(f"{ms:8.3f} ms {n:4d}x {name:16s} {shape}")
