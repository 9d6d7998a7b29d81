"""Bitwise reproducibility of single forward edge ops (edge_mlp_fwd, source_fwd,
target_fwd) at a batch geometry: each op called R times on the same inputs.
    python tools/op_det_probe.py [G] [NF] [NC] [paths] [R]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pfs-neural-net_amd")]
import torch  # noqa: E402

import pfsgnn  # noqa: E402
from pfsgnn.engine import Dims  # noqa: E402
from pfsgnn.native import HipBackend  # noqa: E402

G, NF, NC = (int(a) for a in (sys.argv[1:4] + ["16", "2394", "128"][len(sys.argv[1:4]):]))
paths = (sys.argv[4] if len(sys.argv) > 4 else "bf16x3,bf16x6,mfma").split(",")
R = int(sys.argv[5]) if len(sys.argv) > 5 else 4
F = 10
hb = HipBackend()
d = Dims(G, NF, NC, F)
E, NS, NT = d.E, d.NS, d.NT
torch.manual_seed(1)
c = lambda *s, sc=1.0, off=0.0: (torch.randn(*s, device="cuda") * sc + off).contiguous()  # noqa: E731
xe, xsc, xsh = c(F, E, sc=2, off=3), c(F, sc=0.5, off=1), c(F)
Ps, Pt = c(4 * F, NS), c(4 * F, NT)
W1, W2, b2 = c(4 * F, 4 * F, sc=0.3), c(F, 4 * F, sc=0.3), c(F)
y, sc_, sh_ = c(F, E), c(F, sc=0.3, off=1), c(F)
Qt, Ws1, Ws2, bs2 = c(2 * F, NT), c(2 * F, 2 * F, sc=0.3), c(2 * F, 2 * F, sc=0.3), c(2 * F)
Rs, Wt1 = c(2 * F, NS), c(2 * F, 2 * F, sc=0.3)
for path in paths:
    pfsgnn.set_edge_path(path)
    outs = {"edge_mlp_fwd": [], "source_fwd": [], "target_fwd": []}
    for r in range(R):
        yh, mu, var = hb.edge_mlp_fwd(d, xe, xsc, xsh, Ps, Pt, W1, W2, b2)
        outs["edge_mlp_fwd"].append(torch.cat([yh.reshape(-1), mu, var]).clone())
        hs = torch.zeros(8 * F, NS, device="cuda")
        mom = hb.source_fwd(d, y, sc_, sh_, Qt, Ws1, Ws2, bs2, hs)
        outs["source_fwd"].append(torch.cat([mom.reshape(-1), hs.reshape(-1)]).clone())
        outs["target_fwd"].append(hb.target_fwd(d, y, sc_, sh_, Rs, Wt1).reshape(-1).clone())
    torch.cuda.synchronize()
    for k, v in outs.items():
        nd = [int((v[0] != v[i]).sum().item()) for i in range(1, R)]
        print(f"{path} {k}: elements differing from run 0: {nd} of {v[0].numel()}", flush=True)
