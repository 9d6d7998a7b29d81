"""Drive the two backward edge kernels (edge_mlp_bwd, source_bwd) at the bench
geometry, N times each, for sampling profilers (rocprofv3 --pc-sampling / PMC).
    python tools/pcs_driver.py [N] [path]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pfs-neural-net_amd")]
import torch  # noqa: E402

import pfsgnn  # noqa: E402
from pfsgnn.engine import Dims  # noqa: E402
from pfsgnn.native import HipBackend  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 50
pfsgnn.set_edge_path(sys.argv[2] if len(sys.argv) > 2 else "mfma")
G, NF, NC, F = 16, 2394, 128, 10
hb = HipBackend()
d = Dims(G, NF, NC, F)
gen = torch.Generator(device="cuda").manual_seed(3)
c = lambda *s, sc=1.0, off=0.0: (torch.randn(*s, device="cuda", generator=gen) * sc + off)  # noqa: E731
g_tot, y, xe = c(F, d.E), c(F, d.E), c(F, d.E, sc=2, off=3)
alpha, gam0, gam1, xsc, xsh = c(F), c(F), c(F), c(F, sc=0.3, off=1), c(F)
Ps, Pt, W1, W2 = c(4 * F, d.NS), c(4 * F, d.NT), c(4 * F, 4 * F, sc=0.3), c(F, 4 * F, sc=0.3)
Qt, Ws1, Ws2, bs2 = c(2 * F, d.NT), c(2 * F, 2 * F, sc=0.3), c(2 * F, 2 * F, sc=0.3), c(2 * F)
mean, coef = c(2 * F, d.NS), c(4, 2 * F, d.NS, sc=0.1)
Rs, Wt1, g_hsum, g_next = c(2 * F, d.NS), c(2 * F, 2 * F, sc=0.3), c(2 * F, d.NT), c(F, d.E)
mu1, inv1 = c(F), c(F).abs() + 0.5
for i in range(N):
    gh = [torch.zeros(4 * F, 4 * F, device="cuda"), torch.zeros(F, 4 * F, device="cuda"),
          torch.zeros(F, device="cuda")]
    hb.edge_mlp_bwd(d, g_tot, alpha, gam0, gam1, y, xe, xsc, xsh, Ps, Pt, W1, W2, *gh, want_gxe=True)
    gs = [torch.zeros(2 * F, 2 * F, device="cuda"), torch.zeros(2 * F, 2 * F, device="cuda"),
          torch.zeros(2 * F, device="cuda")]
    hb.source_bwd(d, y, xsc, xsh, Qt, Ws1, Ws2, bs2, mean, coef, (Rs, Wt1, g_hsum), g_next,
                  (mu1, inv1), *gs)
torch.cuda.synchronize()
print("done", N)
