"""Where km_source_fwd_ft's run-to-run differences fall: source_fwd called R
times on the same inputs (op_det_probe.py's), the differing elements of mom /
hs mapped back to (moment, channel, graph, fiber) and histogrammed over the
kernel's structure (fiber lane j16, tile, block, moment, channel), with the
size of the differences.
    python tools/op_det_where.py [G] [NF] [NC] [path] [R]"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pfs-neural-net_amd")]
import torch  # noqa: E402

import pfsgnn  # noqa: E402
from pfsgnn.engine import Dims  # noqa: E402
from pfsgnn.native import HipBackend  # noqa: E402

G, NF, NC = (int(a) for a in (sys.argv[1:4] + ["16", "2394", "128"][len(sys.argv[1:4]):]))
path = sys.argv[4] if len(sys.argv) > 4 else "bf16x6"
R = int(sys.argv[5]) if len(sys.argv) > 5 else 6
F, C = 10, 20
hb = HipBackend()
d = Dims(G, NF, NC, F)
E, NS, NT = d.E, d.NS, d.NT
torch.manual_seed(1)
c = lambda *s, sc=1.0, off=0.0: (torch.randn(*s, device="cuda") * sc + off).contiguous()  # noqa: E731
y, sc_, sh_ = c(F, E), c(F, sc=0.3, off=1), c(F)
Qt, Ws1, Ws2, bs2 = c(2 * F, NT), c(2 * F, 2 * F, sc=0.3), c(2 * F, 2 * F, sc=0.3), c(2 * F)
pfsgnn.set_edge_path(path)
runs = []
for r in range(R):
    hs = torch.zeros(8 * F, NS, device="cuda")
    mom = hb.source_fwd(d, y, sc_, sh_, Qt, Ws1, Ws2, bs2, hs)
    runs.append(torch.stack([mom.reshape(4, C, NS), hs.reshape(4, C, NS)]).clone())
torch.cuda.synchronize()
TPG = (NF + 15) // 16
ntiles = G * TPG
per = (ntiles + 7) // 8
ref = runs[0]
fibers = collections.Counter()
for i in range(1, R):
    diff = runs[i] != ref
    idx = diff.nonzero()
    print(f"run {i}: {idx.shape[0]} elements differ", flush=True)
    if idx.shape[0] == 0:
        continue
    a, b = runs[i][diff].double(), ref[diff].double()
    rel = ((a - b).abs() / b.abs().clamp_min(1e-30))
    print(f"  |diff| max {float((a - b).abs().max()):.3e}, rel max {float(rel.max()):.3e}, rel median {float(rel.median()):.3e}")
    arr, k, o, n = (idx[:, j].cpu() for j in range(4))
    gg, f = n // NF, n % NF
    ft = f // 16
    tile = gg * TPG + ft
    bx = (tile % per) * 8 + tile // per   # tile = (bx & 7) * per + (bx >> 3)
    for name, v in [("array(0 mom,1 hs)", arr), ("moment", k), ("channel", o), ("j16", f % 16),
                    ("bx & 7 (XCD)", bx % 8)]:
        cnt = collections.Counter(v.tolist())
        print(f"  by {name}: {dict(sorted(cnt.items()))}")
    fib = collections.Counter(zip(gg.tolist(), f.tolist()))
    fibers.update(fib.keys())
    print(f"  fibers touched: {len(fib)}; elements per fiber: {sorted(collections.Counter(fib.values()).items())}")
    blocks = collections.Counter(zip(gg.tolist(), ft.tolist()))
    print(f"  tiles touched: {len(blocks)}; fibers per tile: "
          f"{sorted(collections.Counter(collections.Counter((g_, f_ // 16) for g_, f_ in fib).values()).items())}")
    print(f"  first fibers: {sorted(fib)[:12]}")
print(f"fibers touched in any run: {len(fibers)}; in more than one run: "
      f"{sum(1 for v in fibers.values() if v > 1)}")
