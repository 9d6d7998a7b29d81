"""Per-launch cost of small kernels inside a captured HIP graph (GPU box).

Replays graphs of K back-to-back launches of one op and prints us/launch:
torch's own elementwise add, and several libpfsgnn entry points on the
bench's node-table shapes -- the floor every extra launch of the step pays.

    python tools/launch_floor.py [K]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "pfs-neural-net_amd")):
    sys.path.insert(0, p)
import torch  # noqa: E402
from pfsgnn.native import HipBackend  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 200
hb = HipBackend()
F, G, NF, NC = 10, 16, 2394, 128
NS, NT = G * NF, G * NC
r = lambda *s: torch.randn(*s, device="cuda")  # noqa: E731
x4k = torch.zeros(4096, device="cuda")
xs, xt = r(F, NS), r(F, NT)
W = r(4 * F, 4 * F)
g = r(F)
mu, var = r(F), torch.rand(F, device="cuda") + 0.5
dgam, dbet = torch.zeros(F, device="cuda"), torch.zeros(F, device="cuda")

ops = {
    "torch add_ 4096": lambda: x4k.add_(1.0),
    "bn2_bwd_coef C=10": lambda: hb.bn2_bwd_coef(g, g, mu, var, g, 1000, 1e-5, dgam, dbet),
    "graph_reduce 10x38304 (G=16)": lambda: hb.graph_reduce(xs, G),
    "graph_reduce 10x2048 (G=16)": lambda: hb.graph_reduce(xt, G),
    "lin 40x10 . 10x38304": lambda: hb.lin(W, 0, F, xs),
    "lin 40x10 . 10x2048": lambda: hb.lin(W, 0, F, xt),
    "affine_rows 10x38304": lambda: hb.affine_rows(xs, g, g),
}
for name, fn in ops.items():
    fn()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    with torch.cuda.graph(gr):
        for _ in range(K):
            fn()
    gr.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        gr.replay()
    b.record()
    b.synchronize()
    print(f"{name:32s} {a.elapsed_time(b) / 10 / K * 1e3:7.2f} us/launch (graph of {K})", flush=True)
