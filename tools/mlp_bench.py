"""Micro-benchmark of the fused node MLP ops (pfsgnn_mlp_fwd / _bwd) in
isolation: average µs per launch pair over R repetitions, HIP events.

    python tools/mlp_bench.py [N] [R]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "pfs-neural-net_amd")):
    sys.path.insert(0, p)
import torch  # noqa: E402
from pfsgnn.native import HipBackend  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 38304
R = int(sys.argv[2]) if len(sys.argv) > 2 else 20
hb = HipBackend()
F = 10
dev = "cuda"
g = torch.Generator(device="cpu").manual_seed(0)


def r(*s):
    return torch.randn(*s, generator=g).to(dev)


for name, blocks, H, bn in [("S node_mlp_2", [F, 8 * F, F], 10 * F, True),
                            ("T node_mlp_2", [F, 2 * F, F], 4 * F, True)]:
    K = sum(blocks)
    segs, col = [], 0
    for i, rows in enumerate(blocks):
        pg = i == len(blocks) - 1
        segs.append((r(rows, N // 2394 if pg else N).contiguous(), col, pg))
        col += rows
    if N % 2394:
        segs[-1] = (r(blocks[-1], N).contiguous(), segs[-1][1], False)
    W1, b1, W2, b2 = r(H, K), r(H), r(F, H), r(F)
    bnp = (r(F), r(F), torch.zeros(F, device=dev), torch.ones(F, device=dev), 0.1, 1e-5)
    dY = r(F, N)
    for save_z in (True, False):
        for _ in range(3):
            hb.mlp_fwd(segs, N, W1, b1, W2, b2, bn=bnp if bn else None, save_z=save_z)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(R):
            out = hb.mlp_fwd(segs, N, W1, b1, W2, b2, bn=bnp if bn else None, save_z=save_z)
        b.record()
        torch.cuda.synchronize()
        print(f"{name} fwd N={N} K={K} H={H} save_z={save_z}: {a.elapsed_time(b) / R * 1e3:.1f} us "
              f"(with BN apply)", flush=True)
    Y, Z, Yp, mu, var = out if out[1] is not None else hb.mlp_fwd(segs, N, W1, b1, W2, b2, bn=bnp)
    dg, db = torch.zeros(F, device=dev), torch.zeros(F, device=dev)
    outs = [(torch.zeros(rows, N, device=dev), rows, False) for rows in blocks]
    for want_dx in (True, False):
        o = outs if want_dx else []
        for _ in range(3):
            hb.mlp_bwd(dY, Z, W1, W2, K, bn=(Yp, mu, var, bnp[0], 1e-5, dg, db), outs=o)
        torch.cuda.synchronize()
        a.record()
        for _ in range(R):
            hb.mlp_bwd(dY, Z, W1, W2, K, bn=(Yp, mu, var, bnp[0], 1e-5, dg, db), outs=o)
        b.record()
        torch.cuda.synchronize()
        print(f"{name} bwd N={N} want_dx={want_dx}: {a.elapsed_time(b) / R * 1e3:.1f} us "
              f"(with BN sums)", flush=True)
